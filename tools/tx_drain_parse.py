#!/usr/bin/env python3
"""Per-dispatch PMC values of tools/tx_drain_probe.py runs, by scenario and
pass.  The probe's TX dispatches come in a fixed order: per scenario, per
call, the payload pass, the header pass, then the flush read if any (run
the probe with --no-check so no extra fills follow); this maps them back.

  python tools/tx_drain_parse.py --only grp:0:2:none,... --calls C --warmup W DIR [DIR...]
Prints one JSON line per scenario and pass: each counter's median per
dispatch over the measured calls (after the warmup)."""
import argparse
import csv
import glob
import json
import os
from collections import defaultdict


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--only", required=True)
    ap.add_argument("--calls", type=int, required=True)
    ap.add_argument("--warmup", type=int, required=True)
    ap.add_argument("dirs", nargs="+")
    args = ap.parse_args()
    per = defaultdict(dict)
    names = {}
    for d in args.dirs:
        for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
            for r in csv.DictReader(open(f)):
                k = r["Kernel_Name"]
                if not any(s in k for s in ("tcp_tx", "slot_floor")):
                    continue
                key = (d, int(r["Dispatch_Id"]))
                per[key][r["Counter_Name"]] = per[key].get(r["Counter_Name"], 0.0) + float(r["Counter_Value"])
                names[key] = k
    # one counter set per directory (one rocprofv3 pass each): merge by order
    by_dir = defaultdict(list)
    for (d, i) in sorted(per):
        by_dir[d].append((names[(d, i)], per[(d, i)]))
    seqs = list(by_dir.values())
    n = min(len(s) for s in seqs)
    merged = []
    for j in range(n):
        c = {}
        for s in seqs:
            c.update(s[j][1])
        merged.append((seqs[0][j][0], c))
    at = 0
    total = args.warmup + args.calls
    for sc in args.only.split(","):
        gap = sc.split(":")[3]
        step = 3 if gap == "flush" else 2
        rows = merged[at:at + total * step]
        at += total * step
        for pi, pname in enumerate(("payload", "header", "flush")[:step]):
            vals = defaultdict(list)
            for i in range(args.warmup, total):
                if i * step + pi >= len(rows):
                    break
                kname, c = rows[i * step + pi]
                for k, v in c.items():
                    vals[k].append(v)
            med = {k: sorted(v)[len(v) // 2] for k, v in vals.items()}
            print(json.dumps({"scenario": sc, "pass": pname, "kernel": rows[pi][0][:60] if rows else "",
                              "median_per_dispatch": med}))


if __name__ == "__main__":
    main()
