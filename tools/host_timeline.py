#!/usr/bin/env python3
"""Timeline of ns_csum_batch_host's DMA pipeline from one rocprofv3 run with
--kernel-trace --memory-copy-trace (csv): for the last `--calls` calls, every
copy and kernel in start order (stream, start, duration, bytes), and per call
how much of its span each engine was busy and how long nothing ran.

  rocprofv3 --kernel-trace --memory-copy-trace --output-format csv -d D -o run \\
      -- python3 bench.py --mode host --config 3
  python3 tools/host_timeline.py D [--calls 3] [--chunks-per-call 8]
"""
from __future__ import annotations

import argparse
import csv
import glob
import json
import os


def rows(path):
    with open(path, newline="") as f:
        return list(csv.DictReader(f))


def col(r, *names):
    for n in names:
        if n in r and r[n] != "":
            return r[n]
    return None


def union(iv):
    """Total length of the union of intervals."""
    tot, cur_s, cur_e = 0, None, None
    for s, e in sorted(iv):
        if cur_e is None or s > cur_e:
            if cur_e is not None:
                tot += cur_e - cur_s
            cur_s, cur_e = s, e
        else:
            cur_e = max(cur_e, e)
    if cur_e is not None:
        tot += cur_e - cur_s
    return tot


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("dir")
    ap.add_argument("--calls", type=int, default=3)
    ap.add_argument("--chunks-per-call", type=int, default=8)
    args = ap.parse_args()
    kt = glob.glob(os.path.join(args.dir, "**", "*kernel_trace.csv"), recursive=True)
    mt = glob.glob(os.path.join(args.dir, "**", "*memory_copy_trace.csv"), recursive=True)
    ev = []
    for r in rows(kt[0]) if kt else []:
        name = col(r, "Kernel_Name") or ""
        if "nsk::" not in name:
            continue
        ev.append(dict(kind="K", what=name.split("(")[0].replace("void ", "")[:40], s=int(col(r, "Start_Timestamp")),
                       e=int(col(r, "End_Timestamp")), q=col(r, "Queue_Id", "Stream_Id"), bytes=0))
    for r in rows(mt[0]) if mt else []:
        d = col(r, "Direction", "Operation") or "?"
        ev.append(dict(kind="C", what=d, s=int(col(r, "Start_Timestamp")), e=int(col(r, "End_Timestamp")),
                       q=col(r, "Queue_Id", "Stream_Id", "Dst_Agent_Id"), bytes=int(col(r, "Bytes", "Size") or 0)))
    ev.sort(key=lambda x: x["s"])
    batches = [i for i, x in enumerate(ev) if x["kind"] == "K" and "csum_" in x["what"]]
    need = args.calls * args.chunks_per_call
    if len(batches) < need:
        print(json.dumps({"error": f"{len(batches)} batch kernels, need {need}"}))
        return
    first_k = batches[-need]
    # the call's first copy precedes its first kernel: start at the last H2D
    # copies before it
    i0 = first_k
    while i0 > 0 and ev[i0 - 1]["kind"] == "C":
        i0 -= 1
    sel = ev[i0:]
    t0 = sel[0]["s"]
    lines = []
    for x in sel:
        lines.append(f'{x["kind"]} {x["what"]:<40} q={x["q"]} +{(x["s"] - t0) / 1e3:9.1f} us '
                     f'{(x["e"] - x["s"]) / 1e3:8.1f} us {x["bytes"]:>10d} B')
    span = (max(x["e"] for x in sel) - t0) / 1e3
    copies = [(x["s"], x["e"]) for x in sel if x["kind"] == "C"]
    h2d = [(x["s"], x["e"]) for x in sel if x["kind"] == "C" and "D2H" not in x["what"].upper()
           and "DEVICE_TO_HOST" not in x["what"].upper()]
    kern = [(x["s"], x["e"]) for x in sel if x["kind"] == "K"]
    anyb = union(copies + kern) / 1e3
    cbytes = sum(x["bytes"] for x in sel if x["kind"] == "C")
    print("\n".join(lines))
    print(json.dumps({"calls": args.calls, "span_us": round(span, 1), "copy_busy_us": round(union(copies) / 1e3, 1),
                      "h2d_busy_us": round(union(h2d) / 1e3, 1), "kernel_busy_us": round(union(kern) / 1e3, 1),
                      "idle_us": round(span - anyb, 1), "copy_bytes": cbytes,
                      "copy_GBps_over_span": round(cbytes / span / 1e3, 2) if span else None}, indent=1))


if __name__ == "__main__":
    main()
