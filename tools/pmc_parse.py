#!/usr/bin/env python3
"""Summarise rocprofv3 counter CSVs written by tools/profile.sh.

Dispatches of calib_buf / csum_batch are matched in order to the LABEL lines
of tools/pmc_run.py (REPS each).  HBM bytes per launch follow
MI355X_MICROARCH.md §HBM: FETCH_SIZE (KiB) is calibrated against a read of a
known byte count in the same access shape (runs of 8 chunks for cfg2's
kernel's 16-lane nontemporal groups, runs of 4 for per-lane runs; cfg4 mixes
both, weighted by the payload share of each class) because gfx950
under-reports wide streaming reads; the raw values are kept beside the
corrected ones.

  python tools/pmc_parse.py OUTDIR LOGFILE > summary.json
"""
import csv
import glob
import json
import os
import re
import sys
from collections import defaultdict

REPS = 3


def load(outdir):
    rows = []
    for f in glob.glob(os.path.join(outdir, "**", "*counter_collection.csv"), recursive=True):
        rows += list(csv.DictReader(open(f)))
    return rows


def main():
    outdir, log = sys.argv[1], sys.argv[2]
    labels = []
    for line in open(log):
        if line.startswith("LABEL "):
            parts = line.split()
            labels.append((parts[1], dict(p.split("=") for p in parts[2:])))
    rows = load(outdir)
    # per dispatch: {counter: value}
    disp = defaultdict(dict)
    names = {}
    for r in rows:
        k = int(r["Dispatch_Id"])
        disp[k][r["Counter_Name"]] = disp[k].get(r["Counter_Name"], 0.0) + float(r["Counter_Value"])
        names[k] = r["Kernel_Name"]
    ours = [k for k in sorted(disp) if ("calib_" in names[k] or "nsk::" in names[k])]
    out = {}
    pos = 0
    for lab, meta in labels:
        kpl = int(meta.get("kernels", 1))  # dispatches per launch
        ks = ours[pos:pos + REPS * kpl]
        pos += REPS * kpl
        if len(ks) < REPS * kpl:
            break
        counters = sorted({c for k in ks for c in disp[k]})
        avg = {c: sum(disp[k].get(c, 0.0) for k in ks) / REPS for c in counters}  # per launch
        kern = " + ".join(dict.fromkeys(names[k][:80] for k in ks))
        out[lab] = {"kernel": kern, "meta": meta, "avg": avg}
    # FETCH_SIZE calibration per access shape
    cal = {}
    for m in ("calib800", "calib400", "calib102", "calib2164"):
        if m in out and "FETCH_SIZE" in out[m]["avg"]:
            cal[m] = float(out[m]["meta"]["bytes"]) / (out[m]["avg"]["FETCH_SIZE"] * 1024.0)
    for lab in list(out):
        if "algorithmic_bytes" not in out[lab]["meta"] or "FETCH_SIZE" not in out[lab]["avg"]:
            continue
        raw = out[lab]["avg"]["FETCH_SIZE"] * 1024.0
        # the quad-lane small-packet paths (cfg3 and its probes) load whole
        # lines nontemporally: the 16-lane-group shape (calib2164)
        big = float(out[lab]["meta"].get("big_share", 1.0)) if lab != "cfg3" else 1.0
        shape = {"calib2164": big, "calib400": 1.0 - big}
        if "shape" in out[lab]["meta"]:  # one named access shape
            shape = {out[lab]["meta"]["shape"]: 1.0}
        f = None
        if all(cal.get(m) for m, w in shape.items() if w > 0):
            f = sum(w * cal[m] for m, w in shape.items() if w > 0)
        out[lab]["hbm_read_bytes_raw"] = raw
        out[lab]["fetch_calibration"] = {"shape": shape, "factor": f}
        out[lab]["hbm_bytes_per_launch"] = raw * f if f else None
        if "WRITE_SIZE" in out[lab]["avg"]:
            out[lab]["hbm_write_bytes"] = out[lab]["avg"]["WRITE_SIZE"] * 1024.0
    json.dump(out, sys.stdout, indent=1)


if __name__ == "__main__":
    main()
