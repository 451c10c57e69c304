#!/usr/bin/env python3
"""Per-dispatch effective clock from a rocprofv3 --pmc GRBM_GUI_ACTIVE pass
with the kernel trace (tools/clock_probe.sh): clock = GRBM_GUI_ACTIVE / 8
(the counter is summed over the 8 XCDs) / duration (MI355X_MICROARCH.md,
DVFS give-back).  Durations come from the kernel trace of the same run,
matched by dispatch id.  Prints the per-kernel series in launch order and the
first / last deciles.
  python tools/clock_parse.py OUTDIR > clock.json
"""
import csv
import glob
import json
import os
import sys
from collections import defaultdict


def rows(d, pat):
    out = []
    for f in glob.glob(os.path.join(d, "**", pat), recursive=True):
        out += list(csv.DictReader(open(f)))
    return out


def main():
    d = sys.argv[1]
    cnt = defaultdict(dict)
    name = {}
    for r in rows(d, "*counter_collection.csv"):
        k = int(r["Dispatch_Id"])
        cnt[k][r["Counter_Name"]] = cnt[k].get(r["Counter_Name"], 0.0) + float(r["Counter_Value"])
        name[k] = r["Kernel_Name"]
    dur = {}
    for r in rows(d, "*kernel_trace.csv"):
        k = int(r["Dispatch_Id"])
        dur[k] = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) * 1e-9
        name.setdefault(k, r["Kernel_Name"])
    series = defaultdict(list)
    for k in sorted(cnt):
        if "nsk::" not in name[k] or k not in dur or dur[k] <= 0:
            continue
        g = cnt[k].get("GRBM_GUI_ACTIVE")
        series[name[k][:90]].append({"dispatch": k, "us": round(dur[k] * 1e6, 2),
                                     "ghz": round(g / 8 / dur[k] / 1e9, 3) if g else None})
    out = {}
    for kern, s in series.items():
        q = max(1, len(s) // 10)

        def med(xs):
            xs = sorted(x for x in xs if x is not None)
            return xs[len(xs) // 2] if xs else None

        out[kern] = {"launches": len(s),
                     "first_decile": {"us": med([x["us"] for x in s[:q]]), "ghz": med([x["ghz"] for x in s[:q]])},
                     "last_decile": {"us": med([x["us"] for x in s[-q:]]), "ghz": med([x["ghz"] for x in s[-q:]])},
                     "series": s}
    json.dump(out, sys.stdout, indent=1)
    print()


if __name__ == "__main__":
    main()
