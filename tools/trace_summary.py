#!/usr/bin/env python3
"""Per-launch durations of the checksum kernel from a rocprofv3 kernel trace
of `bench.py` (tools/profile.sh), summarised the way bench.py times it: the
launches of the timed region are launches [W, W+K) of csum_hyb or csum_grp in dispatch
order (W warm-up launches before them, one parity launch after).

  python tools/trace_summary.py TRACE_DIR --warmup W --steps K > summary.json
"""
import argparse
import csv
import glob
import json
import os
import statistics


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("trace_dir")
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--steps", type=int, default=50)
    a = ap.parse_args()
    rows = []
    for f in glob.glob(os.path.join(a.trace_dir, "**", "*kernel_trace.csv"), recursive=True):
        rows += [r for r in csv.DictReader(open(f)) if "csum_hyb" in r["Kernel_Name"] or "csum_grp" in r["Kernel_Name"]]
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    dur = [(int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3 for r in rows]
    timed = dur[a.warmup:a.warmup + a.steps]
    span = (int(rows[a.warmup + a.steps - 1]["End_Timestamp"]) - int(rows[a.warmup]["Start_Timestamp"])) / 1e3
    out = {
        "kernel": rows[0]["Kernel_Name"] if rows else None,
        "calls": len(dur),
        "avg_us_all_calls": statistics.mean(dur) if dur else None,
        "timed_region": {"launches": len(timed), "avg_us": statistics.mean(timed),
                         "median_us": statistics.median(timed), "min_us": min(timed), "max_us": max(timed),
                         "first_start_to_last_end_us_per_launch": span / len(timed)},
        "first_call_us": dur[0] if dur else None,
    }
    json.dump(out, __import__("sys").stdout, indent=1)
    print()


if __name__ == "__main__":
    main()
