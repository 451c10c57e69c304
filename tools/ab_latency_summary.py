"""Medians of tools/ab_latency.sh's interleaved rounds (gpurun_out/ab_lat)."""
import glob
import json
import statistics
import sys

d = sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/ab_lat"
for v in ("prev", "cur"):
    runs = [json.load(open(f)) for f in sorted(glob.glob(f"{d}/{v}.*.json"))]
    if not runs:
        continue
    row = {k: [r[k]["gpu_med_us"] for r in runs] for k in ("checksum_1500B", "vv_batch_64KiB_45segs",
                                                           "chains_45_tcp_segments")}
    conc = {c["threads"]: [] for c in runs[0]["concurrent_vv_batch_64KiB"]}
    for r in runs:
        for c in r["concurrent_vv_batch_64KiB"]:
            conc[c["threads"]].append(c["calls_per_s"])
    wrong = sum(c["wrong"] for r in runs for c in r["concurrent_vv_batch_64KiB"])
    print(v, " ".join(f"{k} {row[k]}" for k in row), " ".join(f"{t}thr {conc[t]}" for t in conc))
    print("   medians:", " ".join(f"{k} {statistics.median(row[k]):.2f}" for k in row),
          "; ".join(f"{t} threads {statistics.median(conc[t]):.0f} calls/s" for t in conc), f"; wrong results {wrong}")
