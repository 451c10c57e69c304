"""Merge several runs of tools/crossover.cc (same build, same box pool) into
one: per shape and point the median engine time and the median one-core
time over the runs, their ratio, and the crossover by the tool's own rule
(the smallest size from which the engine is faster at every larger size).
Single runs move by a few percent, enough to shift a crossover that sits
near 1.0 by one step; the gates in go/header/checksum_batch_hip.go are
checked against the merged file.
  python tools/crossover_merge.py OUT.json RUN.json [RUN.json ...]
      [--only SHAPE=RUN.json,RUN.json ...]
--only takes a shape from the listed runs alone (a shape whose code changed
between the runs: only the runs of the current build count).  Runs that
lack a shape are skipped for it."""

import json
import statistics
import sys


def merge(all_runs, only=None):
    out = {}
    shapes = []
    for r in all_runs:
        shapes += [k for k in r if k not in shapes]
    for shape in shapes:
        runs = [all_runs[i] for i in (only or {}).get(shape, range(len(all_runs))) if shape in all_runs[i]]
        unit = runs[0][shape]["unit"]
        pts = []
        for i, p in enumerate(runs[0][shape]["points"]):
            g = statistics.median(r[shape]["points"][i]["gpu_med_us"] for r in runs)
            c = statistics.median(r[shape]["points"][i]["cpu_1core_med_us"] for r in runs)
            pts.append({unit: p[unit], "bytes": p["bytes"], "gpu_med_us": round(g, 2), "cpu_1core_med_us": round(c, 2),
                        "gpu_over_cpu": round(g / c, 3),
                        "runs_gpu_over_cpu": [round(r[shape]["points"][i]["gpu_over_cpu"], 3) for r in runs]})
        x = None
        for p in reversed(pts):
            if p["gpu_over_cpu"] >= 1:
                break
            x = p
        out[shape] = {"unit": unit, "points": pts,
                      "crossover": {unit: x[unit], "bytes": x["bytes"]} if x else None,
                      "runs_crossover": [r[shape]["crossover"] for r in runs]}
    return out


if __name__ == "__main__":
    args = sys.argv[2:]
    only_args = args[args.index("--only") + 1:] if "--only" in args else []
    files = args[:args.index("--only")] if "--only" in args else args
    runs = [json.load(open(f)) for f in files]
    only = {}
    for spec in only_args:
        shape, fl = spec.split("=", 1)
        only[shape] = [files.index(f) for f in fl.split(",")]
    m = merge(runs, only)
    m["_merged_from"] = {"runs": files, "only": {k: [files[i] for i in v] for k, v in only.items()}}
    with open(sys.argv[1], "w") as f:
        json.dump(m, f, indent=1)
        f.write("\n")
    for k, v in m.items():
        if not k.startswith("_"):
            print(k, v["crossover"], v["runs_crossover"])
