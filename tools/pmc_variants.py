#!/usr/bin/env python3
"""Average per-dispatch counters of each kernel instance in a rocprofv3
--pmc output directory (e.g. a tools/tune.py run): which template instance
read how many bytes.  FETCH_SIZE is raw (KiB; see tools/pmc_parse.py for the
calibration to HBM bytes).

  python tools/pmc_variants.py OUTDIR
"""
import collections
import csv
import glob
import os
import sys

rows = []
for f in glob.glob(os.path.join(sys.argv[1], "**", "*counter_collection.csv"), recursive=True):
    rows += list(csv.DictReader(open(f)))
per = collections.defaultdict(lambda: collections.defaultdict(float))
for r in rows:
    per[(r["Kernel_Name"], int(r["Dispatch_Id"]))][r["Counter_Name"]] += float(r["Counter_Value"])
agg = collections.defaultdict(list)
for (k, _), c in per.items():
    if "nsk::" in k:
        agg[k].append(c)
for k, cs in sorted(agg.items()):
    names = sorted({n for c in cs for n in c})
    avg = {n: sum(c.get(n, 0.0) for c in cs) / len(cs) for n in names}
    print(f"{k[:100]}  dispatches {len(cs)}  " + "  ".join(f"{n} {v:.0f}" for n, v in avg.items()))
