#!/usr/bin/env python3
"""Workload for --pmc passes comparing the device-resident RX check (chained,
no stores) with the TX fill (the same table plus two checksum stores per
packet): REPS launches each, in that order, then csum_hyb / fold_scan
counter values per dispatch are printed by `--parse DIR`.

  rocprofv3 --pmc WRITE_SIZE -d OUT -o run --output-format csv -- python3 tools/pmc_tx.py
  python3 tools/pmc_tx.py --parse OUT
"""
import csv
import glob
import os
import sys
from collections import defaultdict

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
REPS = 3


def run():
    import torch

    from netstack_amd import Engine
    from netstack_amd import workloads as W

    dev = torch.device("cuda", 0)
    eng = Engine(0)
    n = 1 << 20
    arena, d, _ = W.rx_batch(n, 7000, dev)
    desc = torch.from_numpy(d.view(np.uint8).copy()).to(dev)
    out = torch.empty(len(d), dtype=torch.int16, device=dev)
    for _ in range(REPS):
        eng.batch_tensors(arena, desc, out, chained=True)
    torch.cuda.synchronize()
    print("LABEL rx", flush=True)
    td = torch.from_numpy(W.tx_desc(n).view(np.uint8).copy()).to(dev)
    for _ in range(REPS):
        eng.batch_tensors(arena, td, out, chained=True, store=True)
    torch.cuda.synchronize()
    print("LABEL tx", flush=True)


def parse(outdir):
    per = defaultdict(lambda: defaultdict(float))
    names = {}
    for f in glob.glob(os.path.join(outdir, "**", "*counter_collection.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            if "nsk::" not in r["Kernel_Name"]:
                continue
            k = int(r["Dispatch_Id"])
            per[k][r["Counter_Name"]] += float(r["Counter_Value"])
            names[k] = "fold_scan" if "fold_scan" in r["Kernel_Name"] else "csum_hyb"
    for k in sorted(per):
        print(k, names[k], dict(per[k]))


if __name__ == "__main__":
    if len(sys.argv) > 2 and sys.argv[1] == "--parse":
        parse(sys.argv[2])
    else:
        run()
