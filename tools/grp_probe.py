#!/usr/bin/env python3
"""The receive ring's shape for descriptor tables (tbl_ring.hip) against
csum_hyb's big-packet instance (what ns_csum_batch_dev runs) on bench.py's cfg2 (1M x 1500 B, two rotating batches
with their tables), interleaved rounds of back-to-back launches, medians;
tools/grp_variants.hip (libns_grpv.so).  Variants 0 and 1 must agree on
every result.
  python tools/grp_probe.py [--rounds 5] [--reps 20]
"""
from __future__ import annotations

import argparse
import ctypes
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import torch  # noqa: E402

from netstack_amd import workloads as W  # noqa: E402

NAMES = {0: "tbl_ring", 1: "hyb", 2: "tbl_ring_no_desc", 3: "no_desc_1460_contig", 4: "no_desc_occ8"}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rounds", type=int, default=5)
    ap.add_argument("--reps", type=int, default=20)
    ap.add_argument("--only", default="")
    args = ap.parse_args()
    dev = torch.device("cuda", 0)
    stream = torch.cuda.current_stream(dev)
    lib = ctypes.CDLL(os.path.join(ROOT, "netstack_amd", "lib", "libns_grpv.so"))
    lib.grpv_launch.argtypes = [ctypes.c_int, ctypes.c_void_p, ctypes.c_uint64, ctypes.c_void_p, ctypes.c_uint32,
                                ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p]
    b = W.config(2)
    arenas = [b.arena_device(dev), W.random_bytes_torch(b.seed + 77, b.arena_bytes, dev)]
    desc = torch.from_numpy(b.desc.view(np.uint8).copy()).to(dev)
    descs = [desc, desc.clone()]
    out = torch.empty(b.n, dtype=torch.int16, device=dev)
    err = torch.zeros(1, dtype=torch.int64, device=dev)
    ks = [int(k) for k in args.only.split(",")] if args.only else sorted(NAMES)

    def launch(k, r):
        assert lib.grpv_launch(k, arenas[r].data_ptr(), b.arena_bytes, descs[r].data_ptr(), b.n, out.data_ptr(),
                               err.data_ptr(), stream.cuda_stream) == 0

    res = {}
    for k in ks:
        launch(k, 0)
        torch.cuda.synchronize()
        res[k] = out.clone()
    parity = bool(torch.equal(res[0], res[1])) if 0 in res and 1 in res else None
    times = {k: [] for k in ks}
    ev = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
    for _ in range(args.rounds):
        for k in ks:
            for j in range(3):
                launch(k, j % 2)
            ev[0].record(stream)
            for j in range(args.reps):
                launch(k, j % 2)
            ev[1].record(stream)
            torch.cuda.synchronize()
            times[k].append(ev[0].elapsed_time(ev[1]) * 1e3 / args.reps)
    algo = b.algorithmic_bytes
    print(json.dumps({"workload": "cfg2: 1M x 1500 B, 2 rotating batches", "algo_bytes": algo,
                      "tbl_ring_equals_hyb": parity, "err": int(err.item()),
                      "variants": {NAMES[k]: {"us": round(float(np.median(v)), 2), "min_us": round(min(v), 2),
                                              "frac": round(algo / float(np.median(v)) / 1e3 / 8000, 4),
                                              "rounds": [round(x, 2) for x in v]} for k, v in times.items()}},
                     indent=1))


if __name__ == "__main__":
    main()
