#!/usr/bin/env python3
"""ns_csum_batch_dev (cfg2's 1M x 1500-B packets, 1504-B stride) with every
packet start shifted by s bytes: 0 (16-B aligned, the bench), 2 (NET_IP_ALIGN),
14 (an Ethernet header before the IP packet), 1 and 7 (odd: the other byte
phase).  Two rotating arenas, median of `--rounds` rounds of `--reps`
launches; fraction of 8 TB/s over cfg2's algorithmic bytes.  Timing only: the
results at every shift are the oracle's in tests/test_gpu_parity.py (odd and
unaligned starts); here each shift's results must not change between its
two launches over the same arena.

  python tools/align_probe.py [--shifts 0,2,14,1,7]
"""
from __future__ import annotations

import argparse
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import torch  # noqa: E402

from netstack_amd import Engine  # noqa: E402
from netstack_amd import workloads as W  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--shifts", default="0,2,14,1,7")
    ap.add_argument("--rounds", type=int, default=5)
    ap.add_argument("--reps", type=int, default=20)
    ap.add_argument("--n", type=int, default=1 << 20)
    args = ap.parse_args()
    n, L, stride = args.n, 1500, 1504
    dev = torch.device("cuda", 0)
    eng = Engine(0)
    stream = torch.cuda.current_stream(dev)
    arenas = [W.random_bytes_torch(21 + r, n * stride + 64, dev) for r in range(2)]
    init = (np.arange(n, dtype=np.uint64) * np.uint64(2654435761) % np.uint64(65536)).astype(np.uint16)
    algo = n * (L + 18)
    print(json.dumps({"start": True, "n": n}), flush=True)
    for sh in (int(x) for x in args.shifts.split(",")):
        d = np.zeros(n, dtype=W.DESC_DTYPE)
        d["off"] = np.arange(n, dtype=np.uint64) * np.uint64(stride) + np.uint64(sh)
        d["len"] = L
        d["initial"] = init
        desc = torch.from_numpy(d.view(np.uint8).copy()).to(dev)
        out = torch.empty(n, dtype=torch.int16, device=dev)
        eng.batch_tensors(arenas[0], desc, out, stream=stream)
        torch.cuda.synchronize()
        first = out.clone()
        times = []
        for _ in range(args.rounds):
            for i in range(2):
                eng.batch_tensors(arenas[i % 2], desc, out, stream=stream)
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record(stream)
            for i in range(args.reps):
                eng.batch_tensors(arenas[i % 2], desc, out, stream=stream)
            e1.record(stream)
            torch.cuda.synchronize()
            times.append(e0.elapsed_time(e1) * 1e3 / args.reps)
        eng.batch_tensors(arenas[0], desc, out, stream=stream)
        torch.cuda.synchronize()
        us = float(np.median(times))
        print(json.dumps({"shift": sh, "us": round(us, 2), "min_us": round(min(times), 2),
                          "frac_of_8TBs": round(algo / us / 1e3 / 8000, 4),
                          "repeatable": bool(torch.equal(out, first))}), flush=True)


if __name__ == "__main__":
    main()
