#!/usr/bin/env python3
"""Independent batches pipelined over several HIP streams: K launches of the
production kernel (ns_csum_batch_dev) over rotating batches, on 1 stream
(each launch waits for the previous one: the dependent-launch boundary and
the launch's ramp and tail are serial, as bench.py times it) and round-robin
over 2 or 4 streams (the next batch's ramp overlaps the previous one's tail).
Each stream writes its own results.  Reports wall time per batch between two
events that bracket all streams.  A caller-side measurement, not a bench
line: bench.py keeps one stream, so its per-launch roofline stays a kernel
duration.

  python tools/overlap_probe.py [--configs 3,4,2] [--reps 200] [--rounds 5]
"""
from __future__ import annotations

import argparse
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
    ap.add_argument("--configs", default="3,4,2")
    ap.add_argument("--reps", type=int, default=200)
    ap.add_argument("--rounds", type=int, default=5)
    ap.add_argument("--streams", default="1,2,4")
    args = ap.parse_args()
    dev = torch.device("cuda", 0)
    eng = Engine(0)
    main_s = torch.cuda.current_stream(dev)
    pool = [main_s] + [torch.cuda.Stream(dev) for _ in range(3)]
    for cfg in [int(c) for c in args.configs.split(",")]:
        rot = {2: 2, 3: 4, 4: 2}[cfg]
        b = W.config(cfg)
        arenas = [b.arena_device(dev)] + [W.random_bytes_torch(b.seed + 77 * r, b.arena_bytes, dev)
                                          for r in range(1, rot)]
        desc = torch.from_numpy(b.desc.view(np.uint8).copy()).to(dev)
        descs = [desc] + [desc.clone() for _ in range(1, rot)]
        outs = [torch.empty(b.n, dtype=torch.int16, device=dev) for _ in range(4)]
        ref = eng.batch_tensors(arenas[0], descs[0]).cpu()
        res = {}
        for _ in range(args.rounds):
            for ns in [int(x) for x in args.streams.split(",")]:
                ss = pool[:ns]
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                torch.cuda.synchronize()
                e0.record(main_s)
                for s in ss[1:]:
                    s.wait_event(e0)
                for k in range(args.reps):
                    j = k % ns
                    eng.batch_tensors(arenas[k % rot], descs[k % rot], outs[j], stream=ss[j])
                for s in ss[1:]:
                    main_s.wait_stream(s)
                e1.record(main_s)
                torch.cuda.synchronize()
                res.setdefault(ns, []).append(e0.elapsed_time(e1) * 1e3 / args.reps)
        # each stream's launch of batch 0 gives the same results as the plain call
        for j in range(4):
            eng.batch_tensors(arenas[0], descs[0], outs[j], stream=pool[j])
        torch.cuda.synchronize()
        ok = all(torch.equal(outs[j].cpu(), ref) for j in range(4))
        ab = b.algorithmic_bytes
        print(f"== cfg{cfg} {b.name}: {ab / 1e6:.1f} MB per batch, {rot} rotating batches, "
              f"per-stream results {'bit-exact' if ok else 'DIFFER'}", flush=True)
        for ns, v in res.items():
            med = float(np.median(v))
            print(f"  {ns} stream(s): {med:8.2f} us per batch (min {np.min(v):8.2f})  "
                  f"{ab / med / 1e3:7.0f} GB/s = {ab / med / 1e3 / 8000 * 100:5.1f}% of 8 TB/s", flush=True)
        del arenas, descs, outs
        torch.cuda.synchronize()
    eng.sync()


if __name__ == "__main__":
    main()
