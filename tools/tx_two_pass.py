#!/usr/bin/env python3
"""TX fill (bench.py --config 8: 1M packets, the fused IPv4 + TCP table)
with its 2M stores in the main kernel (the product) against a read-only
launch followed by a pass that only stores (libns_tune.so store_pass, the
descriptors re-read, results from `out`).  Also the read-only launch and the
store pass alone.  The two-pass fill is checked against rx_batch's arena.

  python tools/tx_two_pass.py [--rounds 5] [--reps 20]
"""
from __future__ import annotations

import argparse
import ctypes
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
    ap.add_argument("--rounds", type=int, default=5)
    ap.add_argument("--reps", type=int, default=20)
    args = ap.parse_args()
    L = ctypes.CDLL(os.path.join(ROOT, "netstack_amd", "lib", "libns_tune.so"))
    L.nsk_store_pass_launch.argtypes = [ctypes.c_void_p, ctypes.c_uint64, ctypes.c_void_p, ctypes.c_uint32,
                                        ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p]
    dev = torch.device("cuda", 0)
    stream = torch.cuda.current_stream(dev)
    sp = stream.cuda_stream
    eng = Engine(0)
    n = 1 << 20
    arena, d = W.tx_batch(n, 7000, dev, fused=True)
    desc = torch.from_numpy(d.view(np.uint8).copy()).to(dev)
    out = torch.empty(len(d), dtype=torch.int16, device=dev)
    err = torch.zeros(1, dtype=torch.int64, device=dev)

    def store_pass():
        assert L.nsk_store_pass_launch(arena.data_ptr(), arena.numel(), desc.data_ptr(), len(d), out.data_ptr(),
                                       err.data_ptr(), sp) == 0

    variants = {
        "tx_product": lambda: eng.batch_tensors(arena, desc, out, store=True),
        "read_only": lambda: eng.batch_tensors(arena, desc, out, store=False),
        "read_then_store_pass": lambda: (eng.batch_tensors(arena, desc, out, store=False), store_pass()),
        "store_pass_only": store_pass,
    }
    # correctness of the two-pass fill
    p = arena.view(n, W.RX_STRIDE)
    p[:, 10:12] = 0
    p[:, 36:38] = 0
    variants["read_then_store_pass"]()
    torch.cuda.synchronize()
    rx, _, _ = W.rx_batch(n, 7000, dev)
    assert torch.equal(arena, rx), "two-pass fill differs from rx_batch"
    assert int(err.item()) == 0
    del rx
    print("two-pass fill == rx_batch arena", flush=True)
    res = {k: [] for k in variants}
    for _ in range(args.rounds):
        for name, fn in variants.items():
            for _ in range(3):
                fn()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record(stream)
            for _ in range(args.reps):
                fn()
            e1.record(stream)
            torch.cuda.synchronize()
            res[name].append(e0.elapsed_time(e1) * 1e3 / args.reps)
    algo = n * W.RX_PKT + 8 * n + len(d) * 18 + 4 * n  # bench.py packet_mode, TX
    for name, ts in res.items():
        med = float(np.median(ts))
        print(f"{name:22s} {med:7.1f} us  ({algo / med / 1e3 / 8000 * 100:5.1f}% of 8 TB/s at TX bytes)  "
              f"rounds {['%.1f' % x for x in ts]}", flush=True)


if __name__ == "__main__":
    main()
