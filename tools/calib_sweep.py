#!/usr/bin/env python3
"""Read-ceiling sweep for the cfg2 roofline (not product code).

Times the product checksum kernel and pure-read calibration kernels of
libns_tune.so (nsk::calib_tile_x) over the SAME rotated cfg2 arenas, in
interleaved rounds, back-to-back launches timed by one event pair (the
bench's method).  Knobs: lane shape (8 x 16 nt loads, 8 x 8, 16 x 8), run
length in lines, a prologue of s_sleep rounds, dynamic LDS per workgroup
(caps residency), and edge lines loaded with the default policy.

  python tools/calib_sweep.py [--rounds 2] [--rotate 2] [--json out.json]
"""
from __future__ import annotations

import argparse
import ctypes
import itertools
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import torch  # noqa: E402

from netstack_amd import Engine  # noqa: E402
from netstack_amd import workloads as W  # noqa: E402

import bench  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rounds", type=int, default=2)
    ap.add_argument("--rotate", type=int, default=2)
    ap.add_argument("--reps", type=int, default=20)
    ap.add_argument("--json", default="")
    args = ap.parse_args()
    L = ctypes.CDLL(os.path.join(ROOT, "netstack_amd", "lib", "libns_tune.so"))
    L.nsk_calib_tile_x_launch.restype = ctypes.c_int
    L.nsk_calib_tile_x_launch.argtypes = [ctypes.c_int, ctypes.c_void_p, ctypes.c_uint64, ctypes.c_uint32,
                                          ctypes.c_uint32, ctypes.c_uint32, ctypes.c_void_p,
                                          ctypes.POINTER(ctypes.c_uint64), ctypes.c_void_p]
    dev = torch.device("cuda", 0)
    eng = Engine(0)
    arenas, descs = [], []
    for r in range(args.rotate):
        b = W.config(2)
        b.seed += 100 * r
        arenas.append(b.arena_device(dev))
        descs.append(torch.from_numpy(b.desc.view(np.uint8).copy()).to(dev))
    algo = W.config(2).algorithmic_bytes
    out = torch.empty(1 << 20, dtype=torch.int16, device=dev)
    outb = torch.zeros(16384, dtype=torch.int32, device=dev)
    stream = torch.cuda.current_stream(dev)
    R = args.rotate

    variants = [("product", None)]
    for mode, lpr, sleep, lds in itertools.product((0, 1, 2, 3), (8, 11, 16), (0, 4, 16), (1024, 9600, 20480)):
        if (mode == 2) != (lpr == 8):
            continue
        variants.append((f"m{mode}_lpr{lpr}_s{sleep}_lds{lds}", (mode, lpr, sleep, lds)))
    res = {name: [] for name, _ in variants}
    for rnd in range(args.rounds):
        for name, cfg in variants:
            if cfg is None:
                us = bench.b2b_us(lambda k: eng.batch_tensors(arenas[k % R], descs[k % R], out, stream=stream),
                                  stream, reps=args.reps)
                res[name].append(algo / us / 1e3)
                continue
            mode, lpr, sleep, lds = cfg
            rb = ctypes.c_uint64(0)

            def launch(k, mode=mode, lpr=lpr, sleep=sleep, lds=lds, rb=rb):
                a = arenas[k % R]
                rc = L.nsk_calib_tile_x_launch(mode, a.data_ptr(), a.numel(), lpr, sleep, lds, outb.data_ptr(),
                                               ctypes.byref(rb), stream.cuda_stream)
                assert rc == 0, rc

            us = bench.b2b_us(launch, stream, reps=args.reps)
            res[name].append(rb.value / us / 1e3)
        print(f"round {rnd} done", file=sys.stderr, flush=True)
    summary = {k: {"GBps_max": max(v), "GBps_min": min(v)} for k, v in res.items()}
    ranked = sorted(summary.items(), key=lambda kv: -kv[1]["GBps_max"])
    for k, v in ranked[:25]:
        print(f"{k:32s} {v['GBps_max']:8.1f} {v['GBps_min']:8.1f}")
    print(f"{'product':32s} {summary['product']['GBps_max']:8.1f} {summary['product']['GBps_min']:8.1f}")
    if args.json:
        json.dump({"rotate": R, "reps": args.reps, "rounds": args.rounds, "GBps": res}, open(args.json, "w"), indent=1)
    eng.close()


if __name__ == "__main__":
    main()
