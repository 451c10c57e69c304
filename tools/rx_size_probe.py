#!/usr/bin/env python3
"""ns_csum_rx_ring across frame sizes: rings of IPv4/TCP (and IPv6/TCP)
frames from 64 B to 9000-B jumbo frames, about 1.5 GB of frames per ring
(n = 1.5 GB / frame, at most 16M slots), two rotating rings, every 1000th
frame corrupted.  Median of `--rounds` rounds of `--reps` launches; the
fraction of 8 TB/s over the algorithmic bytes (frame + 4-B length + 1-B
verdict + 4-B sums per slot); the verdicts must be the generated ones.

  python tools/rx_size_probe.py [--frames 64,256,576,1500,4000,9000] [--v6]
                                 [--variants 40,41]
--variants also times tools/rx_ring_variants.hip's shapes (libns_rxv.so) on
each ring; their verdicts and sums must equal the product's.
"""
from __future__ import annotations

import argparse
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import ctypes  # noqa: E402

import torch  # noqa: E402

from netstack_amd import Engine  # noqa: E402
from netstack_amd import workloads as W  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--frames", default="64,256,576,1500,4000,9000")
    ap.add_argument("--v6", action="store_true")
    ap.add_argument("--eth", action="store_true", help="frames behind a 14-B Ethernet header (link_hdr 14)")
    ap.add_argument("--rounds", type=int, default=5)
    ap.add_argument("--reps", type=int, default=10)
    ap.add_argument("--bytes", type=float, default=1.5e9)
    ap.add_argument("--variants", default="")
    args = ap.parse_args()
    dev = torch.device("cuda", 0)
    eng = Engine(0)
    stream = torch.cuda.current_stream(dev)
    ks = [int(x) for x in args.variants.split(",") if x]
    if ks:
        sys.path.insert(0, os.path.join(ROOT, "tools"))
        from rx_ring_probe import RxGeo
        lib = ctypes.CDLL(os.path.join(ROOT, "netstack_amd", "lib", "libns_rxv.so"))
        lib.rxv_launch.argtypes = [ctypes.POINTER(RxGeo), ctypes.c_void_p, ctypes.c_int]
        lib.rxv_launch.restype = ctypes.c_int
    print(json.dumps({"start": True, "v6": args.v6}), flush=True)
    for fr in (int(x) for x in args.frames.split(",")):
        n = min(16 << 20, int(args.bytes // fr))
        rings = [W.rx_ring_batch_sized(n, fr, 9 + r, dev, v6=args.v6, corrupt_every=1000, eth=args.eth)
                 for r in range(2)]
        arena0, lens, bad, stride = rings[0]
        ring = dict(stride=stride, n=n, link_hdr=14 if args.eth else 0)
        v, _ = eng.rx_ring(arena0, ring, lens)
        torch.cuda.synchronize()
        want = torch.ones(n, dtype=torch.uint8, device=dev)
        want[torch.from_numpy(bad).to(dev)] = 0
        ok = bool(torch.equal(v[:n], want))
        v, s0 = eng.rx_ring(arena0, ring, lens)
        torch.cuda.synchronize()
        v, s0 = v[:n].clone(), s0[:2 * n].clone()
        err = torch.zeros(1, dtype=torch.int64, device=dev)
        verdict = torch.empty(n, dtype=torch.uint8, device=dev)
        sums = torch.empty(2 * n, dtype=torch.int16, device=dev)
        geos = [RxGeo(r[0].data_ptr(), stride, lens.data_ptr(), sums.data_ptr(), verdict.data_ptr(), err.data_ptr(),
                      n, 0, 14 if args.eth else 0, 0, None, 0) for r in rings] if ks else []

        def launcher(k):
            if k < 0:
                return lambda i: eng.rx_ring(rings[i % 2][0], ring, lens, stream=stream)
            return lambda i: lib.rxv_launch(ctypes.byref(geos[i % 2]), stream.cuda_stream, k)

        out = {}
        for k in [-1] + ks:
            f = launcher(k)
            same = None
            if k >= 0:
                verdict.fill_(0xEE)
                f(0)
                torch.cuda.synchronize()
                same = bool(torch.equal(verdict, v) and torch.equal(sums, s0))
            times = []
            for _ in range(args.rounds):
                for i in range(2):
                    f(i)
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record(stream)
                for i in range(args.reps):
                    f(i)
                e1.record(stream)
                torch.cuda.synchronize()
                times.append(e0.elapsed_time(e1) * 1e3 / args.reps)
            us = float(np.median(times))
            algo = n * (fr + (14 if args.eth else 0) + 9)
            out["product" if k < 0 else f"variant_{k}"] = {"us": round(us, 2),
                                                           "frac_of_8TBs": round(algo / us / 1e3 / 8000, 4),
                                                           "same_as_product": same}
        print(json.dumps({"frame": fr, "ipv6": args.v6, "ethernet": args.eth, "slots": n, "stride": stride,
                          "verdicts_as_generated": ok, "shapes": out}), flush=True)
        del rings, arena0, lens, v, want, s0, verdict, sums
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
