#!/usr/bin/env python3
"""The receive-ring kernel's timing variants (tools/rx_ring_variants.hip,
libns_rxv.so) against the product (ns_csum_rx_ring) on bench.py's
`--config 7 --rx-layout ring` workload: 1M x 1500-B IPv4/TCP packets in
1504-B slots.  Rounds of back-to-back launches per variant, interleaved;
median microseconds per launch and the fraction of 8 TB/s over the
algorithmic bytes (packet bytes + 4-B length + 1-B verdict + 4-B sums per
slot).  Every variant's verdicts and sums must equal the product's.
  python tools/rx_ring_probe.py [--rounds 5] [--reps 20] [--only 0,1,2]
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

from netstack_amd import Engine  # noqa: E402
from netstack_amd import workloads as W  # noqa: E402

NAMES = {0: "product", 1: "all_default", 2: "all_nt", 3: "wg2", 4: "wg8", 5: "wg1", 6: "nb16", 7: "nb8",
         8: "occ6", 9: "nb12", 10: "checked_f0", 11: "f1_nb8", 12: "spec_line0", 13: "spec_lines01",
         14: "rotated_lines", 20: "bufs_product", 21: "bufs_nt_sc1", 22: "bufs_all_default", 23: "bufs_sc1",
         24: "bufs_lastline_default", 25: "bufs_lastline_default_nt_sc1", 26: "bufs_ll_sc0_nt",
         27: "bufs_ll_sc0_sc1", 28: "bufs_ll_sc0_nt_sc1", 29: "bufs_ll_sc0",
         30: "bufs_sorted", 50: "read_floor", 31: "bufs_sorted_outputs_in_sorted_order", 32: "bufs_sorted_index_early",
         33: "sort_only", 34: "count_only"}


class RxGeo(ctypes.Structure):
    _fields_ = [("ring", ctypes.c_uint64), ("stride", ctypes.c_uint64), ("len", ctypes.c_void_p),
                ("sums", ctypes.c_void_p), ("verdict", ctypes.c_void_p), ("err", ctypes.c_void_p),
                ("n", ctypes.c_uint32), ("frame_at", ctypes.c_uint32), ("link", ctypes.c_uint32),
                ("view0", ctypes.c_uint32), ("off", ctypes.c_void_p), ("limit", ctypes.c_uint64),
                ("bk_tup", ctypes.c_void_p), ("bk_total", ctypes.c_void_p), ("bk_wgoff", ctypes.c_void_p),
                ("bk_shift", ctypes.c_uint32), ("bk_nb", ctypes.c_uint32)]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rounds", type=int, default=5)
    ap.add_argument("--reps", type=int, default=20)
    ap.add_argument("--n", type=int, default=1 << 20)
    ap.add_argument("--only", default="")
    ap.add_argument("--prev", default="",
                    help="a variants library built from an earlier rx_ring.hip: its product shape is timed "
                         "beside the others as 'prev' (an A/B on one box)")
    ap.add_argument("--rotate", type=int, default=1, help="alternate two rings (1) or re-read one (0)")
    ap.add_argument("--stride", type=int, default=0, help="slot spacing (a multiple of 16 >= 1504; 0: 1504)")
    ap.add_argument("--bufs", default="", choices=("", "shuffled", "ring"),
                    help="the frames as a buffer list (ns_csum_rx_bufs) in shuffled or ring order; variants "
                         "20-23 then (the ring variants need no list)")
    ap.add_argument("--ipv6", action="store_true", help="IPv6/TCP frames instead of IPv4/TCP")
    ap.add_argument("--bk-shift", type=int, default=0,
                    help="variant 30: bucket size 2^shift bytes (0: the arena over at most 128 buckets)")
    ap.add_argument("--trend", type=int, default=0,
                    help="then time this many back-to-back launches of the product one by one (run-long drift)")
    args = ap.parse_args()
    n = args.n
    dev = torch.device("cuda", 0)
    stream = torch.cuda.current_stream(dev)
    eng = Engine(0)
    lib = ctypes.CDLL(os.path.join(ROOT, "netstack_amd", "lib", "libns_rxv.so"))
    lib.rxv_launch.argtypes = [ctypes.POINTER(RxGeo), ctypes.c_void_p, ctypes.c_int]
    lib.rxv_launch.restype = ctypes.c_int
    stride = args.stride or W.RX_STRIDE

    def spread(a):  # the same slots at a wider spacing
        if stride == W.RX_STRIDE:
            return a
        b = torch.zeros(n, stride, dtype=torch.uint8, device=dev)
        b[:, :W.RX_STRIDE] = a.view(n, W.RX_STRIDE)
        return b.view(-1)

    make = W.rx_ring_batch_v6 if args.ipv6 else W.rx_ring_batch
    arena, lens, bad = make(n, 9, dev, corrupt_every=1000)
    arena = spread(arena)
    ring = dict(stride=stride, n=n)
    offs = None
    if args.bufs:  # packet k is the frame in slot perm[k] (bench.py --rx-layout bufs)
        perm = np.random.default_rng(9).permutation(n) if args.bufs == "shuffled" else np.arange(n)
        offs = torch.from_numpy((perm.astype(np.int64) * stride).astype(np.int32)).to(dev)
        lens = lens[torch.from_numpy(perm).to(dev)].contiguous()
        v0, s0 = eng.rx_bufs(arena, ring, offs, lens)
    else:
        v0, s0 = eng.rx_ring(arena, ring, lens)
    torch.cuda.synchronize()
    err = torch.zeros(1, dtype=torch.int64, device=dev)
    verdict = torch.empty(n, dtype=torch.uint8, device=dev)
    sums = torch.empty(2 * n, dtype=torch.int16, device=dev)
    # two rings of the same frames, alternating (3.2 GB > the MALL), as
    # bench.py runs it
    # the product's verdicts: VALID but for the corrupted packets (INVALID)
    want = torch.ones(n, dtype=torch.uint8, device=dev)
    want[torch.from_numpy(bad).to(dev)] = 0
    if args.bufs:
        want = want[torch.from_numpy(perm).to(dev)]
    product_ok = bool(torch.equal(v0, want))
    arena2 = spread(make(n, 9, dev, corrupt_every=1000)[0]) if args.rotate else arena
    limit = arena.numel()
    shift = args.bk_shift or max(12, (limit - 1).bit_length() - 7)
    nb = (limit + (1 << shift) - 1) >> shift
    assert nb <= 128, nb
    tup = torch.empty(n * 4, dtype=torch.int32, device=dev)
    total = torch.zeros(128, dtype=torch.int32, device=dev)
    wgoff = torch.empty(((n + 4095) // 4096) * nb, dtype=torch.int32, device=dev)
    gs = [RxGeo(a.data_ptr(), stride, lens.data_ptr(), sums.data_ptr(), verdict.data_ptr(), err.data_ptr(),
                n, 0, 0, 0, offs.data_ptr() if offs is not None else None, a.numel() if offs is not None else 0,
                tup.data_ptr(), total.data_ptr(), wgoff.data_ptr(), shift, nb)
          for a in (arena, arena2)]
    g = gs[0]
    algo = n * (W.RX_PKT + 9)
    ks = [int(k) for k in args.only.split(",")] if args.only else \
        sorted(k for k in NAMES if (k >= 20) == bool(args.bufs))
    libs = {k: lib for k in ks}
    names = dict(NAMES)
    if args.prev:
        plib = ctypes.CDLL(os.path.abspath(args.prev))
        plib.rxv_launch.argtypes = lib.rxv_launch.argtypes
        plib.rxv_launch.restype = ctypes.c_int
        ks.append(-1)
        libs[-1] = plib
        names[-1] = "prev"
    res = {k: [] for k in ks}
    ok = {}
    for k in ks:  # parity first
        verdict.fill_(0xEE)
        sums.fill_(0x1234)
        assert libs[k].rxv_launch(ctypes.byref(g), stream.cuda_stream, max(k, 0)) == 0
        torch.cuda.synchronize()
        ok[k] = bool(torch.equal(verdict, v0) and torch.equal(sums, s0)) if k not in (31, 33, 34, 50) else None
    ev = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
    for _ in range(args.rounds):
        for k in ks:
            for j in range(3):
                libs[k].rxv_launch(ctypes.byref(gs[j % 2]), stream.cuda_stream, max(k, 0))
            ev[0].record(stream)
            for j in range(args.reps):
                libs[k].rxv_launch(ctypes.byref(gs[j % 2]), stream.cuda_stream, max(k, 0))
            ev[1].record(stream)
            torch.cuda.synchronize()
            res[k].append(ev[0].elapsed_time(ev[1]) * 1e3 / args.reps)
    out = {}
    for k in ks:
        us = float(np.median(res[k]))
        out[names[k]] = {"us": round(us, 2), "min_us": round(min(res[k]), 2), "frac": round(algo / us / 1e3 / 8000, 4),
                         "parity": ok[k]}
    trend = None
    if args.trend:
        evs = [torch.cuda.Event(enable_timing=True) for _ in range(args.trend + 1)]
        evs[0].record(stream)
        for i in range(args.trend):
            lib.rxv_launch(ctypes.byref(gs[i % 2]), stream.cuda_stream, 0)
            evs[i + 1].record(stream)
        torch.cuda.synchronize()
        t = [evs[i].elapsed_time(evs[i + 1]) * 1e3 for i in range(args.trend)]
        q = max(1, args.trend // 10)
        trend = {"per_launch_us": [round(x, 1) for x in t],
                 "first_decile_us": round(float(np.median(t[:q])), 2), "last_decile_us": round(float(np.median(t[-q:])), 2)}
    print(json.dumps({"product_verdicts_as_generated": product_ok,
                      "workload": f"1M x 1500-B {'IPv6' if args.ipv6 else 'IPv4'}/TCP in {stride}-B slots" + (", 2 rotating rings" if args.rotate else ", one ring re-read") + (f", a buffer list in {args.bufs} order" if args.bufs else ""), "algo_bytes": algo, "variants": out,
                      "trend": trend}, indent=1))


if __name__ == "__main__":
    main()
