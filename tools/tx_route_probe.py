#!/usr/bin/env python3
"""ns_csum_tcp_tx over an IPv4 route and an IPv6 route: 1M segments of one
1500-B MTU each (IPv4: MSS 1460, 54-B slots; IPv6: MSS 1440, 74-B slots, no
IPv4 header checksum, 16-B addresses in the pseudo-header), sendTCPBatch's
layout (slots, then the payload view), random bytes, two rotating batches.
Median of `--rounds` rounds of `--reps` back-to-back calls; algorithmic
bytes per segment = payload + IP and TCP headers read + the 2-B fields
written (IPv4 1,504, IPv6 1,502).  The first `--check` segments of batch 0,
filled by the two-pass call, must equal the same segments filled by
ns_csum_tcp_tx_multi (another kernel: the fused per-tile shape); parity with
the oracle is tests/test_gpu_tx_struct.py's (test_many_segments_full_tiles
runs the IPv6 route at this size class).

  python tools/tx_route_probe.py [--rounds 5] [--reps 20] [--check 4096]
                                  [--mss 64,256,536,1460,8960]
--mss: the IPv4 route at those segment sizes instead, ~1.5 GB of payload per
call (n = 1.5 GB / MSS, at most 16M segments).  --split: also time the two
passes one by one (tools/tx_variants.hip 28 and 92 through libns_txv.so).
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

ROUTES = {
    "ipv4": dict(mss=1460, slot=54, ip_at=14, ip_len=20, tcp_at=34, tcp_len=20,
                 src=bytes([10, 0, 0, 1]), dst=bytes([10, 0, 0, 2])),
    "ipv6": dict(mss=1440, slot=74, ip_at=14, ip_len=0, tcp_at=54, tcp_len=20,
                 src=bytes(range(0x20, 0x30)), dst=bytes(range(0xF0, 0x100))),
}


def geometry(route: str, n: int, gap: int = 4096, mss: int = 0) -> tuple[dict, int]:
    r = dict(ROUTES[route])
    if mss:
        r["mss"] = mss
    hdr = n * r["slot"]
    pay_off = (hdr + gap + 255) // 256 * 256
    size = n * r["mss"]
    return dict(hdr_off=0, pay_off=pay_off, size=size, protocol=6, **r), pay_off + size + 64


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rounds", type=int, default=5)
    ap.add_argument("--reps", type=int, default=20)
    ap.add_argument("--n", type=int, default=1 << 20)
    ap.add_argument("--check", type=int, default=4096)
    ap.add_argument("--mss", default="")
    ap.add_argument("--split", action="store_true")
    ap.add_argument("--pay-variant", type=int, default=28, help="--split: the payload pass variant (93: 4-lane)")
    args = ap.parse_args()
    n = args.n
    dev = torch.device("cuda", 0)
    eng = Engine(0)
    print(json.dumps({"start": True, "n": n}), flush=True)
    res = {}
    cases = [(r, 0, n) for r in ROUTES] if not args.mss else \
        [("ipv4", int(m), min(16 << 20, int(1.5e9 // int(m)))) for m in args.mss.split(",")]
    for route, mss, n in cases:
        geo, total = geometry(route, n, mss=mss)
        batches = [W.random_bytes_torch(7100 + b, total, dev) for b in range(2)]
        # cross-check: the first K segments as their own call through
        # ns_csum_tcp_tx_multi, on a copy of batch 0
        k = args.check
        ref = batches[0].clone()
        small = dict(geo, size=k * geo["mss"])
        eng.tcp_tx_multi(ref, [small])
        eng.tcp_tx(batches[0], geo)
        torch.cuda.synchronize()
        ok = bool(torch.equal(batches[0][:k * geo["slot"]], ref[:k * geo["slot"]]))
        del ref
        stream = torch.cuda.current_stream(dev)
        times = []
        for _ in range(args.rounds):
            for i in range(3):
                eng.tcp_tx(batches[i % 2], geo, stream=stream)
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record(stream)
            for i in range(args.reps):
                eng.tcp_tx(batches[i % 2], geo, stream=stream)
            e1.record(stream)
            torch.cuda.synchronize()
            times.append(e0.elapsed_time(e1) * 1e3 / args.reps)
        us = float(np.median(times))
        split = None
        if args.split:
            import ctypes

            sys.path.insert(0, os.path.join(ROOT, "tools"))
            from tx_drain_probe import TxGeo
            from netstack_amd.engine import addr_sum

            txv = ctypes.CDLL(os.path.join(ROOT, "netstack_amd", "lib", "libns_txv.so"))
            txv.txv_launch.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int]
            xs = torch.zeros(n, dtype=torch.int16, device=dev)

            def tg(a):
                return TxGeo(hdr=a.data_ptr() + geo["hdr_off"], pay=a.data_ptr() + geo["pay_off"], size=geo["size"],
                             n=n, mss=geo["mss"], slot=geo["slot"], ip_at=geo["ip_at"], ip_len=geo["ip_len"],
                             tcp_at=geo["tcp_at"], tcp_len=geo["tcp_len"],
                             addr_sum=addr_sum(geo["src"], geo["dst"]), proto=6, mode=3 if geo["ip_len"] else 2,
                             xs=xs.data_ptr(), xstride=1)

            tgs = [tg(b) for b in batches]
            pt, ht = [], []
            for i in range(4 + args.reps):
                e = [torch.cuda.Event(enable_timing=True) for _ in range(3)]
                e[0].record(stream)
                assert txv.txv_launch(ctypes.byref(tgs[i % 2]), stream.cuda_stream, args.pay_variant) == 0
                e[1].record(stream)
                assert txv.txv_launch(ctypes.byref(tgs[i % 2]), stream.cuda_stream, 92) == 0
                e[2].record(stream)
                torch.cuda.synchronize()
                if i >= 4:
                    pt.append(e[0].elapsed_time(e[1]) * 1e3)
                    ht.append(e[1].elapsed_time(e[2]) * 1e3)
            # the split fill must equal the product's (batch 0, refilled by both)
            ref = batches[0].clone()
            eng.tcp_tx(ref, geo)
            assert txv.txv_launch(ctypes.byref(tgs[0]), stream.cuda_stream, args.pay_variant) == 0
            assert txv.txv_launch(ctypes.byref(tgs[0]), stream.cuda_stream, 92) == 0
            torch.cuda.synchronize()
            split = {"payload_variant": args.pay_variant, "payload_pass_us": round(float(np.median(pt)), 2),
                     "header_pass_us": round(float(np.median(ht)), 2), "same_fill": bool(torch.equal(ref, batches[0]))}
            del ref
        per = geo["mss"] + (geo["ip_len"] or 0) + geo["tcp_len"] + (4 if geo["ip_len"] else 2)
        key = f"{route}_mss{geo['mss']}"
        res[key] = {"segments": n, "us": round(us, 2), "split": split, "min_us": round(min(times), 2), "algo_bytes_per_segment": per,
                      "frac_of_8TBs": round(n * per / us / 1e3 / 8000, 4), "first_segments_bit_exact": ok}
        print(json.dumps({key: res[key]}), flush=True)
        del batches
        torch.cuda.empty_cache()
    print(json.dumps({"workload": "2 rotating batches per case", "cases": res}), flush=True)


if __name__ == "__main__":
    main()
