#!/usr/bin/env python3
"""Where the TX fill's header-slot writes go (DESIGN
§4.7): the two passes of ns_csum_tcp_tx launched one by one through
libns_txv.so (tools/tx_variants.hip) with events around each, so every call
gives the payload pass's and the header pass's own durations.

Scenarios (1M x 1460-B segments, sendTCPBatch's layout, 54-B slots):
  P   the payload pass: grp (8-lane groups, txv 28) or win (windowed, 29)
  H   the header pass's store policy: 0 default, 1 nt, 2 sc1, 3 sc0 sc1,
      4 nt sc1, 5 sc0, 6 sc0 nt sc1 (txv 70 + H)
  rot 2: two batches alternating (fresh slots every call, as sendTCPBatch's
      NewPacketDescriptors gives them); 1: one batch re-filled
  gap none; flush: a 1 GiB read of another buffer after each call (evicts
      the MALL: the header pass's dirty lines are written back during it,
      not during the next payload pass); sleep: ~100 us of idle GPU
Every scenario's fill of batch 0 is checked byte for byte afterwards
(workloads.tx_split_expected).  Prints one JSON line per scenario and LABEL
lines for PMC passes (tools/tx_drain_parse.py maps dispatches to them).

  python tools/tx_drain_probe.py [--calls 24] [--warmup 4] [--only grp:0:2:none,...]
"""
from __future__ import annotations

import argparse
import ctypes
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import torch  # noqa: E402

from netstack_amd import workloads as W  # noqa: E402
from netstack_amd.engine import addr_sum  # noqa: E402


class TxGeo(ctypes.Structure):  # nsk::TxGeo (csum_kernels.h)
    _fields_ = [(k, ctypes.c_uint64) for k in ("hdr", "pay", "size", "n")] + \
               [(k, ctypes.c_uint32) for k in ("mss", "slot", "tile", "lds_wave", "ip_at", "ip_len", "tcp_at",
                                               "tcp_len", "addr_sum", "proto", "mode", "lds_rows")] + \
               [("out", ctypes.c_void_p), ("wpg", ctypes.c_uint32), ("pad", ctypes.c_uint32),
                ("xs", ctypes.c_void_p), ("htile", ctypes.c_uint32), ("xstride", ctypes.c_uint32)]


DEFAULT = ["win:0:2:none", "grp:0:2:none", "grp:0:1:none", "grp:0:2:flush", "win:0:2:flush", "grp:0:2:sleep",
           "grp:1:2:none", "grp:2:2:none", "grp:3:2:none", "grp:4:2:none", "grp:5:2:none", "grp:6:2:none",
           "win:1:2:none", "win:3:2:none", "win:0:1:none"]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--calls", type=int, default=24)
    ap.add_argument("--warmup", type=int, default=4)
    ap.add_argument("--n", type=int, default=1 << 20)
    ap.add_argument("--only", default="")
    ap.add_argument("--no-check", action="store_true")
    ap.add_argument("--htile", type=int, default=0, help="header-pass tile (segments per wave; 0: 64)")
    ap.add_argument("--hfloor", action="store_true",
                    help="in place of the header pass (policy 4), a plain copy of the slots onto themselves with "
                         "the same stores (txv 39; timing only: no fields, use --no-check)")
    ap.add_argument("--depth", type=int, default=2, help="header-pass tiles in flight per wave (3: txv 91; 1: one tile per wave, one-shot grid, txv 92)")
    ap.add_argument("--per-cu", type=int, default=0,
                    help="header-pass waves per CU (header policy 4 only, txv 90; 0: 24)")
    args = ap.parse_args()
    n = args.n
    dev = torch.device("cuda", 0)
    stream = torch.cuda.current_stream(dev)
    geo = W.tx_struct_geometry(n)
    batches = [W.tx_split_batch(n, 7000 + r, dev)[0] for r in range(2)]
    want = None if args.no_check else W.tx_split_expected(n, 7000, dev)
    xs = torch.zeros(n, dtype=torch.int16, device=dev)
    big = torch.zeros(1 << 30, dtype=torch.uint8, device=dev)
    sink = torch.zeros(4, dtype=torch.int32, device=dev)
    TXV = ctypes.CDLL(os.path.join(ROOT, "netstack_amd", "lib", "libns_txv.so"))
    TXV.txv_launch.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int]
    asum = addr_sum(geo["src"], geo["dst"])

    def launch(k, a):
        if k == 74 and args.hfloor:
            k = 39
        elif k == 74 and args.depth == 3:
            k = 91
        elif k == 74 and args.depth == 1:
            k = 92
        elif k == 74 and (args.per_cu or args.htile):
            k = 90
        t = TxGeo(hdr=a.data_ptr() + geo["hdr_off"], pay=a.data_ptr() + geo["pay_off"], size=geo["size"], n=n,
                  mss=geo["mss"], slot=geo["slot"], ip_at=geo["ip_at"], ip_len=geo["ip_len"], tcp_at=geo["tcp_at"],
                  tcp_len=geo["tcp_len"], addr_sum=asum, proto=6, mode=3, xs=xs.data_ptr(), xstride=1,
                  htile=args.htile, pad=args.per_cu)
        assert TXV.txv_launch(ctypes.byref(t), stream.cuda_stream, k) == 0

    def flush():  # tools/tx_variants.hip 37: a lane-consecutive read of 1 GiB
        t = TxGeo(hdr=big.data_ptr(), n=(1 << 30) // geo["slot"], slot=geo["slot"], out=sink.data_ptr())
        assert TXV.txv_launch(ctypes.byref(t), stream.cuda_stream, 37) == 0

    scen = args.only.split(",") if args.only else DEFAULT
    for sc in scen:
        p, h, rot, gap = sc.split(":")
        pk, hk, rot = (28 if p == "grp" else 29), 70 + int(h), int(rot)
        total = args.warmup + args.calls
        ev = [[torch.cuda.Event(enable_timing=True) for _ in range(4)] for _ in range(total)]
        torch.cuda.synchronize()
        print(f"LABEL begin {sc}", flush=True)
        for i in range(total):
            a = batches[i % rot]
            e = ev[i]
            e[0].record(stream)
            launch(pk, a)
            e[1].record(stream)
            launch(hk, a)
            e[2].record(stream)
            if gap == "flush":
                flush()
            elif gap == "sleep":
                torch.cuda._sleep(240_000)  # ~100 us at ~2.4 GHz
            e[3].record(stream)
        torch.cuda.synchronize()
        print(f"LABEL end {sc}", flush=True)
        pt = sorted(ev[i][0].elapsed_time(ev[i][1]) * 1e3 for i in range(args.warmup, total))
        ht = sorted(ev[i][1].elapsed_time(ev[i][2]) * 1e3 for i in range(args.warmup, total))
        gt = sorted(ev[i][2].elapsed_time(ev[i][3]) * 1e3 for i in range(args.warmup, total))
        ok = None
        if want is not None:
            b = batches[0]
            hh = b[:n * W.TX_HDR].view(n, W.TX_HDR)
            hh[:, W.TX_IP_AT + 10:W.TX_IP_AT + 12] = 0
            hh[:, W.TX_TCP_AT + 16:W.TX_TCP_AT + 18] = 0
            launch(pk, b)
            launch(hk, b)
            torch.cuda.synchronize()
            ok = bool(torch.equal(b, want))
        med = lambda v: v[len(v) // 2]  # noqa: E731
        mean = lambda v: sum(v) / len(v)  # noqa: E731
        print(json.dumps({"scenario": sc, "htile": args.htile, "per_cu": args.per_cu, "depth": args.depth, "hfloor": args.hfloor,
                          "payload_pass": p, "header_store_policy": int(h), "rotating_batches": rot,
                          "between_calls": gap, "calls": args.calls,
                          "payload_us": {"median": round(med(pt), 2), "mean": round(mean(pt), 2),
                                         "min": round(pt[0], 2), "max": round(pt[-1], 2)},
                          "header_us": {"median": round(med(ht), 2), "mean": round(mean(ht), 2),
                                        "min": round(ht[0], 2), "max": round(ht[-1], 2)},
                          "both_median_us": round(med(pt) + med(ht), 2),
                          "gap_us": round(med(gt), 2), "fill_bit_exact": ok}), flush=True)


if __name__ == "__main__":
    main()
