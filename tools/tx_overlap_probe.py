#!/usr/bin/env python3
"""Can the TX header pass hide behind the payload pass?  ns_csum_tcp_tx's two
passes (tools/tx_variants.hip 28: the group payload pass; 92: the production
header pass, one tile per wave, one-shot, nt sc1 stores) launched over parts
of the batch: the payload pass over part j, then on a second stream the header pass over part
j while the payload pass reads part j + 1; the last part's header pass after
the last payload part.  Against the production sequence (both passes over
the whole batch on one stream).  1M x 1460-B segments, sendTCPBatch's layout,
two rotating batches; every scenario's fill of batch 0 checked byte for byte.

  python tools/tx_overlap_probe.py [--calls 20] [--parts 1,2,4,8] [--prio]
"""
from __future__ import annotations

import argparse
import ctypes
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tools"))

import torch  # noqa: E402

from netstack_amd import workloads as W  # noqa: E402
from netstack_amd.engine import addr_sum  # noqa: E402
from tx_drain_probe import TxGeo  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--calls", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=4)
    ap.add_argument("--rounds", type=int, default=3)
    ap.add_argument("--n", type=int, default=1 << 20)
    ap.add_argument("--parts", default="1,2,4,8")
    ap.add_argument("--prio", action="store_true", help="the header stream at high priority")
    args = ap.parse_args()
    n = args.n
    dev = torch.device("cuda", 0)
    s1 = torch.cuda.current_stream(dev)
    s2 = torch.cuda.Stream(dev, priority=-1 if args.prio else 0)
    geo = W.tx_struct_geometry(n)
    batches = [W.tx_split_batch(n, 7000 + r, dev)[0] for r in range(2)]
    want = W.tx_split_expected(n, 7000, dev)
    xs = torch.zeros(n, dtype=torch.int16, device=dev)
    TXV = ctypes.CDLL(os.path.join(ROOT, "netstack_amd", "lib", "libns_txv.so"))
    TXV.txv_launch.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int]
    asum = addr_sum(geo["src"], geo["dst"])
    mss, slot = geo["mss"], geo["slot"]

    def launch(k, a, s0, s1_, stream):
        t = TxGeo(hdr=a.data_ptr() + geo["hdr_off"] + s0 * slot, pay=a.data_ptr() + geo["pay_off"] + s0 * mss,
                  size=min(geo["size"] - s0 * mss, (s1_ - s0) * mss), n=s1_ - s0, mss=mss, slot=slot, ip_at=geo["ip_at"],
                  ip_len=geo["ip_len"], tcp_at=geo["tcp_at"], tcp_len=geo["tcp_len"], addr_sum=asum, proto=6,
                  mode=3, xs=xs.data_ptr() + 2 * s0, xstride=1)
        assert TXV.txv_launch(ctypes.byref(t), stream.cuda_stream, k) == 0

    def fill(a, parts):
        if parts == 1:
            launch(28, a, 0, n, s1)
            launch(92, a, 0, n, s1)
            return
        cut = [((n * j // parts) + 63) // 64 * 64 for j in range(parts)] + [n]
        done = [torch.cuda.Event() for _ in range(parts)]
        for j in range(parts):
            launch(28, a, cut[j], cut[j + 1], s1)
            if j < parts - 1:
                done[j].record(s1)
                s2.wait_event(done[j])
                launch(92, a, cut[j], cut[j + 1], s2)
        launch(92, a, cut[-2], cut[-1], s1)
        end2 = torch.cuda.Event()
        end2.record(s2)
        s1.wait_event(end2)

    print(json.dumps({"setup": "done", "n": n}), flush=True)
    parts_list = [int(x) for x in args.parts.split(",")]
    res = {p: [] for p in parts_list}
    ok = {}
    for p in parts_list:
        b = batches[0]
        hh = b[:n * W.TX_HDR].view(n, W.TX_HDR)
        hh[:, W.TX_IP_AT + 10:W.TX_IP_AT + 12] = 0
        hh[:, W.TX_TCP_AT + 16:W.TX_TCP_AT + 18] = 0
        fill(b, p)
        torch.cuda.synchronize()
        ok[p] = bool(torch.equal(b, want))
        print(json.dumps({"parts": p, "fill_bit_exact": ok[p]}), flush=True)
    for _ in range(args.rounds):
        for p in parts_list:
            for i in range(args.warmup):
                fill(batches[i % 2], p)
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record(s1)
            for i in range(args.calls):
                fill(batches[i % 2], p)
            e1.record(s1)
            torch.cuda.synchronize()
            res[p].append(e0.elapsed_time(e1) * 1e3 / args.calls)
            print(json.dumps({"parts": p, "round_us": round(res[p][-1], 2)}), flush=True)
    for p in parts_list:
        v = sorted(res[p])
        print(json.dumps({"parts": p, "header_stream_priority": "high" if args.prio else "normal",
                          "us_per_call_median": round(v[len(v) // 2], 2), "us_per_call_min": round(v[0], 2),
                          "rounds": [round(x, 2) for x in res[p]], "fill_bit_exact": ok[p]}), flush=True)


if __name__ == "__main__":
    main()
