#!/usr/bin/env python3
"""TX fill in two layouts of the same 1M 1500-B IPv4/TCP segments (DESIGN.md
§4.5).  Hypothesis from the round-3 counters and timings: the stores cost
what they cost because each packet's two checksum fields lie in their own
DRAM row (the wire layout, one 1,504-B stride per packet), so every written
sector is a row activation plus a read/write turnaround against the read
stream.  In the layout sendTCPBatch itself builds (stack.NewPacketDescriptors:
one buffer of n 54-B header slots, the payload in a separate view;
workloads.tx_split_*), the fields are dense: the same 2M stores fill whole
rows.

Variants, each over 2 rotating batches, median of `--rounds` rounds of
`--reps` back-to-back launches (one HIP event pair per round):
  wire_fused_rx / _tx      bench --config 7 / 8 (2 descriptors per packet)
  wire_chained_rx / _tx    the same packets, 3 chained descriptors
  split_rx / split_tx      the sendTCPBatch layout, 3 chained descriptors
  paired_rx / paired_tx    the sendTCPBatch layout, NS_BATCH_PAIRED (the
                           payload + TCP header pair folded in the tile)
  paired_two_pass          paired_rx, then libns_tune.so's store pass (the
                           table re-read, the results from `out`)
  store_pass_only          that store pass alone, repeated
The store cost of a layout is tx - rx.  Every TX fill is checked byte for
byte against independently computed arenas.

  python tools/tx_layout_probe.py [--rounds 5] [--reps 20]
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


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rounds", type=int, default=5)
    ap.add_argument("--reps", type=int, default=20)
    ap.add_argument("--n", type=int, default=1 << 20)
    args = ap.parse_args()
    n = args.n
    dev = torch.device("cuda", 0)
    stream = torch.cuda.current_stream(dev)
    eng = Engine(0)
    out = torch.empty(3 * n, dtype=torch.int16, device=dev)
    L = ctypes.CDLL(os.path.join(ROOT, "netstack_amd", "lib", "libns_tune.so"))
    L.nsk_store_pass_launch.argtypes = [ctypes.c_void_p, ctypes.c_uint64, ctypes.c_void_p, ctypes.c_uint32,
                                        ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p]
    err = torch.zeros(1, dtype=torch.int64, device=dev)

    def tdesc(d):
        return torch.from_numpy(d.view(np.uint8).copy()).to(dev)

    batches = {}
    for r in range(2):
        seed = 7000 + r
        wire, _ = W.tx_batch(n, seed, dev)
        split, _ = W.tx_split_batch(n, seed, dev)
        batches[r] = (wire, split)
    wd = {f: (tdesc(W.tx_desc(n, f)), tdesc(W._tcp_desc(n, f))) for f in (True, False)}
    sd = (tdesc(W.tx_split_desc(n, True)), tdesc(W.tx_split_desc(n, False)))
    pd = (tdesc(W.tx_split_desc(n, True, True)), tdesc(W.tx_split_desc(n, False, True)))

    variants = {
        "wire_fused_rx": lambda r: eng.batch_tensors(batches[r][0], wd[True][1], out, stream=stream),
        "wire_fused_tx": lambda r: eng.batch_tensors(batches[r][0], wd[True][0], out, stream=stream, store=True),
        "wire_chained_rx": lambda r: eng.batch_tensors(batches[r][0], wd[False][1], out, chained=True, stream=stream),
        "wire_chained_tx": lambda r: eng.batch_tensors(batches[r][0], wd[False][0], out, chained=True,
                                                       stream=stream, store=True),
        "split_rx": lambda r: eng.batch_tensors(batches[r][1], sd[1], out, chained=True, stream=stream),
        "split_tx": lambda r: eng.batch_tensors(batches[r][1], sd[0], out, chained=True, stream=stream, store=True),
        "paired_rx": lambda r: eng.batch_tensors(batches[r][1], pd[1], out, paired=True, stream=stream),
        "paired_tx": lambda r: eng.batch_tensors(batches[r][1], pd[0], out, paired=True, stream=stream, store=True),
    }

    def store_pass(r):
        a = batches[r][1]
        assert L.nsk_store_pass_launch(a.data_ptr(), a.numel(), pd[0].data_ptr(), 3 * n, out.data_ptr(),
                                       err.data_ptr(), stream.cuda_stream) == 0

    variants["paired_two_pass"] = lambda r: (eng.batch_tensors(batches[r][1], pd[0], out, paired=True,
                                                               stream=stream), store_pass(r))
    variants["store_pass_only"] = store_pass
    # correctness of every TX fill (checked after one launch on batch 0)
    checks = {}
    for name in ("wire_fused_tx", "wire_chained_tx", "split_tx", "paired_tx", "paired_two_pass"):
        if name.startswith("wire"):  # the fields back to zero (a fill sums them)
            p = batches[0][0].view(n, W.RX_STRIDE)
            p[:, 10:12] = 0
            p[:, 36:38] = 0
        else:
            h = batches[0][1][:n * W.TX_HDR].view(n, W.TX_HDR)
            h[:, W.TX_IP_AT + 10:W.TX_IP_AT + 12] = 0
            h[:, W.TX_TCP_AT + 16:W.TX_TCP_AT + 18] = 0
        variants[name](0)
        torch.cuda.synchronize()
        want = W.rx_batch(n, 7000, dev)[0] if name.startswith("wire") else W.tx_split_expected(n, 7000, dev)
        got = batches[0][0] if name.startswith("wire") else batches[0][1]
        checks[name] = bool(torch.equal(got, want))
        del want
    assert eng.sync() == 0 and int(err.item()) == 0
    times = {k: [] for k in variants}
    for _ in range(args.rounds):
        for name, f in variants.items():
            for k in range(3):
                f(k % 2)
            a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            a.record(stream)
            for k in range(args.reps):
                f(k % 2)
            b.record(stream)
            b.synchronize()
            times[name].append(a.elapsed_time(b) * 1e3 / args.reps)
    med = {k: float(np.median(v)) for k, v in times.items()}
    res = {"packets": n, "median_us": med, "rounds_us": times, "tx_fill_bit_exact": checks,
           "store_cost_us": {"wire_fused": med["wire_fused_tx"] - med["wire_fused_rx"],
                             "wire_chained": med["wire_chained_tx"] - med["wire_chained_rx"],
                             "split": med["split_tx"] - med["split_rx"],
                             "paired": med["paired_tx"] - med["paired_rx"],
                             "paired_two_pass": med["paired_two_pass"] - med["paired_rx"]}}
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    main()
