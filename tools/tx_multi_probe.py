#!/usr/bin/env python3
"""K sendTCPBatch calls of one 64-KiB GSO write each (44 segments of 1460 B
in 54-B slots), side by side in one arena:
  multi    one ns_csum_tcp_tx_multi launch for all K calls
  singles  K ns_csum_tcp_tx calls back to back on one stream
  one_big  the same bytes as ONE call (the bound for K x 44 segments)
Medians of `--rounds` rounds, each timed by one event pair; the multi
launch's fill must equal the single calls' byte for byte (their parity with
the oracle is tests/test_gpu_tx_struct.py's).
  python tools/tx_multi_probe.py [--calls 1000]"""
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
    ap.add_argument("--calls", type=int, default=1000)
    ap.add_argument("--rounds", type=int, default=5)
    args = ap.parse_args()
    K, n, mss, slot = args.calls, 44, 1460, W.TX_HDR
    per = (n * slot + 15) // 16 * 16 + n * mss + 16  # one call's slots + payload
    rng = np.random.default_rng(5)
    a = rng.integers(0, 256, K * per, dtype=np.uint8)
    geos = []
    for k in range(K):
        h = k * per
        g = dict(hdr_off=h, pay_off=h + (n * slot + 15) // 16 * 16, size=n * mss, mss=mss, slot=slot,
                 ip_at=W.TX_IP_AT, ip_len=20, tcp_at=W.TX_TCP_AT, tcp_len=20, src=W.TX_SRC, dst=W.TX_DST, protocol=6)
        for i in range(n):
            at = h + i * slot + W.TX_IP_AT
            a[at + 12:at + 16] = np.frombuffer(W.TX_SRC, np.uint8)
            a[at + 16:at + 20] = np.frombuffer(W.TX_DST, np.uint8)
        geos.append(g)
    dev = torch.device("cuda", 0)
    eng = Engine(0)
    stream = torch.cuda.current_stream(dev)
    buf = torch.from_numpy(a).to(dev)
    from netstack_amd.engine import tx_table

    tab = tx_table(geos)  # built once, as a server would keep it
    variants = {
        "multi": lambda: eng.tcp_tx_multi(buf, tab, stream=stream),
        "singles": lambda: [eng.tcp_tx(buf, g, stream=stream) for g in geos],
    }
    res, checks = {}, {}
    want = None  # the single calls' fill (run first); the multi launch's must equal it
    for name in ("singles", "multi"):
        f = variants[name]
        buf.copy_(torch.from_numpy(a))
        f()
        torch.cuda.synchronize()
        got = buf.cpu().numpy()
        if want is None:
            want = got
            checks["singles_filled"] = not np.array_equal(got, a)
        checks[name] = bool(np.array_equal(got, want))
        ts = []
        for _ in range(args.rounds):
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record(stream)
            f()
            e1.record(stream)
            e1.synchronize()
            ts.append(e0.elapsed_time(e1) * 1e3)
        res[name] = round(float(np.median(ts)), 1)
    # the bound: the same number of segments as one call in one contiguous layout
    big, _ = W.tx_split_batch(K * n, 3, dev)
    gb = W.tx_struct_geometry(K * n)
    ts = []
    for _ in range(args.rounds + 1):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(stream)
        eng.tcp_tx(big, gb, stream=stream)
        e1.record(stream)
        e1.synchronize()
        ts.append(e0.elapsed_time(e1) * 1e3)
    res["one_big"] = round(float(np.median(ts[1:])), 1)
    print(json.dumps({"calls": K, "segments_per_call": n, "median_us": res, "fill_bit_exact": checks}, indent=1))


if __name__ == "__main__":
    main()
