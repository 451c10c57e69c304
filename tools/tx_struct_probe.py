#!/usr/bin/env python3
"""sendTCPBatch's TX fill two ways over the same 1M segments in its own layout
(54-B header slots, one payload view):
  paired_rx / paired_tx   the NS_BATCH_PAIRED descriptor table (3M
                          descriptors, 48 MB), without / with the stores
  struct                  ns_csum_tcp_tx: the geometry, no table; each wave's
                          header slots written back whole
  struct_v1..v3           its A/B variants (NS_CSUM_TX_VARIANT: 8 windows in
                          flight, nontemporal write-back, default-policy loads)
  struct_t8/t16/t64       8 / 16 / 64 segments per wave (NS_CSUM_TX_TILE)
  struct_fields           2-byte field stores instead (NS_TX_FIELDS_ONLY)
  struct_hdr_only         the IPv4 fields and CHECKSUM_PARTIAL sums only (no
                          payload read: the header-side floor)
  txv_noreduce            libns_txv.so (tools/tx_variants.hip): the stream
                          without any segment reduction (timing only)
  txv_u32 / txv_u4        32 / 4 windows in flight
Each over 2 rotating batches, median of `--rounds` rounds of `--reps`
back-to-back launches.  Every fill is checked byte for byte against
workloads.tx_split_expected.
  python tools/tx_struct_probe.py [--rounds 5] [--reps 20]
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
    geo = W.tx_struct_geometry(n)
    batches = [W.tx_split_batch(n, 7000 + r, dev)[0] for r in range(2)]
    pd = [torch.from_numpy(W.tx_split_desc(n, s, True).view(np.uint8).copy()).to(dev) for s in (True, False)]

    def env(k, v):
        def f(r, **kw):
            old = os.environ.get(k)
            os.environ[k] = v
            try:
                eng.tcp_tx(batches[r], geo, stream=stream, **kw)
            finally:
                if old is None:
                    del os.environ[k]
                else:
                    os.environ[k] = old
        return f

    from netstack_amd.engine import addr_sum

    class TxGeo(ctypes.Structure):
        _fields_ = [(k, ctypes.c_uint64) for k in ("hdr", "pay", "size", "n")] + \
                   [(k, ctypes.c_uint32) for k in ("mss", "slot", "tile", "lds_wave", "ip_at", "ip_len", "tcp_at",
                                                   "tcp_len", "addr_sum", "proto", "mode", "lds_rows")] + \
                   [("out", ctypes.c_void_p), ("wpg", ctypes.c_uint32), ("pad", ctypes.c_uint32)]

    TXV = ctypes.CDLL(os.path.join(ROOT, "netstack_amd", "lib", "libns_txv.so"))
    TXV.txv_launch.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int]

    def txv(k):
        def f(r):
            a = batches[r]
            t = TxGeo(hdr=a.data_ptr() + geo["hdr_off"], pay=a.data_ptr() + geo["pay_off"], size=geo["size"], n=n,
                      mss=geo["mss"], slot=geo["slot"], tile=0, ip_at=geo["ip_at"], ip_len=geo["ip_len"],
                      tcp_at=geo["tcp_at"], tcp_len=geo["tcp_len"], addr_sum=addr_sum(geo["src"], geo["dst"]),
                      proto=6, mode=3)
            assert TXV.txv_launch(ctypes.byref(t), stream.cuda_stream, k) == 0
        return f

    variants = {
        "paired_rx": lambda r: eng.batch_tensors(batches[r], pd[1], out, paired=True, stream=stream),
        "paired_tx": lambda r: eng.batch_tensors(batches[r], pd[0], out, paired=True, stream=stream, store=True),
        "struct": lambda r: eng.tcp_tx(batches[r], geo, stream=stream),
        "struct_v1": env("NS_CSUM_TX_VARIANT", "1"),
        "struct_v2": env("NS_CSUM_TX_VARIANT", "2"),
        "struct_v3": env("NS_CSUM_TX_VARIANT", "3"),
        "struct_t8": env("NS_CSUM_TX_TILE", "8"),
        "struct_t16": env("NS_CSUM_TX_TILE", "16"),
        "struct_t64": env("NS_CSUM_TX_TILE", "64"),
        "struct_fields": lambda r: eng.tcp_tx(batches[r], geo, stream=stream, fields_only=True),
        "struct_hdr_only": lambda r: eng.tcp_tx(batches[r], geo, stream=stream, mode="partial"),
        "txv_noreduce": txv(1),
        "txv_u32": txv(2),
        "txv_u4": txv(3),
    }
    checks = {}
    want = W.tx_split_expected(n, 7000, dev)
    for name, f in variants.items():
        if name.endswith("_rx") or name in ("struct_hdr_only", "txv_noreduce"):
            continue
        h = batches[0][:n * W.TX_HDR].view(n, W.TX_HDR)
        h[:, W.TX_IP_AT + 10:W.TX_IP_AT + 12] = 0
        h[:, W.TX_TCP_AT + 16:W.TX_TCP_AT + 18] = 0
        f(0)
        torch.cuda.synchronize()
        checks[name] = bool(torch.equal(batches[0], want))
    del want
    assert eng.sync() == 0
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
    med = {k: round(float(np.median(v)), 2) for k, v in times.items()}
    print(json.dumps({"packets": n, "median_us": med, "fill_bit_exact": checks,
                      "rounds_us": {k: [round(x, 2) for x in v] for k, v in times.items()}}, indent=1))


if __name__ == "__main__":
    main()
