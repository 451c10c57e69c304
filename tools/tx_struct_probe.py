#!/usr/bin/env python3
"""sendTCPBatch's TX fill two ways over the same 1M segments in its own layout
(54-B header slots, one payload view):
  paired_rx / paired_tx   the NS_BATCH_PAIRED descriptor table (3M
                          descriptors, 48 MB), without / with the stores
  struct                  ns_csum_tcp_tx: the geometry, no table; a payload
                          pass, then a header pass writing the slots back whole
  struct_v1..v3           its A/B variants (ns_csum_set_tx_tuning variant: one
                          fused pass, nontemporal write-back, wave reductions)
  struct_grppay           variant 5: the payload pass in 8-lane groups
  struct_norot            the product on one batch every call (its header
                          slots re-used: their writes stay in the MALL)
  struct_hdr1shot         the header pass one-shot (round 4's), not persistent
  struct_pP_hH            P segments per wave in the payload pass, H in the
                          header pass (NS_CSUM_TX_TILE / _HTILE)
  struct_fields           2-byte field stores instead (NS_TX_FIELDS_ONLY)
  struct_hdr_only         the IPv4 fields and CHECKSUM_PARTIAL sums only (no
                          payload read: the header-side floor)
  txv_*                   libns_txv.so (tools/tx_variants.hip), timing
                          only: noreduce (no segment reductions), u8 / u4 (8 /
                          4 windows in flight), nowb (no header write-back),
                          stream (neither: the bare stream + header reads)
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
    ap.add_argument("--only", default="", help="comma-separated variant names")
    ap.add_argument("--trend", type=int, default=0,
                    help="then time this many back-to-back product calls one by one (rotating batches)")
    args = ap.parse_args()
    n = args.n
    dev = torch.device("cuda", 0)
    stream = torch.cuda.current_stream(dev)
    eng = Engine(0)
    out = torch.empty(3 * n, dtype=torch.int16, device=dev)
    out2 = torch.empty(2 * n, dtype=torch.int16, device=dev)
    geo = W.tx_struct_geometry(n)
    batches = [W.tx_split_batch(n, 7000 + r, dev)[0] for r in range(2)]
    pd = [torch.from_numpy(W.tx_split_desc(n, s, True).view(np.uint8).copy()).to(dev) for s in (True, False)]

    _knob = {"NS_CSUM_TX_VARIANT": "variant", "NS_CSUM_TX_TILE": "tile", "NS_CSUM_TX_HTILE": "htile",
             "NS_CSUM_TX_PASSES": "passes"}

    def env(k, v, k2=None, v2=None):
        """A call with ns_csum_tcp_tx's A/B knobs set through
        ns_csum_set_tx_tuning (the library reads the environment only at
        ns_csum_init), reset to production after it."""
        def f(r, **kw):
            kn = {_knob[k]: int(v)}
            if k2 is not None:
                kn[_knob[k2]] = int(v2)
            eng.set_tx_tuning(**kn)
            try:
                eng.tcp_tx(batches[r], geo, stream=stream, **kw)
            finally:
                eng.set_tx_tuning()
        return f

    from netstack_amd.engine import addr_sum

    class TxGeo(ctypes.Structure):
        _fields_ = [(k, ctypes.c_uint64) for k in ("hdr", "pay", "size", "n")] + \
                   [(k, ctypes.c_uint32) for k in ("mss", "slot", "tile", "lds_wave", "ip_at", "ip_len", "tcp_at",
                                                   "tcp_len", "addr_sum", "proto", "mode", "lds_rows")] + \
                   [("out", ctypes.c_void_p), ("wpg", ctypes.c_uint32), ("pad", ctypes.c_uint32),
                    ("xs", ctypes.c_void_p), ("htile", ctypes.c_uint32), ("xstride", ctypes.c_uint32)]

    TXV = ctypes.CDLL(os.path.join(ROOT, "netstack_amd", "lib", "libns_txv.so"))
    TXV.txv_launch.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int]

    xs = torch.zeros(n, dtype=torch.int16, device=dev)
    sink = torch.zeros(4, dtype=torch.int32, device=dev)

    big = []

    def txv_big(k):
        """A floor kernel (19-27) over 1 GiB of its own: the asymptotic rate
        of the same access shape."""
        def f(r):
            if not big:
                big.append(torch.zeros(1 << 30, dtype=torch.uint8, device=dev))
            t = TxGeo(hdr=big[0].data_ptr(), n=(1 << 30) // geo["slot"], slot=geo["slot"], out=sink.data_ptr())
            assert TXV.txv_launch(ctypes.byref(t), stream.cuda_stream, k) == 0
        return f

    def txv(k, tile=0, rot=True, htile=0):
        def f(r):
            a = batches[r if rot else 0]
            t = TxGeo(hdr=a.data_ptr() + geo["hdr_off"], pay=a.data_ptr() + geo["pay_off"], size=geo["size"], n=n,
                      mss=geo["mss"], slot=geo["slot"], tile=tile, ip_at=geo["ip_at"], ip_len=geo["ip_len"],
                      tcp_at=geo["tcp_at"], tcp_len=geo["tcp_len"], addr_sum=addr_sum(geo["src"], geo["dst"]),
                      proto=6, mode=3, xs=xs.data_ptr() if k >= 8 else None, xstride=1,
                      out=sink.data_ptr() if 19 <= k <= 27 or 36 <= k <= 38 or k == 47 else None,  # the floor kernels' sink only
                      htile=htile)
            assert TXV.txv_launch(ctypes.byref(t), stream.cuda_stream, k) == 0
        return f

    variants = {
        "paired_rx": lambda r: eng.batch_tensors(batches[r], pd[1], out, paired=True, stream=stream),
        "paired_tx": lambda r: eng.batch_tensors(batches[r], pd[0], out, paired=True, stream=stream, store=True),
        "struct": lambda r: eng.tcp_tx(batches[r], geo, stream=stream),
        "struct_fused": env("NS_CSUM_TX_VARIANT", "1"),
        "struct_ntwb": env("NS_CSUM_TX_VARIANT", "2"),
        "struct_hdr1shot": env("NS_CSUM_TX_VARIANT", "4"),
        "struct_grppay": env("NS_CSUM_TX_VARIANT", "5"),
        "txv_pay_group": txv(28),
        "txv_pay_window": txv(29),
        "txv_2p_grp_nt": txv(30),
        "txv_2p_grp_ntwb": txv(31),
        "txv_2p_grp_nt_ntwb": txv(32),
        "txv_pay_group_nt": txv(33),
        "txv_2p_window": txv(9),
        "txv_2p_window_norot": txv(9, rot=False),
        "txv_2p_group_norot": txv(35, rot=False),
        "txv_2p_group": txv(35),
        "txv_2p_grp_ntwb_norot": txv(31, rot=False),
        "struct_fields": lambda r: eng.tcp_tx(batches[r], geo, stream=stream, fields_only=True),
        "struct_hdr_only": lambda r: eng.tcp_tx(batches[r], geo, stream=stream, mode="partial"),
        "txv_stream_t8": txv(5, 8),
        "txv_u16": txv(0),
        "txv_u8": txv(2),
        "txv_u4": txv(3),
        "txv_noreduce": txv(1),
        "txv_stream": txv(5),
        "txv_2p_u12": txv(8),
        "txv_2p_u16": txv(9),
        "txv_2p_u8": txv(10),
        "txv_2p_hdr4": txv(12),
        "txv_2p_hdr16": txv(13),
        "txv_2p_hdr2": txv(14),
        "txv_2p_1shot": txv(15),
        "txv_2p_hdr24": txv(16),
        "txv_2p_hdr32": txv(17),
        "txv_hdr_pass": txv(18),
        "floor_slots_rw": txv(19),
        "floor_slots_rd": txv(20),
        "floor_slots_wr": txv(21),
        "floor_slots_wr_a1": txv(22),
        "floor_slots_wr_a2": txv(23),
        "floor_slots_wr_a3": txv(24),
        "floor_1g_rw": txv_big(19),
        "floor_1g_rd": txv_big(20),
        "floor_1g_wr": txv_big(21),
        "floor_1g_wr_a2": txv_big(23),
        "hdr_pc8": txv(40), "hdr_pc16": txv(41), "hdr_pc32": txv(42), "hdr_pc48": txv(43), "hdr_1shot": txv(44),
        "hdr_t32": txv(18, htile=32), "hdr_t48": txv(18, htile=48), "hdr_1shot_t32": txv(44, htile=32),
        "hdr_t128": txv(18, htile=128), "hdr_t128_pc12": txv(45, htile=128), "hdr_t128_pc16": txv(41, htile=128),
        "hdr_t96_pc12": txv(45, htile=96),
        "hdr_nt": txv(46), "floor_slots_wr_co_nt": txv(47), "floor_1g_wr_co_nt": txv_big(47),
        "floor_1g_rw_co": txv_big(36),
        "floor_1g_rd_co": txv_big(37),
        "floor_1g_wr_co": txv_big(38),
        "floor_slots_rw_co": txv(36),
        "floor_slots_rd_co": txv(37),
        "floor_slots_wr_co": txv(38),
        "floor_slots_rw_a1": txv(25),
        "floor_slots_rw_a2": txv(26),
        "floor_slots_rw_a3": txv(27),
        "struct_out": lambda r: eng.tcp_tx(batches[r], geo, out=out2, stream=stream),
        "struct_norot": lambda r: eng.tcp_tx(batches[0], geo, stream=stream),
        "struct_out_norot": lambda r: eng.tcp_tx(batches[0], geo, out=out2, stream=stream),
    }
    for pt in (4, 8, 16, 32):
        for ht in (16, 32, 64, 96, 128, 192):
            variants[f"struct_p{pt}_h{ht}"] = env("NS_CSUM_TX_TILE", str(pt), "NS_CSUM_TX_HTILE", str(ht))
    if args.only:
        variants = {k: v for k, v in variants.items() if k in args.only.split(",")}
    checks = {}
    want = W.tx_split_expected(n, 7000, dev)
    for name, f in variants.items():
        if name.endswith("_rx") or name in ("struct_hdr_only", "txv_noreduce") or "nowb" in name or "stream" in name \
                or name.startswith(("floor_", "txv_hdr_pass", "hdr_")):
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
    host = {k: [] for k in variants}
    import time
    for _ in range(args.rounds):
        for name, f in variants.items():
            for k in range(3):
                f(k % 2)
            a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            a.record(stream)
            t0 = time.perf_counter()
            for k in range(args.reps):
                f(k % 2)
            host[name].append((time.perf_counter() - t0) * 1e6 / args.reps)
            b.record(stream)
            b.synchronize()
            times[name].append(a.elapsed_time(b) * 1e3 / args.reps)
    med = {k: round(float(np.median(v)), 2) for k, v in times.items()}
    trend = None
    if args.trend:
        evs = [torch.cuda.Event(enable_timing=True) for _ in range(args.trend + 1)]
        evs[0].record(stream)
        for i in range(args.trend):
            eng.tcp_tx(batches[i % 2], geo, stream=stream)
            evs[i + 1].record(stream)
        torch.cuda.synchronize()
        t = [evs[i].elapsed_time(evs[i + 1]) * 1e3 for i in range(args.trend)]
        q = max(1, args.trend // 10)
        trend = {"per_call_us": [round(x, 1) for x in t], "first_decile_us": round(float(np.median(t[:q])), 2),
                 "last_decile_us": round(float(np.median(t[-q:])), 2), "median_us": round(float(np.median(t)), 2)}
    print(json.dumps({"packets": n, "median_us": med, "fill_bit_exact": checks, "trend": trend,
                      "host_enqueue_us_per_call": {k: round(float(np.median(v)), 1) for k, v in host.items()},
                      "rounds_us": {k: [round(x, 2) for x in v] for k, v in times.items()}}, indent=1))


if __name__ == "__main__":
    main()
