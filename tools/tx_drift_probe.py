#!/usr/bin/env python3
"""Does the TX fill slow down over a run because of its own writes?
  Runs 60 back-to-back calls of each, in this order, on one
1M-segment batch: the production two passes; the same two passes with the
header pass's write-back removed (libns_txv.so variant 11, timing only);
the production two passes again.  Run it under rocprofv3 --kernel-trace and
read the per-launch durations in order (tools/tx_drift_probe.py prints the
call boundaries).  python tools/tx_drift_probe.py"""
import ctypes
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import torch  # noqa: E402

from netstack_amd import Engine  # noqa: E402
from netstack_amd import workloads as W  # noqa: E402
from netstack_amd.engine import addr_sum  # noqa: E402


class TxGeo(ctypes.Structure):
    _fields_ = [(k, ctypes.c_uint64) for k in ("hdr", "pay", "size", "n")] + \
               [(k, ctypes.c_uint32) for k in ("mss", "slot", "tile", "lds_wave", "ip_at", "ip_len", "tcp_at",
                                               "tcp_len", "addr_sum", "proto", "mode", "lds_rows")] + \
               [("out", ctypes.c_void_p), ("wpg", ctypes.c_uint32), ("pad", ctypes.c_uint32),
                ("xs", ctypes.c_void_p), ("htile", ctypes.c_uint32), ("xstride", ctypes.c_uint32)]


def main():
    n = 1 << 20
    dev = torch.device("cuda", 0)
    stream = torch.cuda.current_stream(dev)
    eng = Engine(0)
    arena, _ = W.tx_split_batch(n, 7000, dev)
    geo = W.tx_struct_geometry(n)
    xs = torch.empty(n, dtype=torch.int16, device=dev)
    L = ctypes.CDLL(os.path.join(ROOT, "netstack_amd", "lib", "libns_txv.so"))
    L.txv_launch.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int]
    t = TxGeo(hdr=arena.data_ptr() + geo["hdr_off"], pay=arena.data_ptr() + geo["pay_off"], size=geo["size"], n=n,
              mss=geo["mss"], slot=geo["slot"], tile=0, ip_at=geo["ip_at"], ip_len=geo["ip_len"],
              tcp_at=geo["tcp_at"], tcp_len=geo["tcp_len"], addr_sum=addr_sum(geo["src"], geo["dst"]), proto=6,
              mode=3, xs=xs.data_ptr(), htile=0, xstride=1)
    for phase in ("production", "no_writeback", "production_again"):
        for _ in range(60):
            if phase == "no_writeback":
                assert L.txv_launch(ctypes.byref(t), stream.cuda_stream, 11) == 0
            else:
                eng.tcp_tx(arena, geo, stream=stream)
        torch.cuda.synchronize()
        print(f"PHASE {phase} 60 calls", flush=True)


if __name__ == "__main__":
    main()
