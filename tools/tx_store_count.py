#!/usr/bin/env python3
"""What the TX fill's stores cost, by how many there are and where: the
bench's TX batch (1M x 1500-B IPv4/TCP packets, fused 2-descriptor table,
bench.py --config 8) timed back to back over 2 rotating arenas with
  rx        no store flags (the RX pass over the same bytes)
  both      the product's two stores per packet (IPv4 byte 10, TCP byte 36)
  ip        only the IPv4 store
  tcp       only the TCP store
  half      both stores on every other packet (1M stores, half the lines)
  same_sector  timing only: the TCP store moved to packet byte 14, beside the IPv4 one
Interleaved rounds, median per variant.  Results are not checked here (the
TX path's parity is tests/test_gpu_parity.py::test_tx_store_device_resident).

  python tools/tx_store_count.py [--rounds 5] [--reps 20]
"""
from __future__ import annotations

import argparse
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
    args = ap.parse_args()
    dev = torch.device("cuda", 0)
    stream = torch.cuda.current_stream(dev)
    eng = Engine(0)
    n = W.RX_N if hasattr(W, "RX_N") else 1 << 20
    arenas = [W.tx_batch(n, 8000 + r, dev)[0] for r in range(2)]
    base = W.tx_desc(n)
    store = np.uint16(0x4)
    var = {}
    d = base.copy()
    d["flags"] &= ~np.uint16(0xFFFC)
    var["rx"] = d
    var["both"] = base.copy()
    d = base.copy()
    d["flags"][1::2] &= ~store
    var["ip"] = d
    d = base.copy()
    d["flags"][0::2] &= ~store
    var["tcp"] = d
    d = base.copy()
    d["flags"][2::4] &= ~store
    d["flags"][3::4] &= ~store
    var["half"] = d
    d = base.copy()  # timing only: the TCP store moved next to the IPv4 one (packet byte 14, same sector)
    d["flags"][1::2] = (d["flags"][1::2] & np.uint16(0xF)) | np.uint16(2 << 4)
    var["same_sector"] = d
    descs = {k: torch.from_numpy(v.view(np.uint8).copy()).to(dev) for k, v in var.items()}
    out = torch.empty(2 * n, dtype=torch.int16, device=dev)
    res = {k: [] for k in var}
    for k in var:  # warm
        for a in arenas:
            eng.batch_tensors(a, descs[k], out, stream=stream, store=k != "rx")
    torch.cuda.synchronize()
    for _ in range(args.rounds):
        for k in var:
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record(stream)
            for i in range(args.reps):
                eng.batch_tensors(arenas[i % 2], descs[k], out, stream=stream, store=k != "rx")
            e1.record(stream)
            torch.cuda.synchronize()
            res[k].append(e0.elapsed_time(e1) * 1e3 / args.reps)
    eng.sync()
    for k, v in res.items():
        print(f"  {k:6s} median {np.median(v):8.1f} us  min {np.min(v):8.1f}", flush=True)


if __name__ == "__main__":
    main()
