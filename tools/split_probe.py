"""Huge-descriptor batches (csum_split vs the tile kernel): GB/s of payload
per ns_csum_batch_dev, device-resident, for a few layouts (the last three
in arenas above 4 GiB, where every csum_split piece reads through its own
SRD window).
  python tools/split_probe.py"""
import os
import sys
import time

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from netstack_amd import Engine  # noqa: E402
from netstack_amd import workloads as W  # noqa: E402

eng = Engine(0)
for n, L in ((1, 1 << 30), (4, 256 << 20), (64, 16 << 20), (100, 10 << 20), (200, 5 << 20), (255, 4 << 20), (256, 4 << 20), (1024, 1 << 20), (16384, 64 << 10),
             (1, (1 << 32) - 16), (2, 3 << 30), (8, 1 << 30)):
    d, end = W.make_desc(np.full(n, L, np.uint32), np.zeros(n, np.uint16), align=16)
    arena = torch.randint(0, 256, (end,), dtype=torch.uint8, device="cuda")
    desc = torch.from_numpy(d.view(np.uint8).copy()).cuda()
    out = eng.batch_tensors(arena, desc)
    torch.cuda.synchronize()
    t = time.perf_counter()
    for _ in range(10):
        eng.batch_tensors(arena, desc, out)
    torch.cuda.synchronize()
    dt = (time.perf_counter() - t) / 10
    del arena, desc, out
    print(f"{n:6d} x {L >> 10:8d} KiB: {dt * 1e6:9.1f} us  {n * L / dt / 1e9:7.0f} GB/s", flush=True)
