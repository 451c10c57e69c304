"""One 64 KiB descriptor (BASELINE configs[0]) on the device: the tile
kernel (one workgroup) against csum_split (the descriptor cut into pieces
over many workgroups; selected here by sizing the arena at 2 MiB around it),
back-to-back average per launch; the two kernels' results must agree (their
parity with the oracle is tests/test_gpu_parity.py's).
  python tools/single_buffer_probe.py"""
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from netstack_amd import Engine  # noqa: E402
from netstack_amd.workloads import DESC_DTYPE  # noqa: E402

eng = Engine(0)
stream = torch.cuda.current_stream()
rng = np.random.default_rng(1)
host = rng.integers(0, 256, 2 << 20, dtype=np.uint8)
arena_full = torch.from_numpy(host).cuda()
for L in (1500, 16 << 10, 64 << 10, 256 << 10):
    d = np.zeros(1, dtype=DESC_DTYPE)
    d["off"], d["len"] = 0, L
    want = None  # the tile kernel's result; csum_split's must equal it
    desc = torch.from_numpy(d.view(np.uint8).copy()).cuda()
    out = torch.empty(1, dtype=torch.int16, device="cuda")
    for name, arena in (("tile", arena_full[:L]), ("split", arena_full)):
        for _ in range(20):
            eng.batch_tensors(arena, desc, out, stream=stream)
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record(stream)
        for _ in range(500):
            eng.batch_tensors(arena, desc, out, stream=stream)
        b.record(stream)
        torch.cuda.synchronize()
        got = out.cpu().numpy().view(np.uint16).copy()
        want = got if want is None else want
        ok = np.array_equal(got, want)
        print(f"{L:7d} B {name:5s}: {a.elapsed_time(b) * 1e3 / 500:6.2f} us/launch  same_as_tile={ok}", flush=True)
