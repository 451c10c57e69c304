"""One chained run of n descriptors (descriptor 0 a head, every other one
NS_DESC_CONT): host-timed ns_csum_batch_dev(CHAINED) per launch, which
includes the checksum kernel and the run fold (profiles/r01/chain_fold.txt).
  python tools/chain_probe.py"""
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
for n, L in ((1000, 64), (100000, 64), (1000000, 64), (512, 131072)):
    lengths = np.full(n, L, np.uint32)
    flags = np.full(n, 2, np.uint16)
    flags[0] = 0
    d, end = W.make_desc(lengths, np.zeros(n, np.uint16), align=16, flags=flags)
    arena = torch.randint(0, 256, (end,), dtype=torch.uint8, device="cuda")
    desc = torch.from_numpy(d.view(np.uint8).copy()).cuda()
    out = eng.batch_tensors(arena, desc, chained=True)
    torch.cuda.synchronize()
    t = time.perf_counter()
    for _ in range(3):
        eng.batch_tensors(arena, desc, out, chained=True)
    torch.cuda.synchronize()
    print(n, L, "one run: %.1f us/launch" % ((time.perf_counter() - t) / 3 * 1e6), flush=True)
