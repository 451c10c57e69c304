#!/usr/bin/env python3
"""Workload for rocprofv3 --pmc passes (tools/profile.sh): calibration reads
of a known byte count in the product kernel's access shapes, then the product
kernel (ns_csum_batch_dev) on BASELINE configs 2, 3, 4.  Each launch is
repeated REPS times; tools/pmc_parse.py maps dispatches back to labels in the
order printed here."""
import ctypes
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import torch  # noqa: E402

from netstack_amd import Engine  # noqa: E402
from netstack_amd import workloads as W  # noqa: E402

REPS = 3
CAL_BYTES = (1 << 31) - 4096


def main():
    L = ctypes.CDLL(os.path.join(ROOT, "netstack_amd", "lib", "libns_tune.so"))
    L.nsk_calib_launch.argtypes = [ctypes.c_int, ctypes.c_void_p, ctypes.c_uint64, ctypes.c_void_p,
                                   ctypes.c_uint32, ctypes.c_void_p]
    dev = torch.device("cuda", 0)
    sp = torch.cuda.current_stream(dev).cuda_stream
    buf = torch.ones(CAL_BYTES, dtype=torch.uint8, device=dev)
    outb = torch.zeros(65536, dtype=torch.int32, device=dev)
    # runs of 8 / 4 chunks (buffer, default), coalesced nt, 16-lane groups nt
    for mode in (800, 400, 102, 2164):
        for _ in range(REPS):
            assert L.nsk_calib_launch(mode, buf.data_ptr(), CAL_BYTES, outb.data_ptr(), 8192, sp) == 0
        torch.cuda.synchronize()
        print(f"LABEL calib{mode} bytes={CAL_BYTES}", flush=True)
    del buf
    eng = Engine(0)
    for cfg in (2, 3, 4):
        b = W.config(cfg)
        arena = b.arena_device(dev)
        desc = torch.from_numpy(b.desc.view(np.uint8).copy()).to(dev)
        out = torch.empty(b.n, dtype=torch.int16, device=dev)
        for _ in range(REPS):
            eng.batch_tensors(arena, desc, out)
        torch.cuda.synchronize()
        # share of payload in packets csum_hyb sends to 16-lane groups (>= 64 chunks)
        big = float(b.desc["len"][b.desc["len"] >= 1024 - 15].sum()) / max(b.payload_bytes, 1)
        print(f"LABEL cfg{cfg} algorithmic_bytes={b.algorithmic_bytes} payload={b.payload_bytes} "
              f"arena={b.arena_bytes} n={b.n} big_share={big:.4f}", flush=True)
        del arena, desc, out


if __name__ == "__main__":
    main()
