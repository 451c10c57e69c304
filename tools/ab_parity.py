#!/usr/bin/env python3
"""Parity of every variant in a tuning library (default: the small A/B
library, tune_ab.hip) against the production engine over adversarial
layouts: unaligned and odd starts, gaps, permuted and duplicated tables,
empty packets, lengths around the big-packet threshold, packets past the
W-only limit (exact accumulator).  The production path itself is checked
against the oracle by tests/test_gpu_parity.py.

  python tools/ab_parity.py [--lib netstack_amd/lib/libns_tune_ab.so]
"""
from __future__ import annotations

import argparse
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tools"))

import torch  # noqa: E402

from netstack_amd import Engine  # noqa: E402
from netstack_amd import workloads as W  # noqa: E402
import tune  # noqa: E402


def layouts(rng):
    out = []

    def packed(name, ln, align):
        d, end = W.make_desc(ln.astype(np.uint32), rng.integers(0, 65536, len(ln)).astype(np.uint16), align)
        out.append((name, d, end + 64))

    z = W.zipf_lengths(4, 200_000)
    for a in (16, 8, 2, 1):
        packed(f"zipf_align{a}", z, a)
    packed("zipf_64_600_align1", W.zipf_lengths(10, 100_000, 64, 600), 1)
    packed("uniform_200", np.full(100_000, 200), 16)
    packed("uniform_639_align1", np.full(50_000, 639), 1)
    packed("around_big_threshold", rng.integers(600, 700, 60_000), 4)
    packed("random_0_2000_align1", rng.integers(0, 2000, 100_000), 1)
    packed("tiny_0_40", rng.integers(0, 40, 200_000), 1)
    # gaps between packets
    ln = W.zipf_lengths(7, 100_000).astype(np.uint64)
    gap = rng.integers(0, 300, len(ln)).astype(np.uint64)
    off = np.zeros(len(ln), np.uint64)
    off[1:] = np.cumsum(ln[:-1] + gap[:-1])
    d = np.zeros(len(ln), W.DESC_DTYPE)
    d["off"], d["len"], d["initial"] = off, ln, rng.integers(0, 65536, len(ln))
    out.append(("zipf_gaps", d, int(off[-1] + ln[-1]) + 64))
    # permuted and duplicated tables over a packed Zipf arena
    d0, end = W.make_desc(z[:100_000], rng.integers(0, 65536, 100_000).astype(np.uint16), 16)
    out.append(("zipf_permuted", d0[rng.permutation(len(d0))].copy(), end + 64))
    out.append(("zipf_duplicated", np.repeat(d0, 2)[:150_000].copy(), end + 64))
    # the exact accumulator: a few packets past 131,040 B among small ones
    ln = np.concatenate([W.zipf_lengths(9, 20_000), rng.integers(131_041, 300_000, 40)])
    ln = ln[rng.permutation(len(ln))]
    packed("exact_mix", ln, 1)
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--lib", default=os.path.join(ROOT, "netstack_amd", "lib", "libns_tune_ab.so"))
    args = ap.parse_args()
    L = tune.load(args.lib)
    names = [L.nsk_tune_name(v).decode() for v in range(L.nsk_tune_count())]
    dev = torch.device("cuda", 0)
    sp = torch.cuda.current_stream(dev).cuda_stream
    eng = Engine(0)
    err = torch.zeros(1, dtype=torch.int64, device=dev)
    rng = np.random.default_rng(12345)
    fails = 0
    for name, d, nbytes in layouts(rng):
        arena = W.random_bytes_torch(99, nbytes, dev)
        desc = torch.from_numpy(d.view(np.uint8).copy()).to(dev)
        ref = eng.batch_tensors(arena, desc).cpu()
        out = torch.empty(len(d), dtype=torch.int16, device=dev)
        bad = []
        for v, nm in enumerate(names):
            out.fill_(0x5A5A)
            rc = L.nsk_tune_launch(v, arena.data_ptr(), nbytes, desc.data_ptr(), len(d), out.data_ptr(),
                                   err.data_ptr(), sp)
            torch.cuda.synchronize()
            if rc != 0 or not torch.equal(out.cpu(), ref):
                bad.append(nm)
        fails += len(bad)
        print(f"{name:24s} n={len(d):7d}  {'OK' if not bad else 'FAIL: ' + ','.join(bad)}", flush=True)
    print("ALL OK" if fails == 0 else f"{fails} FAILURES", flush=True)
    sys.exit(1 if fails else 0)


if __name__ == "__main__":
    main()
