#!/usr/bin/env python3
"""What a length-classed work list could buy on cfg4 (SURVEY §7 step 5,
VERDICT r02 item 4), measured before building one: the production kernel
(ns_csum_batch_dev) on the Zipf batch as bench.py runs it (2 rotating
arenas and tables, back to back), against the same packets with the
descriptor table reordered so that each 64-descriptor tile holds one length
class (<= 5 chunks, 6-39, >= 40; stable within windows of W descriptors):
  perm    — the table permuted, the arena unchanged (what a class-binned work
            list over the caller's arena would read);
  packed  — the packets re-laid in the permuted order too (an upper bound:
            class-pure tiles over contiguous memory);
  sorted  — packed, ordered by length within each window.
Every variant's results are checked against the baseline's (permuted back).

  python tools/class_probe.py [--window 4096] [--rounds 3] [--reps 40]
"""
from __future__ import annotations

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


def classes(d):
    a = d["off"] & np.uint64(15)
    nch = ((a + d["len"].astype(np.uint64) - np.uint64(1)) >> np.uint64(4)) + np.uint64(1)
    return np.where(nch <= 5, 0, np.where(nch < 40, 1, 2))


def window_order(key, window):
    n = len(key)
    order = np.empty(n, dtype=np.int64)
    for s in range(0, n, window):
        e = min(n, s + window)
        order[s:e] = s + np.argsort(key[s:e], kind="stable")
    return order


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--window", type=int, default=4096)
    ap.add_argument("--rounds", type=int, default=3)
    ap.add_argument("--reps", type=int, default=40)
    ap.add_argument("--json", default="")
    args = ap.parse_args()
    dev = torch.device("cuda", 0)
    stream = torch.cuda.current_stream(dev)
    eng = Engine(0)
    b = W.config(4)
    ab = b.algorithmic_bytes
    cls = classes(b.desc)
    perm = window_order(cls, args.window)
    srt = window_order(b.desc["len"].astype(np.int64), args.window)
    layouts = {}
    arenas = [b.arena_device(dev), W.random_bytes_torch(b.seed + 77, b.arena_bytes, dev)]
    layouts["base"] = (arenas, b.desc, np.arange(b.n))
    layouts["perm"] = (arenas, b.desc[perm].copy(), perm)
    for name, order in (("packed", perm), ("sorted", srt)):
        d, end = W.make_desc(b.desc["len"][order], b.desc["initial"][order], 16)
        size = ((end + 15) // 16) * 16
        layouts[name] = ([W.random_bytes_torch(b.seed + 5, size, dev), W.random_bytes_torch(b.seed + 6, size, dev)],
                         d, order)
    res = {k: [] for k in layouts}
    dd = {}
    for name, (ars, d, order) in layouts.items():
        t = torch.from_numpy(d.view(np.uint8).copy()).to(dev)
        dd[name] = [t, t.clone()]
    ref = eng.batch_tensors(arenas[0], dd["base"][0]).cpu().numpy().view(np.uint16)
    out = torch.empty(b.n, dtype=torch.int16, device=dev)
    for name, (ars, d, order) in layouts.items():
        if name in ("base", "perm"):
            got = eng.batch_tensors(ars[0], dd[name][0]).cpu().numpy().view(np.uint16)
            assert np.array_equal(got, ref[order]), name  # same packets, same results
    for _ in range(args.rounds):
        for name, (ars, d, order) in layouts.items():
            for k in range(4):
                eng.batch_tensors(ars[k % 2], dd[name][k % 2], out)
            a, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            a.record(stream)
            for k in range(args.reps):
                eng.batch_tensors(ars[k % 2], dd[name][k % 2], out)
            e.record(stream)
            torch.cuda.synchronize()
            res[name].append(a.elapsed_time(e) * 1e3 / args.reps)
    summary = {}
    for name, ts in res.items():
        med = float(np.median(ts))
        summary[name] = {"avg_us": ts, "median_us": med, "frac_of_8TBps": ab / med / 1e3 / 8000}
        print(f"{name:7s} {med:7.1f} us  {ab / med / 1e3 / 8000 * 100:5.1f}% of 8 TB/s  rounds {['%.1f' % x for x in ts]}",
              flush=True)
    if args.json:
        json.dump({"window": args.window, "algorithmic_bytes": ab,
                   "class_share": {int(c): float((cls == c).mean()) for c in (0, 1, 2)}, "variants": summary},
                  open(args.json, "w"), indent=1)


if __name__ == "__main__":
    main()
