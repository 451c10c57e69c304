#!/usr/bin/env python3
"""cfg4's time by packet class: the production kernel (ns_csum_batch_dev) on
the Zipf batch as bench.py runs it (2 rotating arenas and tables, back to
back), then on the same table with the packets of one class given length 0
(the arena unchanged, so the other class's packets sit where they were):
  all    — the batch;
  big    — only packets of >= 40 chunks (the 8-lane groups + their edge runs);
  small  — only packets of < 40 chunks (the lane runs).
Bytes per variant are the packets' own bytes + 18 B per descriptor.

  python tools/cfg4_split.py [--rounds 5] [--reps 20]
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


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rounds", type=int, default=5)
    ap.add_argument("--reps", type=int, default=20)
    ap.add_argument("--json", default="")
    args = ap.parse_args()
    dev = torch.device("cuda", 0)
    stream = torch.cuda.current_stream(dev)
    eng = Engine(0)
    b = W.config(4)
    a = b.desc["off"] & np.uint64(15)
    nch = ((a + b.desc["len"].astype(np.uint64) - np.uint64(1)) >> np.uint64(4)) + np.uint64(1)
    big = nch >= 40
    arenas = [b.arena_device(dev), W.random_bytes_torch(b.seed + 77, b.arena_bytes, dev)]
    tables = {}
    for name, keep in (("all", np.ones(b.n, bool)), ("big", big), ("small", ~big)):
        d = b.desc.copy()
        d["len"] = np.where(keep, d["len"], 0)
        t = torch.from_numpy(d.view(np.uint8).copy()).to(dev)
        tables[name] = ([t, t.clone()], int(d["len"].sum(dtype=np.uint64)) + 18 * b.n)
    out = torch.empty(b.n, dtype=torch.int16, device=dev)
    res = {k: [] for k in tables}
    for _ in range(args.rounds):
        for name, (ts, _) in tables.items():
            for k in range(4):
                eng.batch_tensors(arenas[k % 2], ts[k % 2], out)
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record(stream)
            for k in range(args.reps):
                eng.batch_tensors(arenas[k % 2], ts[k % 2], out)
            e1.record(stream)
            torch.cuda.synchronize()
            res[name].append(e0.elapsed_time(e1) * 1e3 / args.reps)
    summary = {}
    for name, ts in res.items():
        med = float(np.median(ts))
        by = tables[name][1]
        summary[name] = {"median_us": med, "bytes": by, "frac_of_8TBps": by / med / 1e3 / 8000, "rounds_us": ts}
        print(f"{name:6s} {med:7.1f} us  {by / 1e6:7.1f} MB  {by / med / 1e3 / 8000 * 100:5.1f}% of 8 TB/s", flush=True)
    if args.json:
        json.dump({"big_share_of_payload": float(b.desc["len"][big].sum() / b.desc["len"].sum()), "variants": summary},
                  open(args.json, "w"), indent=1)


if __name__ == "__main__":
    main()
