#!/usr/bin/env python3
"""Where a launch's time goes, workgroup by workgroup: the tuning library's
csum_hyb variants stamp the time each workgroup finishes (s_memrealtime,
100 MHz; csum_kernels.hip NSK_TIMELINE, tune.hip).  A variant runs back to
back over rotated batches as bench.py times them; the stamps of the last
launch are summarised: finish percentiles, the steady rate of finishing
workgroups and the tail (how long the last 10% take against that rate).

  python tools/timeline.py --config 4 --variant prod [--rot 2] [--rot-desc]
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
sys.path.insert(0, os.path.join(ROOT, "tools"))

import torch  # noqa: E402

from netstack_amd import workloads as W  # noqa: E402
from tune import load  # noqa: E402


def summarise(fin: np.ndarray) -> dict:
    """fin: each workgroup's finish stamp (low word of s_memrealtime)."""
    f = fin.astype(np.int64)
    f = (f - f.min()) & 0xFFFFFFFF  # ticks after the first workgroup finished (10 ns)
    e = np.sort(f) * 10.0 / 1000.0  # us
    n = len(e)
    bins = np.bincount((e / 0.5).astype(np.int64))
    steady = float(np.median(bins[: max(1, len(bins) * 3 // 4)]))
    return {
        "workgroups": n,
        "finish_us_after_first": {"p10": float(e[n // 10]), "p50": float(e[n // 2]), "p90": float(e[n * 9 // 10]),
                                  "p99": float(e[n * 99 // 100]), "last": float(e[-1])},
        "tail_us": {"after_p90": float(e[-1] - e[n * 9 // 10]), "after_p99": float(e[-1] - e[n * 99 // 100])},
        "steady_finishes_per_0.5us": steady,
        # the time the last 10% would take at the steady rate, and the time it took
        "last10pct_at_steady_rate_us": 0.1 * n / max(steady, 1.0) * 0.5,
        "finishes_per_0.5us": bins.tolist(),
    }


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", type=int, default=4)
    ap.add_argument("--variant", default="prod")
    ap.add_argument("--rot", type=int, default=0)
    ap.add_argument("--rot-desc", action="store_true")
    ap.add_argument("--reps", type=int, default=20)
    ap.add_argument("--json", default="")
    args = ap.parse_args()
    L = load()
    L.nsk_tune_timeline.argtypes = [ctypes.c_void_p]
    names = [L.nsk_tune_name(v).decode() for v in range(L.nsk_tune_count())]
    v = names.index(args.variant)
    dev = torch.device("cuda", 0)
    sp = torch.cuda.current_stream(dev).cuda_stream
    rot = args.rot or {3: 4, 4: 2, 2: 2}.get(args.config, 1)
    b = W.config(args.config)
    arenas = [b.arena_device(dev)] + [W.random_bytes_torch(b.seed + 77 * r, b.arena_bytes, dev)
                                      for r in range(1, rot)]
    desc = torch.from_numpy(b.desc.view(np.uint8).copy()).to(dev)
    descs = [desc] + [desc.clone() for _ in range(1, rot)] if args.rot_desc else [desc] * rot
    out = torch.empty(b.n, dtype=torch.int16, device=dev)
    err = torch.zeros(1, dtype=torch.int64, device=dev)
    grid_max = b.n  # at least one descriptor per workgroup
    tl = torch.zeros(grid_max, dtype=torch.int32, device=dev)
    res = {}
    for rnd in range(3):
        assert L.nsk_tune_timeline(None) == 0
        for k in range(args.reps):  # back to back, rotated; stamps only on the last one
            if k == args.reps - 1:
                torch.cuda.synchronize()
                tl.zero_()
                assert L.nsk_tune_timeline(tl.data_ptr()) == 0
                for j in range(3):  # two warm launches keep the device busy into the stamped one
                    a, d = arenas[(k + j) % rot], descs[(k + j) % rot]
                    assert L.nsk_tune_launch(v, a.data_ptr(), b.arena_bytes, d.data_ptr(), b.n, out.data_ptr(),
                                             err.data_ptr(), sp) == 0
            else:
                a, d = arenas[k % rot], descs[k % rot]
                assert L.nsk_tune_launch(v, a.data_ptr(), b.arena_bytes, d.data_ptr(), b.n, out.data_ptr(),
                                         err.data_ptr(), sp) == 0
        torch.cuda.synchronize()
        assert L.nsk_tune_timeline(None) == 0
        t = tl.cpu().numpy().view(np.uint32)
        grid = int(np.count_nonzero(t))
        res[f"round{rnd}"] = summarise(t[:grid])
    r = res["round2"]
    fq = r["finish_us_after_first"]
    print(f"cfg{args.config} {args.variant}: {r['workgroups']} workgroups; finishes after the first: "
          f"p10/p50/p90/p99/last {fq['p10']:.1f}/{fq['p50']:.1f}/{fq['p90']:.1f}/{fq['p99']:.1f}/{fq['last']:.1f} us; "
          f"steady {r['steady_finishes_per_0.5us']:.0f} per 0.5 us: the last 10% took {r['tail_us']['after_p90']:.1f} us "
          f"vs {r['last10pct_at_steady_rate_us']:.1f} at that rate", flush=True)
    if args.json:
        with open(args.json, "w") as f:
            json.dump({"config": args.config, "variant": args.variant, "rot": rot, "rot_desc": args.rot_desc,
                       "rounds": res}, f, indent=1)


if __name__ == "__main__":
    main()
