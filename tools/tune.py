#!/usr/bin/env python3
"""A/B the checksum kernel variants of libns_tune.so in ONE process,
interleaved rounds (cdna_hip_programming.md §5.4 rule 24), on the
BASELINE.json layouts; every variant is parity-checked against the product
kernel's results.  Also times the read-stream calibration kernels.

  python tools/tune.py [--configs 2,3,4] [--rounds 5] [--reps 10] [--variants all]
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

import torch  # noqa: E402  (load torch's HIP runtime first)

from netstack_amd import Engine  # noqa: E402
from netstack_amd import workloads as W  # noqa: E402

TUNE = os.path.join(ROOT, "netstack_amd", "lib", "libns_tune.so")


def load(path=TUNE):
    L = ctypes.CDLL(path)
    L.nsk_tune_count.restype = ctypes.c_int
    L.nsk_tune_name.restype = ctypes.c_char_p
    L.nsk_tune_name.argtypes = [ctypes.c_int]
    L.nsk_tune_launch.restype = ctypes.c_int
    L.nsk_tune_launch.argtypes = [ctypes.c_int, ctypes.c_void_p, ctypes.c_uint64, ctypes.c_void_p,
                                  ctypes.c_uint32, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p]
    if not hasattr(L, "nsk_calib_launch"):  # the small A/B library (tune_ab.hip)
        return L
    L.nsk_calib_launch.restype = ctypes.c_int
    L.nsk_calib_launch.argtypes = [ctypes.c_int, ctypes.c_void_p, ctypes.c_uint64, ctypes.c_void_p,
                                   ctypes.c_uint32, ctypes.c_void_p]
    return L


B2B = {"on": False}


def time_launches(fn, reps, stream):
    """Per-launch event pairs; with --b2b, ONE event pair around `reps`
    back-to-back launches (the way bench.py times them: sustained load, where
    power management can lower the clock) and the average per launch."""
    if B2B["on"]:
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record(stream)
        for _ in range(reps):
            fn()
        b.record(stream)
        torch.cuda.synchronize()
        return [a.elapsed_time(b) * 1e3 / reps]
    ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(reps)]
    for a, b in ev:
        a.record(stream)
        fn()
        b.record(stream)
    torch.cuda.synchronize()
    return [a.elapsed_time(b) * 1e3 for a, b in ev]  # us


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--configs", default="2,3,4")
    ap.add_argument("--rounds", type=int, default=5)
    ap.add_argument("--reps", type=int, default=10)
    ap.add_argument("--variants", default="all")
    ap.add_argument("--calib", action="store_true")
    ap.add_argument("--calib-modes", default="2,4,5,6")
    ap.add_argument("--calib-blocks", default="4096,8192,16384")
    ap.add_argument("--json", default="")
    ap.add_argument("--lib", default=TUNE, help="tuning library (e.g. netstack_amd/lib/libns_tune_ab.so)")
    ap.add_argument("--b2b", action="store_true", help="time back-to-back launches (as bench.py does)")
    ap.add_argument("--rot", type=int, default=0, help="distinct arenas cycled (0: 4 for cfg3, else 1)")
    ap.add_argument("--rot-desc", action="store_true",
                    help="rotate copies of the descriptor table with the arenas (cold tables, as bench.py)")
    ap.add_argument("--n", default="", help="packet counts per config, e.g. 2:2097152")
    args = ap.parse_args()

    L = load(args.lib)
    B2B["on"] = args.b2b
    names = [L.nsk_tune_name(v).decode() for v in range(L.nsk_tune_count())]
    sel = list(range(len(names))) if args.variants == "all" else \
        [names.index(x) for x in args.variants.split(",")]
    dev = torch.device("cuda", 0)
    stream = torch.cuda.current_stream(dev)
    sp = stream.cuda_stream
    eng = Engine(0)
    err = torch.zeros(1, dtype=torch.int64, device=dev)
    report = {"variants": {}, "calib": {}}

    nover = dict((int(k), int(v)) for k, v in (x.split(":") for x in args.n.split(",") if x))
    for cfg in [int(c) for c in args.configs.split(",")]:
        rot = args.rot or (4 if cfg == 3 else 1)
        if cfg == 7:  # bench.py --config 7's RX batch, timed unchained (the main kernel)
            a7, d7, _ = W.rx_batch(nover.get(7, 1 << 20), 7000, dev)
            b = W.Batch("rx_1Mx1500_3desc", 7000, d7, a7.numel())
            arenas = [a7]
        elif cfg in (10, 11, 12):  # mixed shapes: Zipf 64-600 B; half 64-B ACKs, half 1460-B segments (by
            # count); Zipf 200-1000 B
            n = nover.get(cfg, {10: 1 << 22, 11: 1 << 21, 12: 1 << 22}[cfg])
            if cfg == 10:
                ln = W.zipf_lengths(10, n, 64, 600)
            elif cfg == 12:
                ln = W.zipf_lengths(12, n, 200, 1000)
            else:
                ln = np.where(W.splitmix64(11, n) & np.uint64(1), 1460, 64).astype(np.uint32)
            d, end = W.make_desc(ln, W._initials(cfg, n), 16)
            b = W.Batch(f"mix{cfg}", cfg, d, ((end + 15) // 16) * 16)
            arenas = [b.arena_device(dev)] + [W.random_bytes_torch(b.seed + 77 * r, b.arena_bytes, dev)
                                              for r in range(1, rot)]
        elif cfg in (13, 14):  # receive rings: 512-B slots holding Zipf 64-512 B; 256-B slots, 128-256 B
            slot = 512 if cfg == 13 else 256
            n = nover.get(cfg, 1_572_864_000 // slot)
            ln = W.zipf_lengths(cfg, n, 64, 512) if cfg == 13 else \
                (128 + (W.splitmix64(cfg, n) % np.uint64(129))).astype(np.uint32)
            d = np.zeros(n, dtype=W.DESC_DTYPE)
            d["off"] = np.arange(n, dtype=np.uint64) * np.uint64(slot)
            d["len"] = ln
            d["initial"] = W._initials(cfg, n)
            b = W.Batch(f"ring{slot}", cfg, d, n * slot)
            arenas = [b.arena_device(dev)] + [W.random_bytes_torch(b.seed + 77 * r, b.arena_bytes, dev)
                                              for r in range(1, rot)]
        elif cfg >= 100:  # uniform packets of `cfg` bytes, 1.5 GB of payload (TP-rule sweeps)
            b = W.uniform(f"uniform_{cfg}B", 9000 + cfg, nover.get(cfg, (1_572_864_000 // cfg)), cfg)
            arenas = [b.arena_device(dev)] + [W.random_bytes_torch(b.seed + 77 * r, b.arena_bytes, dev)
                                              for r in range(1, rot)]
        else:
            b = W.config(cfg, nover.get(cfg))
            arenas = [b.arena_device(dev)] + [W.random_bytes_torch(b.seed + 77 * r, b.arena_bytes, dev)
                                              for r in range(1, rot)]
        desc = torch.from_numpy(b.desc.view(np.uint8).copy()).to(dev)
        descs = [desc] + [desc.clone() for _ in range(1, rot)] if args.rot_desc else [desc] * rot
        ref = eng.batch_tensors(arenas[0], desc)
        torch.cuda.synchronize()
        ref = ref.cpu()
        out = torch.empty(b.n, dtype=torch.int16, device=dev)
        ab = b.algorithmic_bytes
        res = {v: [] for v in sel}
        state = {"k": 0}

        def launcher(v):
            def f():
                a = arenas[state["k"] % rot]
                dd = descs[state["k"] % rot]
                state["k"] += 1
                rc = L.nsk_tune_launch(v, a.data_ptr(), b.arena_bytes, dd.data_ptr(), b.n,
                                       out.data_ptr(), err.data_ptr(), sp)
                assert rc == 0
            return f

        for v in sel:  # warm + parity
            f = launcher(v)
            state["k"] = 0
            f()
            torch.cuda.synchronize()
            ok = torch.equal(out.cpu(), ref) or names[v].startswith("chained_main")
            if not ok:
                print(f"PARITY FAIL cfg{cfg} {names[v]}", flush=True)
            for _ in range(2):
                f()
        for r in range(args.rounds):
            for v in sel:
                res[v] += time_launches(launcher(v), args.reps, stream)
        print(f"== cfg{cfg} {b.name}: n={b.n} algorithmic={ab/1e6:.1f} MB", flush=True)
        rows = []
        for v in sel:
            med = float(np.median(res[v]))
            rows.append((med, names[v], float(np.min(res[v]))))
            report["variants"].setdefault(f"cfg{cfg}", {})[names[v]] = {
                "median_us": med, "min_us": float(np.min(res[v])), "GBps": ab / med / 1e3}
        for med, nm, mn in sorted(rows):
            print(f"  {nm:16s} median {med:9.1f} us  min {mn:9.1f}  -> {ab / med / 1e3:7.0f} GB/s "
                  f"({ab / med / 1e3 / 8000 * 100:5.1f}% of 8 TB/s)", flush=True)
        del arenas

    if args.calib:
        nbytes = (1 << 31) - 4096  # ~2 GiB, well past the 256 MiB MALL
        buf = torch.empty(nbytes, dtype=torch.uint8, device=dev)
        buf.fill_(1)
        outb = torch.zeros(65536, dtype=torch.int32, device=dev)
        for mode in [int(x) for x in args.calib_modes.split(",")]:
            for blocks in [int(x) for x in args.calib_blocks.split(",")]:
                f = lambda: L.nsk_calib_launch(mode, buf.data_ptr(), nbytes, outb.data_ptr(), blocks, sp)
                f()
                ts = []
                for _ in range(args.rounds):
                    ts += time_launches(f, args.reps, stream)
                med = float(np.median(ts))
                report["calib"][f"mode{mode}_b{blocks}"] = {"median_us": med, "GBps": nbytes / med / 1e3}
                print(f"  calib mode {mode:2d} blocks {blocks:5d}: {med:9.1f} us  {nbytes / med / 1e3:7.0f} GB/s",
                      flush=True)
    if args.json:
        with open(args.json, "w") as f:
            json.dump(report, f, indent=1)


if __name__ == "__main__":
    main()
