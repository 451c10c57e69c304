#!/usr/bin/env python3
"""Workload for rocprofv3 --pmc passes (tools/profile.sh).

--set main (default): calibration reads of a known byte count in the product
kernel's access shapes, then the product kernel (ns_csum_batch_dev) on every
bench.py config: 2, 3, 4, 5, 7 (RX, fused table) and 8 (TX fill).  cfg3's
82 MB batch fits the 256 MiB MALL, so it runs as bench.py runs it: 4
batches with 4 descriptor tables, the measured launches each on a batch last
touched three launches earlier (over 256 MiB of other data), so FETCH_SIZE
counts HBM reads; a label `cfg3warm` covers the launches that cycle the
batches in.
--set cfg3probe: cfg3 rotated through the product's small-packet instance and
the floor kernels of tools/tune.py (libns_tune.so), for the SQ counters.

Each label covers REPS launches (of `kernels` dispatches each, default 1);
tools/pmc_parse.py maps dispatches to labels in the order printed here."""
import argparse
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


def big_share(desc) -> float:
    """Share of payload in packets csum_hyb sends to the 8-lane groups (>= 40 chunks)."""
    ln = desc["len"].astype(np.float64)
    return float(ln[desc["len"] >= 40 * 16 - 15].sum() / max(ln.sum(), 1.0))


def cfg3_rotated(dev):
    b = W.config(3)
    arenas = [b.arena_device(dev)] + [W.random_bytes_torch(b.seed + 77 * r, b.arena_bytes, dev) for r in range(1, 4)]
    t = torch.from_numpy(b.desc.view(np.uint8).copy()).to(dev)
    descs = [t] + [t.clone() for _ in range(3)]
    return b, arenas, descs


def main_set(dev, L):
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
    for cfg in (2, 4, 5):
        b = W.config(cfg)
        arena = b.arena_device(dev)
        desc = torch.from_numpy(b.desc.view(np.uint8).copy()).to(dev)
        out = torch.empty(b.n, dtype=torch.int16, device=dev)
        for _ in range(REPS):
            eng.batch_tensors(arena, desc, out)
        torch.cuda.synchronize()
        print(f"LABEL cfg{cfg} algorithmic_bytes={b.algorithmic_bytes} payload={b.payload_bytes} "
              f"arena={b.arena_bytes} n={b.n} big_share={big_share(b.desc):.4f}", flush=True)
        del arena, desc, out
        torch.cuda.empty_cache()
    b, arenas, descs = cfg3_rotated(dev)
    out = torch.empty(b.n, dtype=torch.int16, device=dev)
    for k in (1, 2, 3):  # cycle the other batches in: batch 0 is now 3 launches (>256 MiB) old
        eng.batch_tensors(arenas[k], descs[k], out)
    torch.cuda.synchronize()
    print(f"LABEL cfg3warm n={b.n}", flush=True)
    for k in (0, 1, 2):
        eng.batch_tensors(arenas[k], descs[k], out)
    torch.cuda.synchronize()
    print(f"LABEL cfg3 algorithmic_bytes={b.algorithmic_bytes} payload={b.payload_bytes} arena={b.arena_bytes} "
          f"n={b.n} big_share=0 rotated=4", flush=True)
    del arenas, descs, out
    torch.cuda.empty_cache()
    for cfg, tx in ((7, False), (8, True)):
        n = 1 << 20
        if tx:
            arena, d = W.tx_batch(n, 7000, dev, fused=True)
        else:
            arena, d, _ = W.rx_batch(n, 7000, dev, corrupt_every=1000, fused=True)
        desc = torch.from_numpy(d.view(np.uint8).copy()).to(dev)
        out = torch.empty(len(d), dtype=torch.int16, device=dev)
        for _ in range(REPS):
            eng.batch_tensors(arena, desc, out, store=tx)
        torch.cuda.synchronize()
        algo = n * W.RX_PKT + 8 * n + len(d) * 18 + (4 * n if tx else 0)  # bench.py packet_mode
        print(f"LABEL cfg{cfg} algorithmic_bytes={algo} payload={n * W.RX_PKT} arena={arena.numel()} n={len(d)} "
              f"big_share={big_share(d):.4f}", flush=True)
        del arena, desc, out
        torch.cuda.empty_cache()
    # cfg 7 as a receive ring (bench.py --rx-layout ring): ns_csum_rx_ring,
    # 8-lane groups reading whole 128-B lines (line 0 default policy, the
    # rest nontemporal): the 16-lane-group calibration shape
    n = 1 << 20
    arena, lens, _ = W.rx_ring_batch(n, 7000, dev, corrupt_every=1000)
    verdict = torch.empty(n, dtype=torch.uint8, device=dev)
    sums = torch.empty(2 * n, dtype=torch.int16, device=dev)
    for _ in range(REPS):
        eng.rx_ring(arena, dict(stride=W.RX_STRIDE, n=n), lens, sums=sums, verdict=verdict)
    torch.cuda.synchronize()
    algo = n * (W.RX_PKT + 9)  # bench.py ring_mode
    print(f"LABEL cfg7ring algorithmic_bytes={algo} payload={n * W.RX_PKT} arena={arena.numel()} n={n} "
          f"shape=calib2164", flush=True)
    del arena, lens, verdict, sums
    torch.cuda.empty_cache()
    # cfg 8 as bench.py runs it by default: sendTCPBatch's layout, NS_BATCH_PAIRED
    n = 1 << 20
    arena, _ = W.tx_split_batch(n, 7000, dev)
    d = W.tx_split_desc(n, True, paired=True)
    desc = torch.from_numpy(d.view(np.uint8).copy()).to(dev)
    out = torch.empty(len(d), dtype=torch.int16, device=dev)
    for _ in range(REPS):
        eng.batch_tensors(arena, desc, out, store=True, paired=True)
    torch.cuda.synchronize()
    algo = n * W.RX_PKT + 8 * n + len(d) * 18 + 4 * n
    print(f"LABEL cfg8split algorithmic_bytes={algo} payload={n * W.RX_PKT} arena={arena.numel()} n={len(d)} "
          f"big_share={big_share(d):.4f}", flush=True)
    del arena, desc, out
    torch.cuda.empty_cache()
    # cfg 8 as bench.py runs it by default: the same layout filled from its
    # geometry (ns_csum_tcp_tx: a payload pass and a header pass per call, so
    # 2 dispatches per launch; since round 6 the payload is read by 8-lane
    # groups, one whole 128-B line per group per instruction, nontemporal
    # past line 0: the group calibration shape)
    arena, _ = W.tx_split_batch(n, 7000, dev)
    geo = W.tx_struct_geometry(n)
    for _ in range(REPS):
        eng.tcp_tx(arena, geo)
    torch.cuda.synchronize()
    algo = n * W.RX_PKT + 4 * n
    print(f"LABEL cfg8struct algorithmic_bytes={algo} payload={n * W.RX_PKT} arena={arena.numel()} n={n} "
          f"kernels=2 shape=calib2164", flush=True)
    del arena
    torch.cuda.empty_cache()


def rx_set(dev, L):
    """The receive paths only: the 16-lane-group calibration read, cfg7 as a
    fused descriptor table and cfg7 as a ring (ns_csum_rx_ring)."""
    sp = torch.cuda.current_stream(dev).cuda_stream
    buf = torch.ones(CAL_BYTES, dtype=torch.uint8, device=dev)
    outb = torch.zeros(65536, dtype=torch.int32, device=dev)
    for _ in range(REPS):
        assert L.nsk_calib_launch(2164, buf.data_ptr(), CAL_BYTES, outb.data_ptr(), 8192, sp) == 0
    torch.cuda.synchronize()
    print(f"LABEL calib2164 bytes={CAL_BYTES}", flush=True)
    del buf
    eng = Engine(0)
    n = 1 << 20
    arena, d, _ = W.rx_batch(n, 7000, dev, corrupt_every=1000, fused=True)
    desc = torch.from_numpy(d.view(np.uint8).copy()).to(dev)
    out = torch.empty(len(d), dtype=torch.int16, device=dev)
    for _ in range(REPS):
        eng.batch_tensors(arena, desc, out)
    torch.cuda.synchronize()
    algo = n * W.RX_PKT + 8 * n + len(d) * 18
    print(f"LABEL cfg7 algorithmic_bytes={algo} payload={n * W.RX_PKT} arena={arena.numel()} n={len(d)} "
          f"big_share={big_share(d):.4f}", flush=True)
    del arena, desc, out
    torch.cuda.empty_cache()
    arena, lens, _ = W.rx_ring_batch(n, 7000, dev, corrupt_every=1000)
    verdict = torch.empty(n, dtype=torch.uint8, device=dev)
    sums = torch.empty(2 * n, dtype=torch.int16, device=dev)
    for _ in range(REPS):
        eng.rx_ring(arena, dict(stride=W.RX_STRIDE, n=n), lens, sums=sums, verdict=verdict)
    torch.cuda.synchronize()
    print(f"LABEL cfg7ring algorithmic_bytes={n * (W.RX_PKT + 9)} payload={n * W.RX_PKT} arena={arena.numel()} "
          f"n={n} shape=calib2164", flush=True)
    # the same frames through a buffer list (bench.py --rx-layout bufs), in
    # ring order and shuffled: the offset table adds 4 B per packet
    for order in ("ring", "shuffled"):
        perm = np.random.default_rng(7000).permutation(n) if order == "shuffled" else np.arange(n)
        offs = torch.from_numpy((perm.astype(np.int64) * W.RX_STRIDE).astype(np.int32)).to(dev)
        ln = lens[torch.from_numpy(perm).to(dev)].contiguous()
        for _ in range(REPS):
            eng.rx_bufs(arena, dict(stride=W.RX_STRIDE, n=n), offs, ln, sums=sums, verdict=verdict)
        torch.cuda.synchronize()
        print(f"LABEL cfg7bufs_{order} algorithmic_bytes={n * (W.RX_PKT + 13)} payload={n * W.RX_PKT} "
              f"arena={arena.numel()} n={n} shape=calib2164", flush=True)


def cfg4probe_set(dev, L):
    """cfg4 as the bench runs it (2 rotating arenas and tables), its two
    packet classes alone (the other class's lengths set to 0, the arena
    unchanged: tools/cfg4_split.py), cfg2 rotated, and the calibration reads
    in the two access shapes cfg4's kernel uses (8-lane nontemporal groups,
    calib2164; per-lane runs of 4 chunks, calib400): which counter per byte
    separates cfg4 from a byte-weighted mix of the two reads.
    Each variant: REPS launches to cycle the arenas in (label _warm), then
    REPS measured, alternating arenas (batch k's table with arena k)."""
    sp = torch.cuda.current_stream(dev).cuda_stream
    buf = torch.ones(CAL_BYTES, dtype=torch.uint8, device=dev)
    outb = torch.zeros(65536, dtype=torch.int32, device=dev)
    for mode in (400, 2164):
        for _ in range(REPS):
            assert L.nsk_calib_launch(mode, buf.data_ptr(), CAL_BYTES, outb.data_ptr(), 8192, sp) == 0
        torch.cuda.synchronize()
        print(f"LABEL calib{mode} bytes={CAL_BYTES}", flush=True)
    del buf
    torch.cuda.empty_cache()
    eng = Engine(0)
    for cfg in (2, 4):
        b = W.config(cfg)
        arenas = [b.arena_device(dev), W.random_bytes_torch(b.seed + 77, b.arena_bytes, dev)]
        a = b.desc["off"] & np.uint64(15)
        nch = ((a + b.desc["len"].astype(np.uint64) - np.uint64(1)) >> np.uint64(4)) + np.uint64(1)
        big = nch >= 40
        variants = [("all", np.ones(b.n, bool))] + ([("big", big), ("small", ~big)] if cfg == 4 else [])
        out = torch.empty(b.n, dtype=torch.int16, device=dev)
        for name, keep in variants:
            d = b.desc.copy()
            d["len"] = np.where(keep, d["len"], 0)
            t = torch.from_numpy(d.view(np.uint8).copy()).to(dev)
            ts = [t, t.clone()]
            for k in range(REPS):  # cycle in (tools/pmc_parse.py matches REPS dispatches per label)
                eng.batch_tensors(arenas[(k + 1) % 2], ts[(k + 1) % 2], out)
            torch.cuda.synchronize()
            print(f"LABEL cfg{cfg}_{name}_warm n={b.n}", flush=True)
            for k in range(REPS):
                eng.batch_tensors(arenas[k % 2], ts[k % 2], out)
            torch.cuda.synchronize()
            payload = int(d["len"].sum(dtype=np.uint64))
            share = float(d["len"][big].sum(dtype=np.uint64)) / max(payload, 1)
            print(f"LABEL cfg{cfg}_{name} algorithmic_bytes={payload + 18 * b.n} payload={payload} "
                  f"arena={b.arena_bytes} n={b.n} big_share={share:.4f} rotated=2", flush=True)
        del arenas, out
        torch.cuda.empty_cache()


def cfg3probe_set(dev, L):
    names = [L.nsk_tune_name(v).decode() for v in range(L.nsk_tune_count())]
    sp = torch.cuda.current_stream(dev).cuda_stream
    b, arenas, descs = cfg3_rotated(dev)
    out = torch.empty(b.n, dtype=torch.int16, device=dev)
    err = torch.zeros(1, dtype=torch.int64, device=dev)
    for name in ("small_wg64_spec", "small_wg64", "floor_quad_nt_wg64", "floor_quad_nt", "quad_direct_nt_wg64"):
        v = names.index(name)
        for k in (1, 2, 3, 0, 1, 2):  # three to cycle in, three measured (see cfg3warm above)
            assert L.nsk_tune_launch(v, arenas[k].data_ptr(), b.arena_bytes, descs[k].data_ptr(), b.n,
                                     out.data_ptr(), err.data_ptr(), sp) == 0
            if k == 3:
                torch.cuda.synchronize()
                print(f"LABEL {name}_warm n={b.n}", flush=True)
        torch.cuda.synchronize()
        print(f"LABEL {name} algorithmic_bytes={b.algorithmic_bytes} n={b.n} rotated=4", flush=True)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--set", default="main", choices=("main", "cfg3probe", "rx", "cfg4probe"))
    args = ap.parse_args()
    L = ctypes.CDLL(os.path.join(ROOT, "netstack_amd", "lib", "libns_tune.so"))
    L.nsk_calib_launch.argtypes = [ctypes.c_int, ctypes.c_void_p, ctypes.c_uint64, ctypes.c_void_p,
                                   ctypes.c_uint32, ctypes.c_void_p]
    L.nsk_tune_count.restype = ctypes.c_int
    L.nsk_tune_name.restype = ctypes.c_char_p
    L.nsk_tune_name.argtypes = [ctypes.c_int]
    L.nsk_tune_launch.restype = ctypes.c_int
    L.nsk_tune_launch.argtypes = [ctypes.c_int, ctypes.c_void_p, ctypes.c_uint64, ctypes.c_void_p,
                                  ctypes.c_uint32, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p]
    dev = torch.device("cuda", 0)
    if args.set == "main":
        main_set(dev, L)
    elif args.set == "rx":
        rx_set(dev, L)
    elif args.set == "cfg4probe":
        cfg4probe_set(dev, L)
    else:
        cfg3probe_set(dev, L)


if __name__ == "__main__":
    main()
