#!/usr/bin/env python3
"""bench.py — device-resident checksum throughput of netstack's RFC 1071 hot
path on MI355X, against the HBM roofline, with the scalar CPU port timed
beside it.

  python bench.py [--gpus N] [--steps K] [--warmup W] [--config 1|2|3|4|5|7|8] [--mode dev|host]

One step = one pass of the checksum engine (ns_csum_batch_dev) over one batch
already resident in HBM.  Default workload = BASELINE.json configs[1]:
1,048,576 x 1500 B TCP payloads per GPU (weak scaling: every rank owns its
own 1M-packet batch, so at N = 8 the job is configs[4]'s 8M x 1500 B, no
collective on the data path).  value = Σ payload bytes of all ranks x K / max
over ranks of the timed wall time, in GiB/s (2^30 B).

For N > 1 launch with
  python -m torch.distributed.run --nnodes=1 --nproc-per-node N \
      --master-addr 127.0.0.1 --master-port P bench.py --gpus N ...
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

METRIC = "checksum GiB/s device-resident (batched MTU pkts), 1/2/4/8 GPU vs HBM roofline"
HBM_PEAK_GBS = 8000.0  # MI355X_MICROARCH.md: 8.0 TB/s spec
GIB = float(1 << 30)

WORKLOADS = {
    1: "cfg1: one 65,536-B buffer, seed 1, initial 0: header.Checksum (BASELINE.json configs[0])",
    2: "cfg2: 1,048,576 x 1500 B TCP payloads per GPU, 16-B-aligned starts (BASELINE.json configs[1])",
    3: "cfg3: 1,048,576 x 64 B min-size packets per GPU, 4 rotating batches (BASELINE.json configs[2])",
    4: "cfg4: 1,048,576 Zipf(1.1) 64-9000 B packets per GPU (BASELINE.json configs[3])",
    5: "cfg5: 8,388,608 x 1500 B packets in total, one contiguous shard of 8M/N per GPU "
       "(BASELINE.json configs[4], strong scaling)",
}


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=50)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--config", type=int, default=2, choices=(1, 2, 3, 4, 5, 7, 8),
                    help="BASELINE.json configs[k-1]; 7 = device-resident RX verification, "
                         "8 = device-resident TX checksum fill (SURVEY §8(f) ranks 2 and 1)")
    ap.add_argument("--mode", default="dev", choices=("dev", "host"))
    ap.add_argument("--rx-layout", default="fused", choices=("fused", "chained", "ring", "bufs"),
                    help="--config 7 (and 8 with --tx-layout wire) descriptor table: 2 independent descriptors "
                         "per packet, or 3 chained; --config 7 ring: no table, a receive ring parsed and verified "
                         "on the device (ns_csum_rx_ring)")
    ap.add_argument("--tx-layout", default="struct", choices=("struct", "split", "wire"),
                    help="--config 8 packets: as sendTCPBatch builds them (header slots + payload view) "
                         "filled from the batch geometry by ns_csum_tcp_tx (struct) or through an "
                         "NS_BATCH_PAIRED descriptor table (split), or wire-contiguous like config 7")
    ap.add_argument("--bufs-order", default="shuffled", choices=("shuffled", "ring"),
                    help="--rx-layout bufs: buffers handed over in shuffled order, or in ring order")
    ap.add_argument("--bufs-stride", type=int, default=0,
                    help="--rx-layout ring / bufs: slot or buffer spacing (a multiple of 16 >= 1504; 0: 1504)")
    ap.add_argument("--tx-calls", type=int, default=1,
                    help="--mode host --config 8: the 1M segments as this many sendTCPBatch calls in one "
                         "ns_csum_tcp_tx_host (23832: one per 64 KiB GSO write)")
    ap.add_argument("--rotate", type=int, default=0,
                    help="distinct batches cycled per step (0 = auto: enough to exceed the 256 MiB MALL)")
    ap.add_argument("--cpu-seconds", type=float, default=10.0, help="CPU-baseline time budget")
    ap.add_argument("--cpu-threads", type=int, default=0, help="threads for the multi-core CPU figure")
    ap.add_argument("--no-cpu", action="store_true", help="skip the CPU-baseline leg (rank 0)")
    ap.add_argument("--no-parity", action="store_true", help="skip every rank's parity sample")
    ap.add_argument("--dist-backend", default="auto", choices=("auto", "nccl", "gloo"),
                    help="control-plane backend for N > 1 (auto: nccl = RCCL on a GPU box); gloo lets "
                         "several ranks share one GPU (RCCL refuses two ranks on one device)")
    ap.add_argument("--pmc-json", default=os.path.join(ROOT, "profiles", "pmc_traffic.json"))
    args = ap.parse_args()
    if args.steps < 1 or args.warmup < 0:
        ap.error("--steps must be >= 1 and --warmup >= 0")
    return args


# ---------------------------------------------------------------------------
# distributed plumbing (also exercised by tests/test_bench_dist.py on gloo)
# ---------------------------------------------------------------------------
class Dist:
    def __init__(self, backend: str | None, device_index: int | None = None):
        """`device_index`: this rank's GPU, already made current; with nccl
        (RCCL) it is bound to the process group, so the barrier runs on it
        rather than on a device RCCL guesses from the rank."""
        import torch.distributed as dist

        self.dist = dist
        self.backend = backend
        self.device_index = device_index if backend == "nccl" else None
        self.world = int(os.environ.get("WORLD_SIZE", "1"))
        self.rank = int(os.environ.get("RANK", "0"))
        self.local = int(os.environ.get("LOCAL_RANK", "0"))
        self.on = self.world > 1
        if self.on and not dist.is_initialized():
            if self.device_index is not None:
                import torch

                dist.init_process_group(backend=backend, device_id=torch.device("cuda", self.device_index))
            else:
                dist.init_process_group(backend=backend)

    def barrier(self):
        if self.on:
            if self.device_index is not None:
                self.dist.barrier(device_ids=[self.device_index])
            else:
                self.dist.barrier()

    def max(self, x: float, device=None) -> float:
        if not self.on:
            return x
        import torch

        t = torch.tensor([x], dtype=torch.float64, device=device if self.backend == "nccl" else "cpu")
        self.dist.all_reduce(t, op=self.dist.ReduceOp.MAX)
        return float(t.item())

    def sum(self, x: float, device=None) -> float:
        if not self.on:
            return x
        import torch

        t = torch.tensor([x], dtype=torch.float64, device=device if self.backend == "nccl" else "cpu")
        self.dist.all_reduce(t, op=self.dist.ReduceOp.SUM)
        return float(t.item())

    def close(self):
        if self.on and self.dist.is_initialized():
            self.dist.destroy_process_group()


def timed_region(step, sync, dist: Dist, steps: int, warmup: int, device=None):
    """W untimed steps, then exactly K timed steps bracketed by barrier +
    device sync on both sides; returns (max-over-ranks seconds, local s)."""
    for _ in range(warmup):
        step()
    sync()
    dist.barrier()
    sync()
    t0 = time.perf_counter()
    for _ in range(steps):
        step()
    sync()
    dist.barrier()
    t1 = time.perf_counter()
    local = t1 - t0
    return dist.max(local, device), local


CALIB_BLOCKS = 16384


def b2b_us(launch, stream, reps: int = 20, warm: int = 3) -> float:
    """Average microseconds per launch over `reps` back-to-back launches
    (launch(k) for k = 0..reps-1), timed by one HIP event pair on the launch
    stream — the method of the timed region."""
    import torch

    for k in range(warm):
        launch(k)
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record(stream)
    for k in range(reps):
        launch(k)
    b.record(stream)
    torch.cuda.synchronize()
    return a.elapsed_time(b) * 1e3 / reps


def pipelined(eng, arenas, descs, n: int, algo_bytes: int, ref_out, stream, nstreams: int = 2, reps: int = 40):
    """A stream of independent batches the way a caller pipelines them:
    launch k on stream k % nstreams, each stream with its own results, so one
    batch's ramp-up overlaps the previous one's tail instead of following its
    dependent-launch boundary.  Measured after the timed region, like
    `unrotated`; the headline and the roofline stay the one-stream kernel
    time.  Returns microseconds per batch over `reps` launches between two
    events that bracket every stream, and whether each stream's results for
    batch 0 equal the timed region's (`ref_out`)."""
    import torch

    dev = ref_out.device
    ss = [stream] + [torch.cuda.Stream(dev) for _ in range(nstreams - 1)]
    outs = [torch.empty(n, dtype=torch.int16, device=dev) for _ in ss]
    rot = len(arenas)

    def run(count):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        torch.cuda.synchronize()
        e0.record(stream)
        for s in ss[1:]:
            s.wait_event(e0)
        for k in range(count):
            eng.batch_tensors(arenas[k % rot], descs[k % rot], outs[k % nstreams], stream=ss[k % nstreams])
        for s in ss[1:]:
            stream.wait_stream(s)
        e1.record(stream)
        torch.cuda.synchronize()
        return e0.elapsed_time(e1) * 1e3 / count

    run(2 * nstreams)
    us = min(run(reps), run(reps))
    for j, s in enumerate(ss):
        eng.batch_tensors(arenas[0], descs[0], outs[j], stream=s)
    torch.cuda.synchronize()
    exact = all(torch.equal(o, ref_out) for o in outs)
    return {"streams": nstreams, "batches": reps, "us_per_batch": us,
            "frac": algo_bytes / us / 1e3 / HBM_PEAK_GBS, "bit_exact_vs_timed": exact,
            "note": ("independent batches round-robin over streams (a caller's pipeline), best of two runs "
                     "after the timed region; not the headline, which is one stream")}


def launch_stats(launch, stream, reps: int = 20):
    """SURVEY §8(d)'s per-launch view, measured after the timed region: `reps`
    launches each bracketed by its own HIP event pair on the launch stream
    (3 warm-ups first); returns sorted per-launch microseconds."""
    import torch

    for _ in range(3):
        launch()
    ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(reps)]
    for a, b in ev:
        a.record(stream)
        launch()
        b.record(stream)
    torch.cuda.synchronize()
    return sorted(a.elapsed_time(b) * 1e3 for a, b in ev)


# Pure-read calibrations (libns_tune.so, not product code), each cycled over
# the same rotated arenas as the timed region: nsk::calib_tile_x, the
# checksum kernel's own big-packet access shape (lane groups of 8 with 16
# nontemporal buffer_load_dwordx4 in flight, or 16 x 8; one run of `lpr`
# whole 128-B lines per group; a non-persistent grid of contiguous tiles;
# `lds` bytes of LDS per workgroup cap its residency) with no descriptors and
# no arithmetic.  These are the fastest shapes of the sweep in
# tools/calib_sweep.py (profiles/r02/calib_sweep.txt).
CALIB_TILE = (("g8u16_lpr11_lds1k", 0, 11, 1024), ("g8u16_lpr11_lds9k", 0, 11, 9600),
              ("g16u8_lpr11_lds1k", 3, 11, 1024), ("g16u8_lpr11_lds9k", 3, 11, 9600),
              ("g8u16_lpr16_lds9k", 0, 16, 9600))


def stream_calibration(arenas, stream, reps: int = 40):
    """Same-run read-stream calibration: pure-read kernels over
    the same arena bytes, rotated like the timed region, back-to-back
    average of `reps` launches each, best of two rounds.  Returns
    {"variants": {...}, "best": ..., "GBps": ...}; None when the tuning
    library is absent."""
    import ctypes

    path = os.path.join(ROOT, "netstack_amd", "lib", "libns_tune.so")
    if not os.path.exists(path):
        return None
    import torch

    L = ctypes.CDLL(path)
    L.nsk_calib_tile_x_launch.restype = ctypes.c_int
    L.nsk_calib_tile_x_launch.argtypes = [ctypes.c_int, ctypes.c_void_p, ctypes.c_uint64, ctypes.c_uint32,
                                          ctypes.c_uint32, ctypes.c_uint32, ctypes.c_void_p,
                                          ctypes.POINTER(ctypes.c_uint64), ctypes.c_void_p]
    outb = torch.zeros(CALIB_BLOCKS, dtype=torch.int32, device=arenas[0].device)
    R = len(arenas)
    variants = {}
    for rnd in range(2):
        for name, mode, lpr, lds in CALIB_TILE:
            rb = ctypes.c_uint64(0)

            def launch(k, mode=mode, lpr=lpr, lds=lds, rb=rb):
                a = arenas[k % R]
                rc = L.nsk_calib_tile_x_launch(mode, a.data_ptr(), a.numel(), lpr, 0, lds, outb.data_ptr(),
                                               ctypes.byref(rb), stream.cuda_stream)
                if rc != 0:
                    raise RuntimeError(f"calibration {name} failed: {rc}")

            us = b2b_us(launch, stream, reps=reps)
            v = {"bytes": int(rb.value), "avg_us": us, "GBps": rb.value / us / 1e3}
            if name not in variants or v["GBps"] > variants[name]["GBps"]:
                variants[name] = v
    best = max(variants, key=lambda k: variants[k]["GBps"])
    return {"what": "pure nontemporal reads of the same rotated arenas in the checksum kernel's big-packet "
                    "shape (nsk::calib_tile_x, libns_tune.so), back-to-back average, best of 2 rounds",
            "variants": variants, "best": best, "GBps": variants[best]["GBps"]}


def floor_calibration(arenas, descs, batch, stream, reps: int = 40):
    """cfg3's same-run ceiling: tools/tune.py's floor kernels for the 1M x 64 B
    layout (floor_quad_nt at 64- and 256-thread workgroups: the quad-lane
    nontemporal loads of the product's small-packet path, the descriptors
    read and the results written, but no payload load waits for its
    descriptor), rotated like the timed region, best of two rounds.  Their
    GB/s counts the same algorithmic bytes as the checksum kernel's."""
    import ctypes

    path = os.path.join(ROOT, "netstack_amd", "lib", "libns_tune.so")
    if not os.path.exists(path):
        return None
    import torch

    L = ctypes.CDLL(path)
    L.nsk_tune_count.restype = ctypes.c_int
    L.nsk_tune_name.restype = ctypes.c_char_p
    L.nsk_tune_name.argtypes = [ctypes.c_int]
    L.nsk_tune_launch.restype = ctypes.c_int
    L.nsk_tune_launch.argtypes = [ctypes.c_int, ctypes.c_void_p, ctypes.c_uint64, ctypes.c_void_p, ctypes.c_uint32,
                                  ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p]
    names = [L.nsk_tune_name(v).decode() for v in range(L.nsk_tune_count())]
    out = torch.empty(batch.n, dtype=torch.int16, device=arenas[0].device)
    err = torch.zeros(1, dtype=torch.int64, device=arenas[0].device)
    R = len(arenas)
    variants = {}
    for _ in range(2):
        for name in ("floor_quad_nt_wg64", "floor_quad_nt"):
            v = names.index(name)

            def launch(k, v=v):
                rc = L.nsk_tune_launch(v, arenas[k % R].data_ptr(), batch.arena_bytes, descs[k % R].data_ptr(),
                                       batch.n, out.data_ptr(), err.data_ptr(), stream.cuda_stream)
                if rc != 0:
                    raise RuntimeError(f"calibration {name} failed: {rc}")

            us = b2b_us(launch, stream, reps=reps)
            g = batch.algorithmic_bytes / us / 1e3
            if name not in variants or g > variants[name]["GBps"]:
                variants[name] = {"avg_us": us, "GBps": g}
    best = max(variants, key=lambda k: variants[k]["GBps"])
    return {"what": "cfg3 floor kernels (libns_tune.so floor_quad_nt): the product's quad-lane access with "
                    "no descriptor -> payload dependency, same rotated batches, back-to-back average, best of 2",
            "variants": variants, "best": best, "GBps": variants[best]["GBps"]}


def pmc_traffic(path: str, cfg):
    """roofline.traffic: HBM bytes per launch (reads + writes) of this config's
    kernel from the committed rocprofv3 --pmc summary (tools/make_traffic.py),
    and where they come from — counters are taken in passes of their own,
    never in the timed run."""
    try:
        pm = json.load(open(path))
    except (OSError, ValueError):
        return None, None
    e = pm.get(f"cfg{cfg}", {})
    if e.get("hbm_bytes_per_launch") is None:
        return None, None
    src = (f"{os.path.relpath(path, ROOT)} ({pm.get('_round', '?')}): rocprofv3 --pmc FETCH_SIZE + WRITE_SIZE "
           f"of {e.get('kernel', '?')[:60]}, calibrated, per launch; ratio to algorithmic "
           f"{(e['hbm_bytes_per_launch'] + e.get('write_bytes', 0.0)) / e['algorithmic_bytes']:.3f}")
    return e["hbm_bytes_per_launch"] + e.get("write_bytes", 0.0), src


def rank_batch(cfg: int, rank: int, world: int = 1):
    """This rank's batch.  cfg 2-4 (weak scaling): the config's layout, a
    distinct seed per rank.  cfg 5 (strong scaling): shard `rank` of `world`
    contiguous packet ranges of the one 8M x 1500 B batch."""
    from netstack_amd import workloads as W

    if cfg == 5:
        return W.config(5).shard(rank, world)
    b = W.config(cfg)
    b.seed = b.seed + 1000 * rank
    return b


# ---------------------------------------------------------------------------
# CPU baseline: oracle (scalar C port of checksum.go) on a bounded sample
# ---------------------------------------------------------------------------
def cpu_baseline(batch, seconds: float, threads: int):
    import oracle as O

    # bounded sample: the first packets of this rank's batch (same bytes);
    # the threaded leg takes at least 64 MiB of payload per pass, so that
    # starting its threads (once per pass) is not what it measures (64-B
    # packets: 65,536 of them are only 4 MiB)
    n_s = min(batch.n, 65536)
    if threads > 1:
        mean = max(float(batch.desc["len"][:n_s].mean()), 1.0)
        n_s = min(batch.n, max(n_s, int((64 << 20) / mean)))
    d = batch.desc[:n_s].copy()
    span = int(d["off"][-1] + d["len"][-1])
    arena = batch.host_bytes(0, span)
    payload = int(d["len"].sum())
    out = np.zeros(n_s, dtype=np.uint16)
    O.c_batch_mt(arena, d, threads, out)  # warm
    reps, t0 = 0, time.perf_counter()
    while True:
        O.c_batch_mt(arena, d, threads, out)
        reps += 1
        el = time.perf_counter() - t0
        if el >= seconds:
            break
    return {"value": payload * reps / el / GIB, "unit": "GiB/s", "cores": threads, "kind": "port",
            "sample": f"{n_s} packets ({payload} B) of the rank-0 batch x {reps} passes, {el:.1f} s; "
                      f"oracle/csum_oracle.c scalar 2-B/iteration loop (checksum.go:41-43), "
                      f"{'single thread' if threads == 1 else f'{threads} pthreads, packet-parallel'}"}, \
        (arena, d, out)


def parity_sample(batch, out_dev, k: int = 65536) -> dict:
    """Bit-exact check of the measured launch's own results: the first and
    the last k packets of this rank's batch against the oracle (C port of
    checksum.go) on the same bytes, generated on the host."""
    import oracle as O

    got = out_dev.cpu().numpy().view(np.uint16)
    n = batch.n
    checked, ok = 0, True
    for a, b in ((0, min(k, n)), (max(min(k, n), n - k), n)):
        if b <= a:
            continue
        d = batch.desc[a:b].copy()
        lo = (int(d["off"].min()) // 16) * 16
        hi = int((d["off"] + d["len"].astype(np.uint64)).max())
        d["off"] -= np.uint64(lo)
        want, bad = O.c_batch(batch.host_bytes(lo, hi), d)
        ok = ok and bad == 0 and bool(np.array_equal(got[a:b], want))
        checked += b - a
    return {"packets": checked, "bit_exact": ok,
            "which": "first and last 65536 packets of the timed batch, results of the measured kernel"}


def kernel_name(arena_bytes: int, n: int, chained: bool = False, store: bool = False) -> str:
    """The csum_hyb instance launch_batch picks (csum_kernels.hip
    launch_batch / launch_hyb / launch_hyb_tp), as rocprofv3 names it."""
    win = "true" if arena_bytes + 64 >= 0xFFFF0000 else "false"
    ch = "true" if chained else "false"
    if arena_bytes // n >= 256:
        want = (64 << 10) // max(arena_bytes // n, 1)  # kTileBytes
        tp = next((t for t in (256, 128, 64, 32, 16, 8, 4, 2) if want >= t), 1)
        return f"nsk::csum_hyb<256,{tp},8,16,4,2,0,{win},2,{ch}>"
    return f"nsk::csum_hyb<64,64,16,8,4,2,5,{win},1,{ch}>"


def usable_cpus() -> dict:
    """The CPUs this process may run on: its affinity set (what `nproc`
    reports without OMP_NUM_THREADS), capped by the cgroup's CPU quota where
    one is set (a GPU box gives each GPU's jobs a share of a larger
    machine: there the affinity set is the whole machine)."""
    aff = len(os.sched_getaffinity(0))
    quota = None
    try:
        with open("/sys/fs/cgroup/cpu.max") as f:
            q, period = f.read().split()
        if q != "max":
            quota = -(-int(q) // int(period))
    except (OSError, ValueError):
        pass
    return {"affinity": aff, "cgroup_quota_cpus": quota, "usable": min(aff, quota) if quota else aff}


def device_ordinal(backend: str, local_rank: int, ndev: int, local_world: int) -> int:
    """This rank's GPU: one per rank.  With nccl (RCCL) a node must have a GPU
    for every local rank — RCCL rejects two ranks on one device, and mapping
    ranks modulo the count would hide a launch with too many ranks — so that
    is refused with a message.  With gloo (the control plane only) ranks
    beyond the GPU count share them, which the one-GPU box's multi-rank tests
    use."""
    if backend == "nccl" and (local_world > ndev or local_rank >= ndev):
        raise SystemExit(f"bench.py: {max(local_world, local_rank + 1)} ranks on this node but {ndev} GPU(s): "
                         f"the nccl (RCCL) backend needs one GPU per rank; launch at most {ndev} ranks, "
                         f"or pass --dist-backend gloo to share GPUs")
    return local_rank % max(1, ndev)


def main():
    args = parse()
    import torch

    from netstack_amd import Engine

    backend = args.dist_backend if args.dist_backend != "auto" else ("nccl" if torch.cuda.is_available() else "gloo")
    # one rank per GPU, made current before the process group exists
    ordinal = device_ordinal(backend, int(os.environ.get("LOCAL_RANK", "0")),
                             torch.cuda.device_count(), int(os.environ.get("LOCAL_WORLD_SIZE", "1")))
    torch.cuda.set_device(ordinal)
    dist = Dist(backend, ordinal)
    if dist.on and args.gpus != dist.world:
        print(f"warning: --gpus {args.gpus} != WORLD_SIZE {dist.world}", file=sys.stderr)
    dev = torch.device("cuda", ordinal)
    eng = Engine(ordinal)

    cfg = args.config
    if cfg == 8 and args.mode == "host":
        return tx_host_mode(args, dist, eng, dev)
    if cfg == 7 and args.mode == "host" and args.rx_layout != "ring":  # (bufs: device-resident only)
        raise SystemExit("--mode host --config 7 takes --rx-layout ring (ns_csum_rx_ring_host)")
    if cfg in (7, 8):
        return packet_mode(args, dist, eng, dev, tx=cfg == 8)
    if cfg == 1:
        return single_buffer_mode(args, dist, eng, dev)
    batch = rank_batch(cfg, dist.rank, dist.world)
    # Enough distinct batches per rank that one rotation exceeds the 256 MiB
    # MALL (cfg2: 2 x 1.5 GB, cfg3: 4 x 82 MB, cfg4: 2 x 0.67 GB); cfg5's
    # 12.6 GB batch is re-read as is.
    rotate = args.rotate or {2: 2, 3: 4, 4: 2, 5: 1}[cfg]
    if cfg == 5 and rotate != 1:
        raise SystemExit("--rotate applies to cfg 2-4 only")
    if args.mode == "host":
        return host_mode(args, dist, eng, batch, dev)

    arenas, descs = [], []
    for r in range(rotate):
        b = batch if r == 0 else rank_batch(cfg, dist.rank + 100 * r)
        arenas.append(b.arena_device(dev))
        descs.append(torch.from_numpy(b.desc.view(np.uint8).copy()).to(dev))
    out = torch.empty(batch.n, dtype=torch.int16, device=dev)
    stream = torch.cuda.current_stream(dev)

    # HIP events on the launch stream (torch's current) bracketing the K timed
    # launches: average launch duration = (end - start) / K, which counts the
    # ~0.6 us dependent-launch boundary too.  (An event pair around EVERY
    # launch costs ~10 us per step on MI355X — profiles/r01 trace — and would
    # slow the very steps it measures.)
    ev = [torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)]
    state = {"i": 0}

    def step():
        k = state["i"]
        if k == args.warmup:
            ev[0].record(stream)
        eng.batch_tensors(arenas[k % rotate], descs[k % rotate], out, stream=stream)
        state["i"] = k + 1
        if state["i"] == args.warmup + args.steps:
            ev[1].record(stream)

    wall, local = timed_region(step, torch.cuda.synchronize, dist, args.steps, args.warmup, dev)
    bad = eng.sync()
    kern_avg_s = ev[0].elapsed_time(ev[1]) / 1e3 / args.steps

    # per-launch statistics and the same-run read calibration (untimed), then
    # one more launch of the same kernel instance over arenas[0]: its results
    # are what the CPU leg checks against the oracle
    per_launch = launch_stats(lambda: eng.batch_tensors(arenas[0], descs[0], out, stream=stream), stream)
    # the same batch re-read back to back (no rotation: part of it may be
    # served by the MALL) — reported beside the rotated headline
    unrot_us = b2b_us(lambda k: eng.batch_tensors(arenas[0], descs[0], out, stream=stream), stream)
    # cfg3's 64-B packets are not read in the big-packet shape: its ceiling is
    # the floor kernel of the same access (quad-lane, nontemporal, payload
    # loads not waiting for the descriptors), over the same rotated batches
    calib = floor_calibration(arenas, descs, batch, stream) if cfg == 3 else stream_calibration(arenas, stream)
    eng.batch_tensors(arenas[0], descs[0], out, stream=stream)
    torch.cuda.synchronize()
    pipe = pipelined(eng, arenas, descs, batch.n, batch.algorithmic_bytes, out, stream) if rotate > 1 else None

    payload_rank = batch.payload_bytes
    total_payload = dist.sum(float(payload_rank), dev)
    algo_bytes = batch.algorithmic_bytes
    achieved_gbs = algo_bytes / kern_avg_s / 1e9
    traffic, traffic_src = pmc_traffic(args.pmc_json, cfg)

    result = {
        "metric": METRIC,
        "value": total_payload * args.steps / wall / GIB,
        "unit": "GiB/s",
        "n_gpus": dist.world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": wall / args.steps * 1e3,
        "higher_is_better": True,
        "scaling": "strong" if cfg == 5 else "weak",
        "vs_baseline": None,
        "dtype": "u8",
        "data": "synthetic (splitmix64 bytes, random per-packet initial), resident in HBM",
        "config": {
            "workload": WORKLOADS[cfg],
            "packets_per_gpu": batch.n,
            "payload_bytes_per_gpu": payload_rank,
            "global_packets": int(dist.sum(float(batch.n), dev)),
            "parallelism": f"shard{dist.world} (independent batches, no collective)",
            "rotating_batches": rotate,
        },
        "roofline": {
            "bound": "hbm",
            "achieved": achieved_gbs,
            "peak": HBM_PEAK_GBS,
            "unit": "GB/s",
            "frac": achieved_gbs / HBM_PEAK_GBS,
            "traffic": traffic,
            "traffic_source": traffic_src,
            "kernel": kernel_name(batch.arena_bytes, batch.n),
            "algorithmic_bytes_per_launch": algo_bytes,
            "avg_launch_us": kern_avg_s * 1e6,
            "rotating_batches": rotate,
            "basis": (f"avg_launch_us over the timed region's back-to-back launches cycling {rotate} distinct "
                      f"batches ({rotate * (batch.arena_bytes + 18 * batch.n) / 2**20:.0f} MiB of arenas, "
                      f"descriptor tables and results > the 256 MiB MALL)"
                      if rotate > 1 else "avg_launch_us over the timed region's back-to-back launches"),
            "unrotated": {"avg_launch_us": unrot_us, "frac": algo_bytes / unrot_us / 1e3 / HBM_PEAK_GBS,
                          "note": "batch 0 re-read back to back, 20 launches: may hit the MALL"},
            "per_launch_us": {"median": per_launch[len(per_launch) // 2], "min": per_launch[0],
                              "max": per_launch[-1], "launches": len(per_launch),
                              "note": "own event pair per launch, after the timed region (batch 0)"},
            "stream_calibration": calib,
            "frac_of_calibration": (achieved_gbs / calib["GBps"]) if calib else None,
            "calibration_basis": ("algorithmic GB/s of the cfg3 floor kernels (payload and descriptor reads, "
                                  "result writes; no descriptor -> payload dependency)" if cfg == 3 else
                                  "pure read GB/s of the same rotated arenas in the big-packet shape"),
        },
        "bad_descriptors": bad,
    }
    # per GPU: the whole-job value split evenly, and the
    # spread of the ranks' own kernel averages (roofline above is rank 0's)
    kmax = dist.max(kern_avg_s, dev)
    kmin = -dist.max(-kern_avg_s, dev)
    result["per_gpu"] = {"value": result["value"] / dist.world, "unit": "GiB/s",
                         "kernel_avg_us_min": kmin * 1e6, "kernel_avg_us_max": kmax * 1e6}
    if pipe is not None:
        # whole-job rate of the pipelined stream of batches: every rank's
        # payload over the slowest rank's time per batch
        pipe["value"] = total_payload / (dist.max(pipe["us_per_batch"], dev) * 1e-6) / GIB
        pipe["unit"] = "GiB/s"
        pfail = dist.sum(0.0 if pipe["bit_exact_vs_timed"] else 1.0, dev)  # every rank joins
        pipe["bit_exact_vs_timed"] = pfail == 0
        result["pipelined"] = pipe

    if not args.no_parity:
        # Every rank checks its own measured launch's results (the first and
        # last 65,536 packets of its batch or shard) against the oracle; the
        # count of failing ranks is all-reduced.
        ps = parity_sample(batch, out)
        failed = dist.sum(0.0 if ps["bit_exact"] else 1.0, dev)
        ps["scope"] = ("sampled: the first and last 65,536 results of the measured launch on every rank; "
                       "every result is checked at full size by pytest -m gpu")
        ps["ranks_checked"] = dist.world
        ps["ranks_failed"] = int(failed)
        ps["bit_exact"] = ps["bit_exact"] and failed == 0
        result["parity_sample"] = ps
    if dist.rank == 0 and dist.world > 1:
        result["cpu_baseline_note"] = "timed at N=1 only (bench.py --gpus 1), not beside a multi-GPU run"
    elif dist.rank == 0 and not args.no_cpu:
        # The CPU leg (rank 0 at N=1): the oracle timed as the scalar baseline.
        cb, _ = cpu_baseline(batch, args.cpu_seconds, 1)
        result["cpu_baseline"] = cb
        cpus = usable_cpus()
        th = args.cpu_threads or cpus["usable"]
        cbm, _ = cpu_baseline(batch, max(2.0, args.cpu_seconds / 4), th)
        cbm["host_cpus"] = cpus
        result["cpu_baseline_multicore"] = cbm

    if dist.rank == 0:
        print(json.dumps(result), flush=True)
    eng.close()
    dist.close()


RX_N = 1 << 20


def packet_mode(args, dist, eng, dev, tx: bool):
    """Device-resident IPv4/TCP packet batches: 1M 1500-B
    packets per GPU in HBM, two independent descriptors per packet
    (workloads._tcp_desc, fused: the IPv4 header; the pseudo-header addresses
    followed by the TCP header and payload, one contiguous piece with the
    length and protocol words as its initial), one ns_csum_batch_dev per
    step.  `--rx-layout chained` measures the three-descriptor chained table
    instead (the checksum kernel plus the fold_scan pass that folds runs).

    RX (config 7, rank 2: segment.parse / the IPv4 header check): every
    1000th packet has a corrupted payload byte; the check after the timed
    region requires exactly those TCP sums to fail and every IPv4 header and
    every other TCP segment to sum to 0xffff (segment.go:180,
    checker.go:51-53) — a size-independent property over all 1M packets.

    TX (config 8, rank 1: buildTCPHdr + addIPHeader for a whole batch): the
    same segments with zeroed checksum fields, ns_csum_batch_dev_store writes
    ^sum into both fields of every packet (connect.go:662-663, ipv4.go:236).
    By default (`--tx-layout struct`) the segments are laid out as
    sendTCPBatch builds them: stack.NewPacketDescriptors' one buffer of 54-B
    header slots (route.go:181-188) and the payload in a view of its own
    (workloads.tx_split_*), and ns_csum_tcp_tx fills them from the batch's
    geometry (no table: a payload pass, then a header pass that writes the
    slots back whole).  `--tx-layout split` fills the same layout through a
    table of three descriptors per packet, the payload + TCP header pair
    folded in the tile (NS_BATCH_PAIRED).  `--tx-layout wire` keeps config
    7's wire-contiguous packets.  The fields are re-zeroed after
    the timed region and filled by one more launch; the check requires the
    whole arena to equal one whose checksums torch integer ops computed
    independently, and every filled segment to verify.

    value = packet bytes / s (GiB/s)."""
    import torch

    from netstack_amd import workloads as W

    seed = 7000 + dist.rank
    if not tx and args.rx_layout in ("ring", "bufs"):
        return ring_host_mode(args, dist, eng, dev, seed) if args.mode == "host" else \
            ring_mode(args, dist, eng, dev, seed)
    struct = tx and args.tx_layout == "struct"
    split = tx and args.tx_layout in ("split", "struct")
    fused = args.rx_layout == "fused"
    chained = not fused and not split
    k = W.per_packet(fused)
    geo = W.tx_struct_geometry(RX_N)
    if split:
        arena, _ = W.tx_split_batch(RX_N, seed, dev)
        d = W.tx_split_desc(RX_N, True, paired=True)
        ip_at, tcp_at = W.tx_split_order(RX_N, True)
        k = 3
        bad_idx = np.zeros(0, np.int64)
    elif tx:
        arena, d = W.tx_batch(RX_N, seed, dev, fused=fused)
        bad_idx = np.zeros(0, np.int64)
    else:
        arena, d, bad_idx = W.rx_batch(RX_N, seed, dev, corrupt_every=1000, fused=fused)
    desc = torch.from_numpy(d.view(np.uint8).copy()).to(dev)
    out = torch.empty(2 * RX_N if struct else len(d), dtype=torch.int16, device=dev)
    stream = torch.cuda.current_stream(dev)
    ev = [torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)]
    state = {"i": 0}
    # Every layout alternates between two batches of the same packets (3.2 GB
    # > the 256 MiB MALL), as cfg2's rotating batches: no launch re-reads what
    # the one before it left in the MALL, and the structured fill writes header
    # slots the previous call did not, as sendTCPBatch's fresh
    # NewPacketDescriptors buffers are (re-filling one batch leaves its 57 MB
    # of slot writes in the MALL between calls).  The checks
    # below run on the first batch.
    if split:
        arenas = [arena, W.tx_split_batch(RX_N, seed, dev)[0]]
    elif tx:
        arenas = [arena, W.tx_batch(RX_N, seed, dev, fused=fused)[0]]
    else:
        arenas = [arena, W.rx_batch(RX_N, seed, dev, corrupt_every=1000, fused=fused)[0]]

    def fill(j=0):
        a = arenas[j % 2]
        if struct:
            eng.tcp_tx(a, geo, out=out, stream=stream)
        else:
            eng.batch_tensors(a, desc, out, chained=chained, stream=stream, store=tx, paired=split)

    def step():
        k = state["i"]
        if k == args.warmup:
            ev[0].record(stream)
        fill(k)
        state["i"] = k + 1
        if state["i"] == args.warmup + args.steps:
            ev[1].record(stream)

    wall, _ = timed_region(step, torch.cuda.synchronize, dist, args.steps, args.warmup, dev)
    bad = eng.sync()
    kern_avg_s = ev[0].elapsed_time(ev[1]) / 1e3 / args.steps
    k_cpu = k * 65536
    span = int((d["off"][:k_cpu] + d["len"][:k_cpu].astype(np.uint64)).max())
    if struct:  # the oracle's sample: the first 65,536 segments' slots and payload
        span = geo["pay_off"] + 65536 * geo["mss"]
    if tx:
        # untimed: re-zero both fields, fill them with one launch, check
        if split:
            h = arena[:RX_N * W.TX_HDR].view(RX_N, W.TX_HDR)
            h[:, W.TX_IP_AT + 10:W.TX_IP_AT + 12] = 0
            h[:, W.TX_TCP_AT + 16:W.TX_TCP_AT + 18] = 0
        else:
            p = arena.view(RX_N, W.RX_STRIDE)
            p[:, 10:12] = 0
            p[:, 36:38] = 0
        before = arena[:span].cpu().numpy() if dist.rank == 0 and not args.no_cpu else None
        fill()
        torch.cuda.synchronize()
        bad += eng.sync()
        rx = W.tx_split_expected(RX_N, seed, dev) if split else W.rx_batch(RX_N, seed, dev)[0]
        arena_ok = bool(torch.equal(arena, rx))
        del rx
        vd = W.tx_split_desc(RX_N, False, paired=True) if split else W._tcp_desc(RX_N, fused)
        chk = torch.from_numpy(vd.view(np.uint8).copy()).to(dev)
        vres = eng.batch_tensors(arena, chk, chained=chained, stream=stream, paired=split).cpu().numpy().view(np.uint16)
        res = out.cpu().numpy().view(np.uint16)
        ip_ok = vres[ip_at if split else slice(0, None, k)] == 0xFFFF
        tcp_fail = np.flatnonzero(vres[tcp_at if split else slice(k - 1, None, k)] != 0xFFFF)
        prop_ok = arena_ok and bool(ip_ok.all()) and tcp_fail.size == 0
    else:
        before = None
        res = out.cpu().numpy().view(np.uint16)
        ip_ok = res[0::k] == 0xFFFF
        tcp_fail = np.flatnonzero(res[k - 1::k] != 0xFFFF)
        prop_ok = bool(ip_ok.all()) and np.array_equal(tcp_fail, bad_idx)
    fails = dist.sum(0.0 if prop_ok else 1.0, dev)
    pkt_bytes = RX_N * W.RX_PKT
    total = dist.sum(float(pkt_bytes), dev)
    n_desc = 0 if struct else len(d)
    # packet bytes + the 8-B address re-read + per descriptor: 16-B read and
    # a u16 result written (chained: also a u32 partial + u16 flag written,
    # then read back); TX adds the two 2-B field stores per packet.  The
    # structured fill reads each segment's payload and its two headers (the
    # pseudo-header's addresses are the route's) and writes the two fields.
    if struct:
        algo = pkt_bytes + 4 * RX_N
    else:
        algo = pkt_bytes + 8 * RX_N + n_desc * (16 + 2 + (12 if chained else 0)) + (4 * RX_N if tx else 0)
    achieved = algo / kern_avg_s / 1e9
    traffic, traffic_src = (pmc_traffic(args.pmc_json, "8struct") if struct else
                            pmc_traffic(args.pmc_json, "8split") if split else
                            pmc_traffic(args.pmc_json, 8 if tx else 7) if fused else (None, None))
    check = {"ipv4_all_valid": bool(ip_ok.all()), "tcp_failures": int(tcp_fail.size),
             "expected_failures": int(bad_idx.size), "ok": prop_ok, "ranks_failed": int(fails)}
    if tx:
        check["arena_equals_rx_batch"] = arena_ok
    result = {
        "metric": ("TX checksum fill" if tx else "RX checksum verification")
        + " GiB/s device-resident (IPv4 + TCP, 1500-B packets)",
        "value": total * args.steps / wall / GIB, "unit": "GiB/s", "n_gpus": dist.world,
        "steps": args.steps, "warmup": args.warmup, "ms_per_step": wall / args.steps * 1e3,
        "higher_is_better": True, "scaling": "weak", "vs_baseline": None, "dtype": "u8",
        "data": ("synthetic packets to send (checksum fields zero), resident in HBM" if tx else
                 "synthetic received packets (valid IPv4/TCP checksums, 1 in 1000 corrupted), resident in HBM"),
        "config": {"workload": ("tx" if tx else "rx") + ": 1,048,576 x 1500-B IPv4/TCP packets per GPU, "
                   + ("in sendTCPBatch's layout (54-B header slots + a payload view), filled from the "
                      "batch geometry (ns_csum_tcp_tx, no descriptor table)" if struct
                      else "in sendTCPBatch's layout (54-B header slots + a payload view), 3 descriptors each "
                      "(IPv4 header; payload + pseudo-header addresses and TCP header, NS_BATCH_PAIRED)" if split
                      else "2 descriptors each (IPv4 header; pseudo-header addresses + TCP segment)" if fused
                      else "3 chained descriptors each") + (", 2 checksum stores" if tx else ""),
                   "packets_per_gpu": RX_N, "descriptors_per_gpu": n_desc, "rotating_batches": 2},
        "roofline": {"bound": "hbm", "achieved": achieved, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                     "frac": achieved / HBM_PEAK_GBS, "traffic": traffic, "traffic_source": traffic_src,
                     "kernel": ("nsk::tcp_tx_pay<13,0,8> (payload pass, 8-lane groups) + nsk::tcp_tx_hdr<4,4,1> "
                                "(header pass, one tile per wave, nt sc1 slot stores)"
                                if struct else kernel_name(arena.numel(), n_desc, chained=chained, store=tx or split)
                                + (" + nsk::fold_scan" if chained else "")),
                     "layout": ("struct (sendTCPBatch: header slots + payload view, ns_csum_tcp_tx)" if struct
                                else "split (sendTCPBatch: header slots + payload view)" if split else "wire"),
                     "algorithmic_bytes_per_launch": algo, "avg_launch_us": kern_avg_s * 1e6},
        "bad_descriptors": bad,
        "property_check": check,
    }
    if dist.rank == 0 and not args.no_cpu:
        import oracle as O

        # CPU leg: the oracle on the first 65,536 packets' descriptors, same
        # bytes (TX: the bytes before the checked launch, and its stores)
        src = before if tx else arena[:span].cpu().numpy()
        if struct:  # sendTCPBatch's checksum steps over the first 65,536 segments
            g = geo
            stored, want = O.c_send_tcp_batch(src, g["hdr_off"], g["pay_off"], 65536 * g["mss"], g["mss"],
                                              g["slot"], g["ip_at"], g["ip_len"], g["tcp_at"], g["tcp_len"],
                                              g["src"], g["dst"], g["protocol"])
            ps = {"packets": 65536, "bit_exact": bool(np.array_equal(res[:2 * 65536], want))}
            # the sample's slots as filled, and its payload unchanged
            hs, po = 65536 * g["slot"], g["pay_off"]
            got = arena[:span].cpu().numpy()
            ps["stores_bit_exact"] = bool(np.array_equal(got[:hs], stored[:hs]) and
                                          np.array_equal(got[po:span], stored[po:span]))
        else:
            want, _ = O.c_batch_paired(src, d[:k_cpu]) if split else O.c_batch(src, d[:k_cpu], chained=chained)
            ps = {"packets": k_cpu // k, "bit_exact": bool(np.array_equal(res[:k_cpu], want))}
        if tx and not struct:
            stored, _ = O.apply_stores(src, d[:k_cpu], want)
            ps["stores_bit_exact"] = bool(np.array_equal(arena[:span].cpu().numpy(), stored))
        result["parity_sample"] = ps
        if struct:
            # CPU leg: the same 65,536 segments through the oracle's C
            # restatement of sendTCPBatch's checksum steps, one core, timed
            # (bounded by --cpu-seconds); value in packet bytes per second
            result["cpu_baseline"] = send_tcp_batch_cpu(O, src, geo, args.cpu_seconds)
    if dist.rank == 0:
        print(json.dumps(result), flush=True)
    eng.close()
    dist.close()


def send_tcp_batch_cpu(O, src, g, seconds):
    """CPU leg of config 8: the first 65,536 segments through the oracle's C
    restatement of sendTCPBatch's checksum steps, one core, timed for about
    `seconds`; value in packet bytes per second."""
    from netstack_amd import workloads as W

    work = np.ascontiguousarray(src).copy()
    reps, t0 = 0, time.perf_counter()
    while True:
        O.c_send_tcp_batch(work, g["hdr_off"], g["pay_off"], 65536 * g["mss"], g["mss"], g["slot"],
                           g["ip_at"], g["ip_len"], g["tcp_at"], g["tcp_len"], g["src"], g["dst"], copy=False)
        reps += 1
        el = time.perf_counter() - t0
        if el >= seconds:
            break
    return {"value": 65536 * W.RX_PKT * reps / el / GIB, "unit": "GiB/s", "cores": 1, "kind": "port",
            "sample": f"65,536 segments ({65536 * W.RX_PKT} packet bytes) of the rank-0 batch x {reps} passes, "
                      f"{el:.1f} s; oracle_send_tcp_batch (sendTCPBatch + buildTCPHdr + addIPHeader's checksum "
                      f"steps over oracle/csum_oracle.c's scalar loop), single thread"}


def tx_calls(geo, calls):
    """cfg8's geometry as `calls` sendTCPBatch calls of consecutive segments
    (each its own geometry: the fill is affine in the segment index)."""
    n = -(-geo["size"] // geo["mss"])
    per = -(-n // calls)
    out = []
    for a in range(0, n, per):
        out.append(dict(geo, hdr_off=geo["hdr_off"] + a * geo["slot"], pay_off=geo["pay_off"] + a * geo["mss"],
                        size=min(geo["size"] - a * geo["mss"], per * geo["mss"])))
    return out


def tx_host_mode(args, dist, eng, dev):
    """`--mode host --config 8`: sendTCPBatch's fill over HOST memory
    (ns_csum_tcp_tx_host), config 8's 1M x 1460-B segments per GPU in
    sendTCPBatch's layout (54-B header slots + the payload view) in a pinned
    host arena, as --tx-calls calls (1, or e.g. 23,832 = one per 64 KiB GSO
    write: many connections' calls in one).  Each step is one synchronous
    call: the slots and payload go to the device, the fill runs there, and
    the fields are written into the host slots.  The refills are idempotent
    (the fields are summed as zero).  After the timed region the host arena
    must equal tx_split_expected's (torch integer ops).  Recorded in DESIGN.md
    as the PCIe-inclusive rate; the device-resident line is --mode dev."""
    import torch

    from netstack_amd import workloads as W
    from netstack_amd.engine import tx_table

    seed = 7000 + dist.rank
    geo = W.tx_struct_geometry(RX_N)
    src = W.tx_split_batch(RX_N, seed, dev)[0].cpu()
    arena = torch.empty(src.numel(), dtype=torch.uint8).pin_memory()
    arena.copy_(src)
    del src
    a = arena.numpy()
    before = a[:geo["pay_off"] + 65536 * geo["mss"]].copy() if dist.rank == 0 and not args.no_cpu else None
    calls = tx_calls(geo, max(1, args.tx_calls))
    table = tx_table(calls)

    def step():
        eng.tcp_tx_host(a, table)

    wall, _ = timed_region(step, lambda: None, dist, args.steps, args.warmup, dev)
    want = W.tx_split_expected(RX_N, seed, dev)
    ok = bool(torch.equal(arena.to(dev), want))
    del want
    fails = dist.sum(0.0 if ok else 1.0, dev)
    total = dist.sum(float(RX_N * W.RX_PKT), dev)
    result = {
        "metric": "TX checksum fill GiB/s host-inclusive (H2D + fill + fields written back; IPv4 + TCP, 1500-B packets)",
        "value": total * args.steps / wall / GIB, "unit": "GiB/s", "n_gpus": dist.world,
        "steps": args.steps, "warmup": args.warmup, "ms_per_step": wall / args.steps * 1e3,
        "higher_is_better": True, "scaling": "weak", "vs_baseline": None, "dtype": "u8",
        "data": "synthetic packets to send (checksum fields zero before the first call), pinned host memory",
        "config": {"workload": "tx: 1,048,576 x 1500-B IPv4/TCP packets per GPU in sendTCPBatch's layout "
                               "(54-B header slots + a payload view) in host memory, ns_csum_tcp_tx_host",
                   "calls": len(calls), "segments_per_call": -(-RX_N // len(calls)),
                   "staging": "64 MiB chunks, 4 in flight (one stream each); sums to mapped memory, fields "
                              "written by the host"},
        "property_check": {"arena_equals_expected": ok, "ranks_failed": int(fails)},
    }
    if dist.rank == 0 and not args.no_cpu:
        import oracle as O

        result["cpu_baseline"] = send_tcp_batch_cpu(O, before, geo, args.cpu_seconds)
    if dist.rank == 0:
        print(json.dumps(result), flush=True)
    eng.close()
    dist.close()


def ring_mode(args, dist, eng, dev, seed):
    """`--config 7 --rx-layout ring`: the receive path of 1M received 1500-B
    IPv4/TCP packets per GPU, one per 1504-B slot of a ring in HBM, with no
    descriptor table: one ns_csum_rx_ring per step parses every packet's
    headers on the device (IsValid, the fragment checks, segment.parse's
    length checks), takes the pseudo-header from the packet's own addresses
    and writes each slot's verdict (NS_PKB_*) and its two sums.  Every 1000th
    packet has a corrupted payload byte: the check after the timed region
    requires exactly those to be INVALID, every other VALID and every IPv4
    header to sum to 0xffff, over all 1M slots; the first 65,536 slots are
    compared bit for bit with the oracle's C restatement (oracle_rx_ring),
    which is also the timed CPU leg.  value = packet bytes / s (GiB/s)."""
    import torch

    from netstack_amd import workloads as W

    arena, lens, bad_idx = W.rx_ring_batch(RX_N, seed, dev, corrupt_every=1000)
    # two rings of the same frames, alternating (3.2 GB > the 256 MiB MALL, as
    # cfg2's rotating batches: no launch re-reads what the one before it left
    # in the MALL)
    rings = [arena, W.rx_ring_batch(RX_N, seed, dev, corrupt_every=1000)[0]]
    bufs = args.rx_layout == "bufs"
    stride = W.RX_STRIDE
    if args.bufs_stride and args.bufs_stride != W.RX_STRIDE:
        # the same slots spread to a wider spacing (a pool of line-aligned
        # buffers when it is a multiple of 128): the frames do not move
        # within their buffers
        stride = args.bufs_stride
        if stride % 16 or stride < W.RX_STRIDE:
            raise SystemExit("--bufs-stride must be a multiple of 16 and at least 1504")

        def spread(a):
            b = torch.zeros(RX_N, stride, dtype=torch.uint8, device=dev)
            b[:, :W.RX_STRIDE] = a.view(RX_N, W.RX_STRIDE)
            return b.view(-1)

        rings = [spread(r) for r in rings]
        arena = rings[0]
    ring = dict(stride=stride, n=RX_N)
    if bufs:
        # `--rx-layout bufs` (ns_csum_rx_bufs): the same buffers handed over in
        # a shuffled order, as a NIC's buffer pool returns them: packet k is
        # the frame in slot perm[k], found through an offset table
        perm = np.random.default_rng(seed).permutation(RX_N) if args.bufs_order == "shuffled" else np.arange(RX_N)
        offs = torch.from_numpy((perm.astype(np.int64) * stride).astype(np.int32)).to(dev)
        lens = lens[torch.from_numpy(perm).to(dev)].contiguous()
        inv = np.empty(RX_N, dtype=np.int64)
        inv[perm] = np.arange(RX_N)
        bad_idx = np.sort(inv[bad_idx])
    verdict = torch.empty(RX_N, dtype=torch.uint8, device=dev)
    sums = torch.empty(2 * RX_N, dtype=torch.int16, device=dev)
    stream = torch.cuda.current_stream(dev)
    ev = [torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)]
    state = {"i": 0}

    def step():
        k = state["i"]
        if k == args.warmup:
            ev[0].record(stream)
        if bufs:
            eng.rx_bufs(rings[k % 2], ring, offs, lens, sums=sums, verdict=verdict, stream=stream)
        else:
            eng.rx_ring(rings[k % 2], ring, lens, sums=sums, verdict=verdict, stream=stream)
        state["i"] = k + 1
        if state["i"] == args.warmup + args.steps:
            ev[1].record(stream)

    wall, _ = timed_region(step, torch.cuda.synchronize, dist, args.steps, args.warmup, dev)
    bad = eng.sync()
    kern_avg_s = ev[0].elapsed_time(ev[1]) / 1e3 / args.steps
    v = verdict.cpu().numpy()
    sm = sums.cpu().numpy().view(np.uint16)
    want = np.ones(RX_N, dtype=np.uint8)
    want[bad_idx] = 0
    ip_ok = bool((sm[0::2] == 0xFFFF).all())
    tcp_fail = np.flatnonzero(sm[1::2] != 0xFFFF)
    prop_ok = ip_ok and bool((v == want).all()) and np.array_equal(tcp_fail, bad_idx) and bad == 0
    fails = dist.sum(0.0 if prop_ok else 1.0, dev)
    pkt_bytes = RX_N * W.RX_PKT
    total = dist.sum(float(pkt_bytes), dev)
    # per slot: the packet's bytes and its u32 length read (bufs: and its u32
    # offset); its verdict (1 B) and its two u16 sums written
    algo = pkt_bytes + RX_N * (4 + 1 + 4 + (4 if bufs else 0))
    achieved = algo / kern_avg_s / 1e9
    traffic, traffic_src = pmc_traffic(args.pmc_json, "7bufs" if bufs else "7ring")
    result = {
        "metric": "RX checksum verification GiB/s device-resident (IPv4 + TCP, 1500-B packets)",
        "value": total * args.steps / wall / GIB, "unit": "GiB/s", "n_gpus": dist.world,
        "steps": args.steps, "warmup": args.warmup, "ms_per_step": wall / args.steps * 1e3,
        "higher_is_better": True, "scaling": "weak", "vs_baseline": None, "dtype": "u8",
        "data": "synthetic received packets (valid IPv4/TCP checksums, 1 in 1000 corrupted), resident in HBM",
        "config": {"workload": (f"rx buffer list: 1,048,576 x 1500-B IPv4/TCP packets per GPU in buffers spaced "
                                f"{stride} B apart, handed over in {args.bufs_order} order through an offset table, "
                                "parsed and verified on the device (ns_csum_rx_bufs)" if bufs else
                                f"rx ring: 1,048,576 x 1500-B IPv4/TCP packets per GPU in {stride}-B slots, parsed "
                                "and verified on the device from the slots' lengths (ns_csum_rx_ring, no table)"),
                   "packets_per_gpu": RX_N, "descriptors_per_gpu": 0, "rotating_batches": 2},
        "roofline": {"bound": "hbm", "achieved": achieved, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                     "frac": achieved / HBM_PEAK_GBS, "traffic": traffic, "traffic_source": traffic_src,
                     "kernel": "nsk::rx_ring<13,0,2,4,1,1,0,1>" if bufs else "nsk::rx_ring<13>",
                     "layout": "buffer list (shuffled 1504-B buffers, u32 offsets and lengths)" if bufs
                     else "ring (1504-B slots, u32 lengths)",
                     "algorithmic_bytes_per_launch": algo, "avg_launch_us": kern_avg_s * 1e6},
        "bad_descriptors": bad,
        "property_check": {"ipv4_all_valid": ip_ok, "tcp_failures": int(tcp_fail.size),
                           "expected_failures": int(bad_idx.size), "verdicts_as_expected": bool((v == want).all()),
                           "ok": prop_ok, "ranks_failed": int(fails)},
    }
    if dist.rank == 0 and not args.no_cpu and not bufs and stride == W.RX_STRIDE:
        import oracle as O

        k = 65536
        src = arena[:k * W.RX_STRIDE].cpu().numpy()
        ln = lens[:k].cpu().numpy().view(np.uint32)
        ov, osm = O.c_rx_ring(src, ln, W.RX_STRIDE, k)
        result["parity_sample"] = {"packets": k, "bit_exact": bool(np.array_equal(ov, v[:k]) and
                                                                      np.array_equal(osm, sm[:2 * k]))}
        reps, t0 = 0, time.perf_counter()
        while True:
            O.c_rx_ring(src, ln, W.RX_STRIDE, k)
            reps += 1
            el = time.perf_counter() - t0
            if el >= args.cpu_seconds:
                break
        result["cpu_baseline"] = {
            "value": k * W.RX_PKT * reps / el / GIB, "unit": "GiB/s", "cores": 1, "kind": "port",
            "sample": f"{k:,} slots ({k * W.RX_PKT} packet bytes) of the rank-0 ring x {reps} passes, {el:.1f} s; "
                      "oracle_rx_ring (dispatch + HandlePacket + IsValid + segment.parse's checksum over "
                      "oracle/csum_oracle.c's scalar loop), single thread"}
    if dist.rank == 0:
        print(json.dumps(result), flush=True)
    eng.close()
    dist.close()


def ring_host_mode(args, dist, eng, dev, seed):
    """`--mode host --config 7 --rx-layout ring`: the same 1M-slot receive
    ring in pinned HOST memory (recvmmsg's buffers), verified by one
    ns_csum_rx_ring_host per step: the slots and lengths go up over PCIe, the
    parse and the sums run on the device, verdicts and sums come back through
    mapped memory.  The property check of ring_mode on the results.  The
    PCIe-inclusive rate, recorded in DESIGN.md; the device-resident line is
    --mode dev."""
    import torch

    from netstack_amd import workloads as W

    arena_d, lens_d, bad_idx = W.rx_ring_batch(RX_N, seed, dev, corrupt_every=1000)
    arena = torch.empty(arena_d.numel(), dtype=torch.uint8).pin_memory()
    arena.copy_(arena_d)
    lens = lens_d.cpu().numpy().view(np.uint32).copy()
    del arena_d, lens_d
    a = arena.numpy()
    ring = dict(stride=W.RX_STRIDE, n=RX_N)
    res = {}

    def step():
        res["v"], res["s"] = eng.rx_ring_host(a, ring, lens)

    wall, _ = timed_region(step, lambda: None, dist, args.steps, args.warmup, dev)
    v, sm = res["v"], res["s"]
    want = np.ones(RX_N, dtype=np.uint8)
    want[bad_idx] = 0
    ip_ok = bool((sm[0::2] == 0xFFFF).all())
    tcp_fail = np.flatnonzero(sm[1::2] != 0xFFFF)
    prop_ok = ip_ok and bool((v == want).all()) and np.array_equal(tcp_fail, bad_idx) and eng.sync() == 0
    fails = dist.sum(0.0 if prop_ok else 1.0, dev)
    total = dist.sum(float(RX_N * W.RX_PKT), dev)
    result = {
        "metric": "RX checksum verification GiB/s host-inclusive (H2D + parse + verdicts back; IPv4 + TCP, "
                  "1500-B packets)",
        "value": total * args.steps / wall / GIB, "unit": "GiB/s", "n_gpus": dist.world,
        "steps": args.steps, "warmup": args.warmup, "ms_per_step": wall / args.steps * 1e3,
        "higher_is_better": True, "scaling": "weak", "vs_baseline": None, "dtype": "u8",
        "data": "synthetic received packets (valid IPv4/TCP checksums, 1 in 1000 corrupted), pinned host memory",
        "config": {"workload": "rx ring: 1,048,576 x 1500-B IPv4/TCP packets per GPU in 1504-B slots in host "
                               "memory, ns_csum_rx_ring_host",
                   "packets_per_gpu": RX_N,
                   "staging": "64 MiB chunks of whole slots, 4 in flight (one stream each); verdicts and sums "
                              "to mapped memory"},
        "property_check": {"ipv4_all_valid": ip_ok, "tcp_failures": int(tcp_fail.size),
                           "expected_failures": int(bad_idx.size), "verdicts_as_expected": bool((v == want).all()),
                           "ok": prop_ok, "ranks_failed": int(fails)},
    }
    if dist.rank == 0:
        print(json.dumps(result), flush=True)
    eng.close()
    dist.close()


def single_buffer_mode(args, dist, eng, dev):
    """BASELINE.json configs[0]: one 65,536-B buffer (splitmix64 seed 1),
    header.Checksum(buf, 0) (checksum.go:52-55).  The reference times this on
    the host CPU; here three things are timed on the same buffer, each
    checked bit for bit against the oracle:
      - the scalar CPU port of checksum.go:41-43 (oracle/csum_oracle.c, one
        core) — the reference's own path, restated (cpu_baseline);
      - the synchronous C-ABI call ns_csum_checksum (what the Go shim calls:
        copy into mapped staging, one launch, one wait), median latency over
        `steps` calls through ctypes — `value`;
      - the kernel alone on the buffer resident in HBM (ns_csum_batch_dev,
        one descriptor), back-to-back average.
    One buffer per call is latency-bound, not bandwidth-bound: this config is
    plumbing, as BASELINE.json says, not the headline."""
    import torch

    import oracle as O
    from netstack_amd import workloads as W

    b = W.config(1)
    buf = b.arena_host()[:65536].copy()
    d1 = b.desc.copy()
    want = int(O.c_batch(buf, d1)[0][0])
    # warm-up + timed synchronous calls
    for _ in range(args.warmup + 3):
        got = eng.checksum(buf, 0)
    dist.barrier()
    lat = []
    ok = got == want
    t0 = time.perf_counter()
    for _ in range(max(args.steps, 20)):
        a = time.perf_counter()
        r = eng.checksum(buf, 0)
        lat.append(time.perf_counter() - a)
        ok = ok and r == want
    wall = time.perf_counter() - t0
    dist.barrier()
    lat.sort()
    med = lat[len(lat) // 2]
    # the kernel alone, buffer and descriptor resident in HBM
    arena = torch.from_numpy(buf).to(dev)
    desc = torch.from_numpy(d1.view(np.uint8).copy()).to(dev)
    out = torch.empty(1, dtype=torch.int16, device=dev)
    stream = torch.cuda.current_stream(dev)
    kern_us = b2b_us(lambda k: eng.batch_tensors(arena, desc, out, stream=stream), stream, reps=200)
    ok = ok and (int(out.cpu().numpy().view(np.uint16)[0]) == want)
    result = {
        "metric": "header.Checksum GiB/s on one 64 KiB buffer (BASELINE configs[0], plumbing)",
        "value": 65536 / med / GIB, "unit": "GiB/s", "n_gpus": dist.world,
        "steps": len(lat), "warmup": args.warmup, "ms_per_step": wall / len(lat) * 1e3,
        "higher_is_better": True, "scaling": "weak", "vs_baseline": None, "dtype": "u8",
        "data": "synthetic (splitmix64 seed 1), initial 0",
        "config": {"workload": WORKLOADS[1], "call": "ns_csum_checksum (synchronous, ctypes)"},
        "sync_call_us": {"median": med * 1e6, "min": lat[0] * 1e6, "max": lat[-1] * 1e6},
        "kernel_only_us": kern_us,
        "result": {"got": got, "want": want, "bit_exact": bool(ok)},
    }
    if dist.rank == 0 and not args.no_cpu:
        # 1 core, the scalar port: many descriptors over the one buffer, so
        # the per-call Python overhead is not what is timed
        reps_per = 2048
        dd = np.repeat(d1, reps_per)
        outc = np.zeros(reps_per, dtype=np.uint16)
        O.c_batch_mt(buf, dd, 1, outc)
        reps, t0 = 0, time.perf_counter()
        while True:
            O.c_batch_mt(buf, dd, 1, outc)
            reps += 1
            el = time.perf_counter() - t0
            if el >= args.cpu_seconds:
                break
        calls = reps * reps_per
        result["cpu_baseline"] = {
            "value": 65536 * calls / el / GIB, "unit": "GiB/s", "cores": 1, "kind": "port",
            "per_call_us": el / calls * 1e6, "bit_exact": bool((outc == want).all()),
            "sample": f"{calls} Checksum(buf, 0) calls over the one 64 KiB buffer in {el:.1f} s; "
                      "oracle/csum_oracle.c scalar 2-B/iteration loop (checksum.go:41-43), single thread"}
    if dist.rank == 0:
        print(json.dumps(result), flush=True)
    eng.close()
    dist.close()


def host_mode(args, dist, eng, batch, dev):
    """Host-inclusive rate: pinned host arena -> H2D -> kernel -> D2H,
    pipelined by ns_csum_batch_host (recorded in DESIGN.md, never `value`)."""
    import torch

    arena = torch.empty(batch.arena_bytes, dtype=torch.uint8).pin_memory()
    arena.numpy()[:] = batch.arena_host()
    a = arena.numpy()
    # the descriptor table pinned too, as a caller that builds it in place
    # would have it (a pageable table is copied into pinned staging first)
    dt = torch.empty(batch.desc.nbytes, dtype=torch.uint8).pin_memory()
    dt.numpy()[:] = batch.desc.view(np.uint8)
    d = dt.numpy().view(batch.desc.dtype)

    def step():
        eng.batch_host(a, d)

    wall, _ = timed_region(step, lambda: None, dist, args.steps, args.warmup, dev)
    total_payload = dist.sum(float(batch.payload_bytes), dev)
    if dist.rank == 0:
        print(json.dumps({
            "metric": "checksum GiB/s host-inclusive (H2D + kernel + D2H, pinned)",
            "value": total_payload * args.steps / wall / GIB, "unit": "GiB/s",
            "n_gpus": dist.world, "steps": args.steps, "warmup": args.warmup,
            "ms_per_step": wall / args.steps * 1e3, "higher_is_better": True, "scaling": "weak",
            "config": {"workload": WORKLOADS[args.config], "packets_per_gpu": batch.n,
                       "staging": "64 MiB / 128K-descriptor chunks, 4 in flight (one stream each), results written to mapped "
                                  "memory; arena and table pinned"},
        }), flush=True)
    eng.close()
    dist.close()


if __name__ == "__main__":
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    main()
