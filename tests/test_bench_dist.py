"""CPU, world_size 2 over gloo: the N>1 plumbing of bench.py (barrier-bracketed
timed region, MAX over ranks, SUM of payload) and the shard plan that splits
one batch into per-rank ranges with no collective on the data path.  The
per-rank "engine" here is the oracle (this container has no GPU); on the box
bench.py runs the HIP engine in the same structure."""
import os
import socket
import sys

import numpy as np
import pytest
import torch.multiprocessing as mp

from conftest import ROOT


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank),
                      WORLD_SIZE=str(world), LOCAL_RANK=str(rank))
    sys.path.insert(0, ROOT)
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import bench
    import oracle as O
    from netstack_amd import engine
    from netstack_amd import workloads as W

    try:
        d = bench.Dist("gloo")
        assert d.on and d.world == world and d.rank == rank
        # one global batch, byte-balanced contiguous shards
        b = W.config(4, n=6000)
        first = engine.shard_plan(b.desc, world)
        lo, hi = int(first[rank]), int(first[rank + 1])
        arena = b.arena_host()
        mine = b.desc[lo:hi]
        out = {}

        def step():
            out["r"] = O.c_batch(arena, mine)[0]

        wall, local = bench.timed_region(step, lambda: None, d, steps=3, warmup=1)
        assert wall >= local
        total = d.sum(float(mine["len"].sum()))
        d.close()
        q.put((rank, lo, hi, out["r"].tolist(), wall, total))
    except Exception as e:  # pragma: no cover - surfaced by the parent
        q.put((rank, "error", repr(e)))


def test_two_rank_gloo_sharded_bench_plumbing():
    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = [q.get(timeout=180) for _ in range(world)]
    for p in procs:
        p.join(timeout=60)
    for r in res:
        assert r[1] != "error", r
    res.sort()
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import oracle as O
    from netstack_amd import workloads as W

    b = W.config(4, n=6000)
    want = O.c_batch(b.arena_host(), b.desc)[0].tolist()
    # shards tile the batch exactly once, in order, and reproduce the whole
    assert res[0][1] == 0 and res[0][2] == res[1][1] and res[1][2] == b.n
    assert res[0][3] + res[1][3] == want
    # every rank reports the same MAX wall time and the SUM of payload
    assert res[0][4] == pytest.approx(res[1][4])
    assert res[0][5] == res[1][5] == float(b.payload_bytes)
    # byte balance of the plan
    sizes = [int(b.desc["len"][r[1]:r[2]].sum()) for r in res]
    assert abs(sizes[0] - sizes[1]) <= 9000


def test_cfg5_strong_scaling_shards_reproduce_the_whole_batch():
    """bench.py --config 5: each of N ranks takes one contiguous shard of the
    8M x 1500 B batch (here 4096 packets) with rebased offsets; the shards'
    results concatenate to the unsharded ones, and bench.parity_sample passes
    on correct results and catches a single wrong one."""
    import torch

    sys.path.insert(0, ROOT)
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import bench
    import oracle as O
    from netstack_amd import workloads as W

    whole = W.config(5, n=4096)
    arena = whole.arena_host()
    want = O.c_batch(arena, whole.desc)[0]
    for world in (1, 2, 4, 8):
        got = []
        for r in range(world):
            s = whole.shard(r, world)
            assert s.base % 8 == 0 and int(s.desc["off"].min()) < 16
            sa = s.arena_host()
            assert np.array_equal(sa, arena[s.base:s.base + s.arena_bytes])
            res = O.c_batch(sa, s.desc)[0]
            got.append(res)
            out = torch.from_numpy(res.view(np.int16).copy())
            p = bench.parity_sample(s, out, k=100)
            assert p["bit_exact"] and p["packets"] == min(200, s.n)
            bad = res.copy()
            bad[-1] ^= 1
            assert not bench.parity_sample(s, torch.from_numpy(bad.view(np.int16)), k=100)["bit_exact"]
        assert np.array_equal(np.concatenate(got), want)
    assert "true" in bench.kernel_name(12_583_000_000, 8 << 20)
    assert bench.kernel_name(1_577_058_304, 1 << 20) == "nsk::csum_hyb<256,32,8,16,4,2,0,false,2,false>"
    assert bench.kernel_name(67_108_864, 1 << 20) == "nsk::csum_hyb<64,64,16,8,4,2,5,false,1,false>"


def test_nccl_refuses_more_ranks_than_gpus():
    """Under nccl (RCCL) every local rank needs its own GPU: bench.py refuses
    a launch with more ranks on the node than GPUs, with a message, instead
    of mapping ranks modulo the device count.  gloo may share GPUs (the
    one-GPU box's multi-rank tests)."""
    import bench

    assert [bench.device_ordinal("nccl", r, 8, 8) for r in range(8)] == list(range(8))
    for local_rank, ndev, world in ((1, 1, 2), (0, 1, 2), (7, 4, 8), (2, 2, 1)):
        with pytest.raises(SystemExit) as e:
            bench.device_ordinal("nccl", local_rank, ndev, world)
        assert "one GPU per rank" in str(e.value)
    assert [bench.device_ordinal("gloo", r, 1, 8) for r in range(8)] == [0] * 8
    assert bench.device_ordinal("gloo", 5, 2, 8) == 1


def test_nccl_process_group_is_bound_to_the_rank_device(monkeypatch):
    """What a one-GPU box cannot show about the 8-GPU nccl (RCCL) run,
    pinned on CPU: bench.Dist hands init_process_group this rank's device
    (eager communicator on the right GPU) and its barrier names that device,
    while gloo passes neither; main() makes the device current before the
    process group exists, builds the engine on the same ordinal, and times
    the CPU leg only at N=1 (no rank waits on rank 0's CPU work)."""
    import inspect

    import torch
    import torch.distributed as tdist

    import bench

    calls = []
    monkeypatch.setattr(tdist, "is_initialized", lambda: False)
    monkeypatch.setattr(tdist, "init_process_group", lambda **kw: calls.append(("init", kw)))
    monkeypatch.setattr(tdist, "barrier", lambda **kw: calls.append(("barrier", kw)))
    monkeypatch.setenv("WORLD_SIZE", "8")
    monkeypatch.setenv("RANK", "5")
    monkeypatch.setenv("LOCAL_RANK", "5")
    d = bench.Dist("nccl", 5)
    d.barrier()
    assert calls[0] == ("init", {"backend": "nccl", "device_id": torch.device("cuda", 5)})
    assert calls[1] == ("barrier", {"device_ids": [5]})
    calls.clear()
    g = bench.Dist("gloo", 5)
    g.barrier()
    assert calls == [("init", {"backend": "gloo"}), ("barrier", {})]

    src = inspect.getsource(bench.main)
    i_dev, i_pg, i_eng = src.index("torch.cuda.set_device(ordinal)"), src.index("Dist(backend, ordinal)"), \
        src.index("Engine(ordinal)")
    assert i_dev < i_pg < i_eng
    assert 'elif dist.rank == 0 and not args.no_cpu' in src and "dist.world > 1" in src


@pytest.mark.parametrize("world", [1, 2, 4, 8])
def test_per_rank_device_footprint(world):
    """Per-rank HBM of the driver's scaling runs: the default
    cfg2 (weak: every rank its own 1M x 1500 B batch, distinct seeds, 2
    rotating batches + tables + results) and cfg5 (strong: 1/N of the one 8M x
    1500 B batch, 12.6 / 6.3 / 3.2 / 1.6 GB shards that tile it exactly).
    Both sit far below a 288 GB MI355X; nothing scales with N per rank except
    the cfg5 shard, which shrinks."""
    import bench
    from netstack_amd import workloads as W

    b2 = [bench.rank_batch(2, r, world) for r in range(world)]
    assert len({b.seed for b in b2}) == world and {b.n for b in b2} == {1 << 20}
    per_rank = 2 * (b2[0].arena_bytes + 16 * b2[0].n) + 2 * b2[0].n
    assert 3.1e9 < per_rank < 3.3e9
    whole = W.config(5)
    shards = [whole.shard(r, world) for r in range(world)]
    assert sum(s.n for s in shards) == 8 << 20 and {s.n for s in shards} == {(8 << 20) // world}
    total = sum(int(s.desc["len"].sum()) for s in shards)
    assert total == int(whole.desc["len"].sum())
    for s in shards:
        assert abs(s.arena_bytes - whole.arena_bytes / world) < 64
        assert s.arena_bytes + 18 * s.n < 13e9 / world


def test_cfg8_defaults_to_the_structured_tx_fill():
    """bench.py --config 8 measures ns_csum_tcp_tx over sendTCPBatch's layout
    by default; the paired table and the wire layout stay
    selectable, and the PMC entry each line reads is its own."""
    import sys

    import bench
    from netstack_amd import workloads as W

    old = sys.argv
    try:
        sys.argv = ["bench.py", "--config", "8"]
        assert bench.parse().tx_layout == "struct"
        for lay in ("split", "wire"):
            sys.argv = ["bench.py", "--config", "8", "--tx-layout", lay]
            assert bench.parse().tx_layout == lay
    finally:
        sys.argv = old
    src = open(bench.__file__).read()
    assert 'pmc_traffic(args.pmc_json, "8struct") if struct' in src
    g = W.tx_struct_geometry(1 << 20)
    pay, total = W.tx_split_layout(1 << 20)
    assert g["pay_off"] == pay and g["hdr_off"] + (1 << 20) * g["slot"] <= pay
    assert g["pay_off"] + g["size"] == total and g["tcp_at"] + g["tcp_len"] == g["slot"]


@pytest.mark.parametrize("calls", [1, 7, 23832, 1 << 20])
def test_tx_calls_tile_the_batch(calls):
    """bench.py --mode host --config 8 --tx-calls K cuts cfg8's geometry into
    K sendTCPBatch calls of consecutive segments: together they cover every
    segment once, with sendTCPBatch's own segment lengths (connect.go:679-691),
    and each call's slots and payload follow the previous call's."""
    import bench
    from netstack_amd import workloads as W

    g = W.tx_struct_geometry(1 << 20)
    parts = bench.tx_calls(g, calls)
    n = -(-g["size"] // g["mss"])
    segs = [-(-p["size"] // p["mss"]) for p in parts]
    assert sum(segs) == n and len(parts) <= calls
    assert sum(p["size"] for p in parts) == g["size"]
    hdr, pay = g["hdr_off"], g["pay_off"]
    for p, k in zip(parts, segs):
        assert p["hdr_off"] == hdr and p["pay_off"] == pay
        assert all(p[f] == g[f] for f in ("mss", "slot", "ip_at", "ip_len", "tcp_at", "tcp_len", "src", "dst"))
        hdr += k * g["slot"]
        pay += p["size"]
    assert all(p["size"] % g["mss"] == 0 for p in parts[:-1])
