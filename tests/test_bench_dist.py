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
