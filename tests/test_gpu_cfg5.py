"""GPU: BASELINE.json configs[4] (cfg5: 8,388,608 x 1500 B split over N GPUs,
SURVEY §8(d) Cfg 5 / §8(e)) on the HIP engine — the shards bench.py --config 5
gives each rank, every result against the oracle; the whole 12.6 GB batch on
one GPU (per-tile SRD windows); and bench.py itself as a world-size-2 job with
the real engine in both ranks (two processes on the one GPU, gloo control
plane: RCCL refuses two ranks on one device)."""
import json
import os
import socket
import subprocess
import sys

import numpy as np
import pytest

from conftest import ROOT

pytestmark = pytest.mark.gpu


def _run_shard(engine, b):
    import torch

    import oracle as O

    arena = b.arena_device("cuda")
    desc = torch.from_numpy(b.desc.view(np.uint8).copy()).cuda()
    out = engine.batch_tensors(arena, desc)
    torch.cuda.synchronize()
    assert engine.sync() == 0
    got = out.cpu().numpy().view(np.uint16)
    host = arena.cpu().numpy()
    del arena, desc, out
    torch.cuda.empty_cache()
    want = O.c_batch_mt(host, b.desc, min(16, os.cpu_count() or 1))
    return got, want


@pytest.mark.slow
@pytest.mark.parametrize("world", [2, 4, 8])
def test_cfg5_first_and_last_shards(engine, world):
    """bench.rank_batch(5, r, N) for r = 0 and N-1 (4M, 2M, 1M packets per
    shard; shard arenas of 6.3 / 3.2 / 1.6 GB): every result bit-exact."""
    sys.path.insert(0, ROOT)
    import bench

    for r in (0, world - 1):
        b = bench.rank_batch(5, r, world)
        assert b.n == (8 << 20) // world
        got, want = _run_shard(engine, b)
        assert np.array_equal(got, want), (world, r, int((got != want).sum()))


@pytest.mark.slow
def test_cfg5_whole_batch_on_one_gpu(engine):
    """The unsharded 8M x 1500 B batch (12.6 GB arena, above the 4 GiB of one
    buffer resource: per-tile SRD windows), every result against the oracle."""
    sys.path.insert(0, ROOT)
    import bench

    b = bench.rank_batch(5, 0, 1)
    assert b.n == 8 << 20 and b.arena_bytes > 2 * (4 << 30)
    got, want = _run_shard(engine, b)
    assert np.array_equal(got, want), int((got != want).sum())


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


@pytest.mark.slow
@pytest.mark.parametrize("config,world", [(5, 2), (2, 2), (5, 4), (5, 8), (2, 8)])
def test_bench_multi_rank_with_the_hip_engine(config, world):
    """bench.py under torch.distributed.run with 2, 4 and 8 ranks, each
    running the HIP engine on its own batch (cfg2: weak scaling, 8 ranks =
    BASELINE configs[4]'s 8M x 1500 B) or shard (cfg5: strong scaling, 8
    shards of 1.6 GB) — all on this box's one GPU, with the gloo control
    plane (RCCL refuses two ranks on one device; bench.py refuses that under
    nccl, tests/test_bench_dist.py).  The JSON line reports every rank, the
    summed payload and every rank's parity sample bit-exact.  The 8-GPU
    scaling curve itself is the driver's (SCALE_rNN.json)."""
    env = dict(os.environ, MASTER_ADDR="127.0.0.1", PYTHONUNBUFFERED="1")
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", str(world),
           "--master-addr", "127.0.0.1", "--master-port", str(_free_port()),
           os.path.join(ROOT, "bench.py"), "--gpus", str(world), "--config", str(config), "--steps", "3",
           "--warmup", "1", "--no-cpu", "--dist-backend", "gloo"]
    r = subprocess.run(cmd, cwd=ROOT, env=env, capture_output=True, text=True, timeout=600)
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-4000:]
    lines = [l for l in r.stdout.splitlines() if l.startswith("{")]
    assert len(lines) == 1, r.stdout  # rank 0 prints one line
    res = json.loads(lines[0])
    assert res["n_gpus"] == world and res["value"] > 0
    assert res["scaling"] == ("strong" if config == 5 else "weak")
    assert res["config"]["global_packets"] == (8 << 20 if config == 5 else world << 20)
    ps = res["parity_sample"]
    assert ps["bit_exact"] and ps["ranks_checked"] == world and ps["ranks_failed"] == 0
    assert res["bad_descriptors"] == 0
