"""GPU: the completion word of synchronous calls (csum_kernels.hip
zc_complete, csum_api.cpp run_zero_copy; DESIGN.md §5 "The checksum launch
signals itself").  A caller spins on a word in coherent host memory and then
reads its results; the kernel's release/acquire chain is what makes every
result visible first.  These tests issue many back-to-back calls whose
expected results all differ from the previous call's, so a result read
before it landed shows as a mismatch, and check every one against the
oracle — idle, and with a device-resident batch streaming on another stream
(uneven load: MI355X_MICROARCH.md asks for hand-offs to be tested under
it)."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def _calls(engine, rng, n):
    """n back-to-back synchronous calls of mixed shapes: one workgroup
    (Checksum) and many (a VectorisedView batch of up to 400 segments, whose
    pass spreads over several workgroups, each counting itself done)."""
    import oracle as O

    bad = []
    for k in range(n):
        if k % 3 == 2:
            buf = rng.integers(0, 256, int(rng.integers(2000, 200_000)), dtype=np.uint8)
            cuts = np.sort(rng.integers(0, buf.size, 4))
            views = [buf[:cuts[0]], buf[cuts[0]:cuts[1]], buf[cuts[1]:cuts[2]], buf[cuts[2]:]]
            segs = [(int(o), int(rng.integers(1, 3000)), int(rng.integers(0, 65536)))
                    for o in rng.integers(0, buf.size, int(rng.integers(100, 400)))]
            got = engine.vv_batch(views, segs).tolist()
            vb = [bytes(v) for v in views]
            want = [O.c_checksum_vv_with_offset(vb, i, o, s) for o, s, i in segs]
            if got != want:
                bad.append((k, "vv_batch", sum(a != b for a, b in zip(got, want))))
        else:
            buf = rng.integers(0, 256, int(rng.integers(1, 3000)), dtype=np.uint8)
            ini = int(rng.integers(0, 65536))
            got = engine.checksum(buf, ini)
            if got != O.c_checksum(bytes(buf), ini):
                bad.append((k, "checksum"))
    return bad


def test_back_to_back_small_calls_every_result_fresh(engine):
    rng = np.random.default_rng(2026)
    bad = _calls(engine, rng, 3000)
    assert not bad, bad[:10]


def test_small_calls_under_uneven_load(engine):
    """The same calls while a 375 MB device-resident batch runs over and over
    on a side stream (some workgroups of a pass then wait behind it, others
    not), and the big batch itself checked afterwards."""
    import torch

    import oracle as O
    from netstack_amd import workloads as W

    n, L = 250_000, 1500
    lengths = np.full(n, L, dtype=np.uint32)
    rng = np.random.default_rng(7)
    d, end = W.make_desc(lengths, rng.integers(0, 65536, n).astype(np.uint16), align=16)
    arena = torch.randint(0, 256, (end,), dtype=torch.uint8, device="cuda")
    desc = torch.from_numpy(d.view(np.uint8).copy()).cuda()
    out = torch.zeros(n, dtype=torch.int16, device="cuda")
    side = torch.cuda.Stream()
    bad = []
    for rnd in range(4):
        for _ in range(40):
            engine.batch_tensors(arena, desc, out, stream=side)
        bad += _calls(engine, rng, 200)
    side.synchronize()
    assert not bad, bad[:10]
    host = arena.cpu().numpy()
    k = np.arange(0, n, 97)
    want, _ = O.c_batch(host, d[k])
    assert np.array_equal(out.cpu().numpy().view(np.uint16)[k], want)


def test_stats_count_calls_passes_and_reset():
    """ns_csum_get_stats (a fresh context): every synchronous call is counted
    and timed, small calls run as zero-copy passes (none late on an idle
    device), a chained device-resident batch on a new stream grows its
    scratch once, ns_csum_stream_release retires it, and reset zeroes every
    counter."""
    import torch

    from netstack_amd import Engine
    from netstack_amd import workloads as W

    eng = Engine(0)
    try:
        st = eng.stats(reset=True)
        for _ in range(20):
            eng.checksum(np.arange(1500, dtype=np.uint8), 7)
        st = eng.stats()
        assert st["calls"] == 20 and 20 >= st["zc_passes"] >= 1 and st["zc_late"] == 0, st
        assert 0 < st["call_ns_max"] < 1e9 and st["zc_pass_ns_max"] <= st["call_ns_max"], st
        lengths = np.full(1000, 100, np.uint32)
        d, end = W.make_desc(lengths, np.zeros(1000, np.uint16), align=1, flags=np.full(1000, 2, np.uint16))
        s = torch.cuda.Stream()
        eng.batch_tensors(torch.zeros(end, dtype=torch.uint8, device="cuda"),
                          torch.from_numpy(d.view(np.uint8).copy()).cuda(), chained=True, stream=s)
        s.synchronize()
        eng.stream_release(s)
        st = eng.stats(reset=True)
        assert st["growths"] >= 1 and st["retires"] == 1, st
        assert all(v == 0 for v in eng.stats().values())
    finally:
        eng.close()
