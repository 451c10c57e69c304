"""GPU: ns_csum_rx_bufs — the receive ring's device-side parse and checks
(recvMMsgDispatcher.dispatch, IPv4/IPv6 HandlePacket + IsValid,
segment.parse, handleICMP) over buffers at per-packet
offsets of one arena, as a NIC's buffer pool hands them over, instead of a
fixed-stride ring.  Every buffer's verdict and sums against
oracle/packets.py verify_frame over that buffer's bytes, and against
ns_csum_rx_ring over the same frames in ring order; buffers in shuffled
order with gaps, link headers and first views, a nonzero ring_off, and
buffers that are misaligned or reach past the arena (MALFORMED, sums 0,
counted by ns_csum_sync)."""

import numpy as np
import pytest

from test_gpu_rx_ring import _frames, _ring, _run

pytestmark = pytest.mark.gpu


def _pool(frames, cap, seed, ring_off=0):
    """An arena of random bytes holding each frame in a buffer of `cap` bytes
    at a shuffled, 16-B-aligned offset with random gaps between buffers.
    Returns (arena, offsets from ring_off, lengths)."""
    rng = np.random.default_rng(seed)
    n = len(frames)
    order = rng.permutation(n)
    offs = np.zeros(max(n, 1), dtype=np.uint32)
    pos = 0
    for k in order:
        pos += 16 * int(rng.integers(0, 8))
        offs[k] = pos
        pos += cap
    arena = rng.integers(0, 256, ring_off + pos + 64, dtype=np.uint8)
    lens = np.zeros(max(n, 1), dtype=np.uint32)
    for k, f in enumerate(frames):
        f = bytes(f)[:cap]
        at = ring_off + int(offs[k])
        arena[at:at + len(f)] = np.frombuffer(f, dtype=np.uint8)
        lens[k] = len(f)
    return arena, offs, lens


def _want(arena, offs, lens, ring):
    import packets as P

    cap, off0 = ring["stride"], ring.get("ring_off", 0)
    v, s = [], []
    for k in range(ring["n"]):
        at = off0 + int(offs[k])
        r = P.verify_frame(bytes(arena[at:at + cap]), int(lens[k]), ring.get("frame_at", 0), ring.get("link_hdr", 0),
                           ring.get("first_view", 0))
        v.append(r[0])
        s += [r[1], r[2]]
    return np.array(v, dtype=np.uint8), np.array(s, dtype=np.uint16)


def _run_bufs(engine, arena, offs, lens, ring):
    import torch

    dev = torch.device("cuda", 0)
    a = torch.from_numpy(arena).to(dev)
    o = torch.from_numpy(offs.view(np.int32)).to(dev)
    ln = torch.from_numpy(lens.view(np.int32)).to(dev)
    verdict, sums = engine.rx_bufs(a, ring, o, ln)
    torch.cuda.synchronize()
    n = ring["n"]
    return verdict[:n].cpu().numpy(), sums[:2 * n].cpu().numpy().view(np.uint16)


@pytest.mark.parametrize("link_hdr,first_view,ring_off", [(0, 0, 0), (14, 128, 0), (14, 128, 48), (0, 200, 16)])
def test_pool_matches_oracle_and_ring(engine, link_hdr, first_view, ring_off):
    rng = np.random.default_rng(5700 + link_hdr + ring_off)
    _, frames = _frames(rng, 400, link_hdr)
    cap = (max(len(f) for f in frames) + 15) // 16 * 16
    arena, offs, lens = _pool(frames, cap, seed=5701 + ring_off, ring_off=ring_off)
    ring = dict(ring_off=ring_off, stride=cap, n=len(frames), link_hdr=link_hdr, first_view=first_view)
    verdict, sums = _run_bufs(engine, arena, offs, lens, ring)
    wv, ws = _want(arena, offs, lens, ring)
    assert np.array_equal(verdict, wv) and np.array_equal(sums, ws)
    assert {0, 1, 2, 3} <= set(verdict.tolist())
    # the same frames as a fixed-stride ring: the same answers
    ra, rl = _ring(frames, cap)
    rv, rs = _run(engine, ra, rl, dict(stride=cap, n=len(frames), link_hdr=link_hdr, first_view=first_view))
    assert np.array_equal(verdict, rv) and np.array_equal(sums, rs)
    assert engine.sync() == 0


@pytest.mark.parametrize("link_hdr,first_view", [(0, 0), (14, 128)])
def test_minimum_sizes(engine, link_hdr, first_view):
    """The minimum-size rows (tests/pktgen.py MIN_SIZE; ICMPv6 8 B,
    network/ipv6/icmp.go:68) from a shuffled pool: the oracle's verdicts and
    sums, and the reference's verdict table."""
    from pktgen import min_size_frames

    rng = np.random.default_rng(5950 + link_hdr)
    frames, want = min_size_frames(rng, link_hdr)
    arena, offs, lens = _pool(frames, 128, seed=5951, ring_off=16)
    ring = dict(ring_off=16, stride=128, n=len(frames), link_hdr=link_hdr, first_view=first_view)
    verdict, sums = _run_bufs(engine, arena, offs, lens, ring)
    wv, ws = _want(arena, offs, lens, ring)
    assert np.array_equal(verdict, wv) and np.array_equal(sums, ws)
    assert verdict.tolist() == want


@pytest.mark.parametrize("link_hdr,first_view", [(0, 128), (14, 128)])
def test_fuzzed_header_fields(engine, link_hdr, first_view):
    """Header fields at their boundaries (pktgen.fuzz_fields) from a shuffled
    pool: the oracle's verdicts and sums."""
    from pktgen import ethernet, fuzzed_packets

    rng = np.random.default_rng(5970 + link_hdr)
    frames = [ethernet(p) if link_hdr else p for p in fuzzed_packets(rng, 2000)]
    cap = (max(len(f) for f in frames) + 15) // 16 * 16
    arena, offs, lens = _pool(frames, cap, seed=5971, ring_off=32)
    ring = dict(ring_off=32, stride=cap, n=len(frames), link_hdr=link_hdr, first_view=first_view)
    verdict, sums = _run_bufs(engine, arena, offs, lens, ring)
    wv, ws = _want(arena, offs, lens, ring)
    assert np.array_equal(verdict, wv) and np.array_equal(sums, ws)
    assert {0, 1, 2, 3} <= set(verdict.tolist())


def test_bad_buffers_are_malformed_and_counted(engine):
    rng = np.random.default_rng(5800)
    _, frames = _frames(rng, 64, 14, max_payload=1400)
    cap = 1504
    arena, offs, lens = _pool(frames, cap, seed=5801)
    ring = dict(stride=cap, n=len(frames), link_hdr=14, first_view=128)
    bad = {3: offs[3] + 8, 17: arena.size - cap + 16, 40: 0xFFFFFFF0}  # misaligned, past the end, far past
    for k, o in bad.items():
        offs[k] = o
    verdict, sums = _run_bufs(engine, arena, offs, lens, ring)
    assert engine.sync() == len(bad)
    for k in range(len(frames)):
        if k in bad:
            assert verdict[k] == 3 and sums[2 * k] == 0 and sums[2 * k + 1] == 0, k
    good = [k for k in range(len(frames)) if k not in bad]
    wv, ws = _want(arena, offs[good], lens[good], dict(ring, n=len(good)))
    assert np.array_equal(verdict[good], wv)
    assert np.array_equal(sums.reshape(-1, 2)[good].reshape(-1), ws)


def test_errors(engine):
    import ctypes

    import torch

    from netstack_amd import _lib

    L, h = _lib.lib(), engine._h
    a = torch.zeros(4096, dtype=torch.uint8, device="cuda")
    o = torch.zeros(4, dtype=torch.int32, device="cuda")
    ln = torch.zeros(4, dtype=torch.int32, device="cuda")
    v = torch.zeros(4, dtype=torch.uint8, device="cuda")

    def call(stride=1504, n=4, ring_off=0, off=o, lens=ln, verdict=v, arena_bytes=4096):
        r = _lib.NsRxRing(ring_off, stride, n, 0, 0, 0, 0)
        return L.ns_csum_rx_bufs(h, a.data_ptr(), arena_bytes, ctypes.byref(r),
                                 off.data_ptr() if off is not None else None,
                                 lens.data_ptr() if lens is not None else None, None,
                                 verdict.data_ptr() if verdict is not None else None, None)

    assert call() == _lib.NS_OK
    assert call(stride=1500) == _lib.NS_EINVAL  # not a multiple of 16
    assert call(off=None) == _lib.NS_EINVAL
    assert call(lens=None) == _lib.NS_EINVAL
    assert call(verdict=None) == _lib.NS_EINVAL  # no output at all
    assert call(ring_off=8) == _lib.NS_EINVAL  # arena + ring_off not 16-B aligned
    assert call(ring_off=8192) == _lib.NS_ERANGE
    assert call(n=0, off=None, lens=None) == _lib.NS_OK
    torch.cuda.synchronize()
    # those buffers lie inside the arena (empty frames: MALFORMED, not counted)
    assert engine.sync() == 0
    assert (v.cpu().numpy() == 3).all()
