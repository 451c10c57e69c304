"""GPU: ns_csum_rx_ring_host — a receive ring in HOST memory (recvmmsg's
buffers as link/fdbased/packet_dispatchers.go:258-317 fills them), parsed
and verified on the device with no host planning.  Every slot's verdict and
sums against oracle/packets.py verify_frame (the CPU restatement of the
receive dispatch, HandlePacket/IsValid and segment.parse) and against
ns_csum_rx_ring over a device copy of the same ring: link headers, first
views, padded frames, unaligned ring offsets, small rings (written through
the BAR, no DMA), a staging budget of a few slots (chunks cycling through the
four pipeline slots), outputs one at a time, and the error paths."""

import ctypes

import numpy as np
import pytest

from test_gpu_rx_ring import _frames, _oracle, _ring, _run

pytestmark = pytest.mark.gpu


def _want(arena, lens, ring):
    w = _oracle(arena, lens, ring)
    return (np.array([x[0] for x in w], dtype=np.uint8),
            np.array([v for x in w for v in x[1:]], dtype=np.uint16))


@pytest.mark.parametrize("link_hdr,first_view,frame_at", [(0, 0, 0), (14, 128, 0), (14, 128, 10), (0, 200, 4)])
def test_host_ring_matches_oracle_and_device(engine, link_hdr, first_view, frame_at):
    rng = np.random.default_rng(5300 + link_hdr + frame_at)
    _, frames = _frames(rng, 300, link_hdr)
    stride = (max(len(f) for f in frames) + frame_at + 15) // 16 * 16
    arena, ln = _ring(frames, stride, frame_at)
    ring = dict(stride=stride, n=len(frames), frame_at=frame_at, link_hdr=link_hdr, first_view=first_view)
    verdict, sums = engine.rx_ring_host(arena, ring, ln)
    wv, ws = _want(arena, ln, ring)
    assert np.array_equal(verdict, wv) and np.array_equal(sums, ws)
    dv, ds = _run(engine, arena, ln, ring)
    assert np.array_equal(verdict, dv) and np.array_equal(sums, ds)
    assert {0, 1, 2, 3} <= set(verdict.tolist())


@pytest.mark.parametrize("n", [1, 8, 200])
def test_small_ring_through_a_bar_stage(engine, n):
    """Rings of up to ~1 MiB go through a gather stage written through the
    BAR (no DMA): the same verdicts and sums as the oracle and the device
    ring."""
    rng = np.random.default_rng(5600 + n)
    _, frames = _frames(rng, n, 14, max_payload=1400)
    arena, ln = _ring(frames, 1504, ring_off=5)
    ring = dict(ring_off=5, stride=1504, n=n, link_hdr=14, first_view=128)
    verdict, sums = engine.rx_ring_host(arena, ring, ln)
    wv, ws = _want(arena, ln, ring)
    assert np.array_equal(verdict, wv) and np.array_equal(sums, ws)


@pytest.mark.parametrize("link_hdr,first_view,ring_off", [(0, 0, 0), (14, 128, 5)])
def test_minimum_sizes(engine, link_hdr, first_view, ring_off):
    """The minimum-size rows (tests/pktgen.py MIN_SIZE; ICMPv6 8 B,
    network/ipv6/icmp.go:68) in a host ring small enough for the BAR stage:
    the oracle's verdicts and sums, the device ring's, and the reference's
    verdict table."""
    from pktgen import min_size_frames

    rng = np.random.default_rng(5960 + link_hdr)
    frames, want = min_size_frames(rng, link_hdr)
    arena, ln = _ring(frames, 128, ring_off=ring_off)
    ring = dict(ring_off=ring_off, stride=128, n=len(frames), link_hdr=link_hdr, first_view=first_view)
    verdict, sums = engine.rx_ring_host(arena, ring, ln)
    wv, ws = _want(arena, ln, ring)
    assert np.array_equal(verdict, wv) and np.array_equal(sums, ws)
    assert verdict.tolist() == want


@pytest.mark.parametrize("link_hdr,first_view", [(0, 0), (14, 128)])
def test_fuzzed_header_fields(engine, link_hdr, first_view):
    """Header fields at their boundaries (pktgen.fuzz_fields) in a host ring:
    the oracle's verdicts and sums, and the device ring's."""
    from pktgen import ethernet, fuzzed_packets

    rng = np.random.default_rng(5980 + link_hdr)
    frames = [ethernet(p) if link_hdr else p for p in fuzzed_packets(rng, 2000)]
    stride = (max(len(f) for f in frames) + 15) // 16 * 16
    arena, ln = _ring(frames, stride, ring_off=3)
    ring = dict(ring_off=3, stride=stride, n=len(frames), link_hdr=link_hdr, first_view=first_view)
    verdict, sums = engine.rx_ring_host(arena, ring, ln)
    wv, ws = _want(arena, ln, ring)
    assert np.array_equal(verdict, wv) and np.array_equal(sums, ws)
    assert {0, 1, 2, 3} <= set(verdict.tolist())


@pytest.mark.parametrize("ring_off", [0, 3, 1000])
def test_small_staging_and_unaligned_ring(oracle_mod, ring_off):
    """A staging budget of 7 slots: the ring goes up in chunks that cycle
    through the four pipeline slots; the host ring need not be 16-B aligned."""
    from netstack_amd import Engine

    rng = np.random.default_rng(5400 + ring_off)
    _, frames = _frames(rng, 333, 14, max_payload=1400)
    stride = 1504
    arena, ln = _ring(frames, stride, ring_off=ring_off)
    ring = dict(ring_off=ring_off, stride=stride, n=len(frames), link_hdr=14, first_view=128)
    with Engine(0, staging_bytes=7 * stride) as eng:
        verdict, sums = eng.rx_ring_host(arena, ring, ln)
        assert eng.sync() == 0
    wv, ws = _want(arena, ln, ring)
    assert np.array_equal(verdict, wv) and np.array_equal(sums, ws)


def test_one_output_and_errors(engine):
    from netstack_amd import _lib

    rng = np.random.default_rng(5500)
    _, frames = _frames(rng, 64, 0, max_payload=1400)
    stride = 1504
    arena, ln = _ring(frames, stride)
    ring = dict(stride=stride, n=len(frames))
    wv, ws = _want(arena, ln, ring)
    L, h = _lib.lib(), engine._h
    r = _lib.NsRxRing(0, stride, len(frames), 0, 0, 0, 0)
    v = np.zeros(len(frames), np.uint8)
    s = np.zeros(2 * len(frames), np.uint16)
    assert L.ns_csum_rx_ring_host(h, arena.ctypes.data, arena.size, ctypes.byref(r), ln.ctypes.data, None,
                                  v.ctypes.data) == _lib.NS_OK
    assert np.array_equal(v, wv)
    assert L.ns_csum_rx_ring_host(h, arena.ctypes.data, arena.size, ctypes.byref(r), ln.ctypes.data, s.ctypes.data,
                                  None) == _lib.NS_OK
    assert np.array_equal(s, ws)
    assert L.ns_csum_rx_ring_host(h, arena.ctypes.data, arena.size, ctypes.byref(r), ln.ctypes.data, None,
                                  None) == _lib.NS_EINVAL  # no output
    assert L.ns_csum_rx_ring_host(h, arena.ctypes.data, arena.size, ctypes.byref(r), None, s.ctypes.data,
                                  None) == _lib.NS_EINVAL  # no lengths
    with pytest.raises(ValueError):  # stride not a multiple of 16
        engine.rx_ring_host(arena, dict(ring, stride=1500), ln)
    with pytest.raises(_lib.ChecksumError) as e:  # past the arena
        engine.rx_ring_host(arena[:stride * len(frames) - 1], ring, ln)
    assert e.value.status == _lib.NS_ERANGE
    v0, s0 = engine.rx_ring_host(arena, dict(ring, n=0), ln)
    assert v0.size == 0 and s0.size == 0
