"""CPU: the two restatements of the receive ring's per-slot rules agree
(oracle/packets.py verify_frame, the Python one, and oracle_rx_ring in
oracle/csum_oracle.c, the C one bench.py times as the CPU baseline), and
verify_frame reduces to verify (pinned by the reference's fixtures through
tests/test_rx_contract.py) for every framing the ring supports."""
import numpy as np
import pytest

import oracle as O
import packets as P
from pktgen import ethernet, random_packet, views_bufconfig


def _ring(frames, stride, frame_at, seed):
    rng = np.random.default_rng(seed)
    arena = rng.integers(0, 256, len(frames) * stride, dtype=np.uint8)
    lens = np.zeros(len(frames), dtype=np.uint32)
    for k, f in enumerate(frames):
        f = bytes(f)[:stride - frame_at]
        arena[k * stride + frame_at:k * stride + frame_at + len(f)] = np.frombuffer(f, dtype=np.uint8)
        lens[k] = frame_at + len(f)
    return arena, lens


@pytest.mark.parametrize("link_hdr,first_view,frame_at", [(0, 0, 0), (0, 128, 0), (14, 128, 0), (14, 128, 10),
                                                           (14, 0, 4)])
def test_c_ring_matches_verify_frame(link_hdr, first_view, frame_at):
    rng = np.random.default_rng(600 + link_hdr + first_view + frame_at)
    frames = []
    for _ in range(250):
        p = random_packet(rng, 3000)
        if rng.random() < 0.3 and len(p):  # header damage
            p[int(rng.integers(0, min(len(p), 80)))] = int(rng.integers(0, 256))
        frames.append(ethernet(p, int(rng.choice([0x0800, 0x86DD, 0x0806]))) if link_hdr and rng.random() < 0.1
                      else ethernet(p) if link_hdr else bytes(p))
    stride = (max(len(f) for f in frames) + frame_at + 15) // 16 * 16
    arena, lens = _ring(frames, stride, frame_at, 1)
    lens[::37] = stride + 1  # longer than the slot
    lens[5::41] = frame_at + link_hdr  # the link header alone
    v, s = O.c_rx_ring(arena, lens, stride, len(frames), frame_at=frame_at, link_hdr=link_hdr,
                       first_view=first_view, nthreads=3)
    seen = set()
    for k in range(len(frames)):
        want = P.verify_frame(bytes(arena[k * stride:(k + 1) * stride]), int(lens[k]), frame_at, link_hdr,
                              first_view)
        assert (int(v[k]), int(s[2 * k]), int(s[2 * k + 1])) == want, k
        seen.add(want[0])
    assert seen == {P.INVALID, P.VALID, P.UNCHECKED, P.MALFORMED}


@pytest.mark.parametrize("link_hdr", [0, 14])
def test_verify_frame_is_verify_over_the_links_views(link_hdr):
    """verify_frame(BufConfig framing) == verify(the views recvMMsgDispatcher
    hands up) — the function ns_csum_packet_buffers is checked against."""
    rng = np.random.default_rng(700 + link_hdr)
    for _ in range(300):
        p = bytes(random_packet(rng, 3000))
        frame = ethernet(p) if link_hdr else p
        if not p or (not link_hdr and (p[0] >> 4) not in (4, 6)):
            continue
        vv = views_bufconfig(p, link_hdr)
        want = P.verify(b"", [bytes(v) for v in vv.Views()], vv.Size())
        assert P.verify_frame(frame, len(frame), 0, link_hdr, 128) == want


@pytest.mark.parametrize("link_hdr,first_view", [(0, 0), (0, 128), (14, 128), (0, 64)])
def test_c_ring_matches_verify_frame_on_fuzzed_fields(link_hdr, first_view):
    """Every header field the receive rules read, set to its boundaries
    (pktgen.fuzz_fields): both restatements give the same verdicts and sums."""
    from pktgen import fuzzed_packets

    rng = np.random.default_rng(900 + link_hdr + first_view)
    pk = fuzzed_packets(rng, 1500)
    frames = [ethernet(p) if link_hdr else p for p in pk]
    stride = (max(len(f) for f in frames) + 15) // 16 * 16
    arena, lens = _ring(frames, stride, 0, 2)
    v, s = O.c_rx_ring(arena, lens, stride, len(frames), link_hdr=link_hdr, first_view=first_view, nthreads=3)
    seen = set()
    for k in range(len(frames)):
        want = P.verify_frame(bytes(arena[k * stride:(k + 1) * stride]), int(lens[k]), 0, link_hdr, first_view)
        assert (int(v[k]), int(s[2 * k]), int(s[2 * k + 1])) == want, (k, pk[k][:64].hex())
        seen.add(want[0])
    assert seen == {P.INVALID, P.VALID, P.UNCHECKED, P.MALFORMED}
