"""CPU: the receive path's minimum-size rules, one row per protocol and first-
view length, each asserted against the reference line that sets it (the
table is tests/pktgen.py MIN_SIZE):

  IPv4   first view < 20 → dropped   stack/nic.go:774, header/ipv4.go:281
  IPv6   first view < 40 → dropped   stack/nic.go:774, header/ipv6.go:208
  TCP    first view < 20 → dropped   stack/nic.go:851; segment.go:159
  UDP    first view < 8  → dropped   stack/nic.go:851 (no checksum otherwise)
  ICMPv4 first view < 8  → dropped   network/ipv4/icmp.go:60
  ICMPv6 first view < 8  → dropped   network/ipv6/icmp.go:68 (ICMPv6MinimumSize,
                                     header/icmpv6.go:35 — not the 4-B
                                     ICMPv6HeaderSize of :32)

Both restatements are held to it: oracle/packets.py (verify, verify_frame)
and oracle_rx_verify in oracle/csum_oracle.c (through oracle_rx_ring), for
whole messages in one view, in TUN and Ethernet frames with the link's
BufConfig views, and for longer messages whose first view is cut at every
length.  The device paths are held to the same rows in tests/test_gpu_rx_*.py
and tests/test_gpu_packet.py."""
import numpy as np
import pytest

import oracle as O
import packets as P
from pktgen import MIN_SIZE, ethernet, min_size_verdict, short_message, short_messages


def _c_verdicts(frames, link_hdr, first_view):
    stride = (max(len(f) for f in frames) + 15) // 16 * 16
    arena = np.random.default_rng(1).integers(0, 256, len(frames) * stride, dtype=np.uint8)
    lens = np.zeros(len(frames), dtype=np.uint32)
    for k, f in enumerate(frames):
        arena[k * stride:k * stride + len(f)] = np.frombuffer(bytes(f), dtype=np.uint8)
        lens[k] = len(f)
    v, s = O.c_rx_ring(arena, lens, stride, len(frames), link_hdr=link_hdr, first_view=first_view)
    return [(int(v[k]), int(s[2 * k]), int(s[2 * k + 1])) for k in range(len(frames))], arena, lens, stride


def test_the_table_names_the_reference_constants():
    assert MIN_SIZE == {"tcp": 20, "udp": 8, "icmp4": 8, "icmp6": 8}


@pytest.mark.parametrize("link_hdr,first_view", [(0, 0), (0, 128), (14, 128), (14, 0), (0, 64), (14, 78)])
def test_whole_messages(link_hdr, first_view):
    """Messages of 0 .. minimum + 2 bytes: under the minimum MALFORMED, from
    it the checksum's verdict (UNCHECKED for UDP), in both restatements."""
    rng = np.random.default_rng(8000 + link_hdr + first_view)
    rows = short_messages(rng)
    frames = [ethernet(p) if link_hdr else bytes(p) for _, _, _, p in rows]
    got, arena, lens, stride = _c_verdicts(frames, link_hdr, first_view)
    seen = set()
    for k, (kind, v6, length, p) in enumerate(rows):
        want = min_size_verdict(kind, length)
        py = P.verify_frame(bytes(arena[k * stride:(k + 1) * stride]), int(lens[k]), 0, link_hdr, first_view)
        assert py[0] == want, (kind, v6, length, py)
        assert got[k] == py, (kind, v6, length, got[k], py)
        assert P.verify(b"", [bytes(p)], len(p))[0] == want
        seen.add((kind, v6, want))
    # every protocol shows both sides of its gate
    assert {(k, v, 3) for k, v, _ in seen} <= seen


@pytest.mark.parametrize("kind,v6", [("tcp", False), ("tcp", True), ("udp", False), ("udp", True),
                                     ("icmp4", False), ("icmp6", True)])
def test_first_view_cut_at_every_length(kind, v6):
    """A well-formed message of minimum + 40 bytes whose transport first view
    is cut at 1 .. minimum + 2 bytes (the rest in a second view): the gate is
    on the first view, not the message.  ICMPv6 sums its views with a restart
    each (icmpv6.go:214-216), so an odd cut changes the sum: VALID at even
    cuts, whatever the restatement gives at odd ones (INVALID or, rarely,
    VALID), never MALFORMED."""
    rng = np.random.default_rng(8100 + MIN_SIZE[kind] + v6)
    ipl = 40 if v6 else 20
    for cut in range(1, MIN_SIZE[kind] + 3):
        p = bytes(short_message(rng, kind, MIN_SIZE[kind] + 40, v6))
        views = [p[:ipl + cut], p[ipl + cut:]]
        v = P.verify(b"", views, len(p))[0]
        want = min_size_verdict(kind, cut)
        if kind == "icmp6" and cut >= 8 and cut % 2:
            assert v in (P.VALID, P.INVALID), (cut, v)
        else:
            assert v == want, (cut, v, want)
        # the C restatement with the same cut (the link's first view)
        got, _, _, _ = _c_verdicts([p], 0, ipl + cut)
        assert got[0] == P.verify_frame(p, len(p), 0, 0, ipl + cut), cut
        assert got[0][0] == v, cut


@pytest.mark.parametrize("v6", [False, True])
def test_network_header_first_view(v6):
    """The IP header against the packet's first view (IsValid on
    Data.First()): a first view under 20 / 40 bytes is MALFORMED however long
    the packet; at exactly the header the view is trimmed away whole and the
    TCP segment's first view is the next one (VALID); one or two bytes past
    it, the TCP first view is 1-2 bytes (MALFORMED, nic.go:851)."""
    rng = np.random.default_rng(8200 + v6)
    ipl = 40 if v6 else 20
    for cut in range(1, ipl + 3):
        p = bytes(short_message(rng, "tcp", 60, v6))
        v = P.verify(b"", [p[:cut], p[cut:]], len(p))[0]
        want = P.MALFORMED if cut < ipl or cut > ipl else P.VALID
        assert v == want, (cut, v)
        got, _, _, _ = _c_verdicts([p], 0, cut)
        assert got[0][0] == v, cut


def test_icmpv6_header_size_is_not_the_gate():
    """4-7-B ICMPv6 messages (a whole ICMPv6HeaderSize, less than
    ICMPv6MinimumSize) are dropped before any checksum, whatever their
    checksum field says — the case round 5's restatements got wrong."""
    rng = np.random.default_rng(8300)
    for length in range(4, 8):
        p = short_message(rng, "icmp6", length)
        for field in (0, 0xFFFF, int(rng.integers(0, 65536))):
            p[42:44] = field.to_bytes(2, "big")
            assert P.verify(b"", [bytes(p)], len(p)) == (P.MALFORMED, 0, 0)
            got, _, _, _ = _c_verdicts([bytes(p)], 0, 0)
            assert got[0] == (P.MALFORMED, 0, 0)
