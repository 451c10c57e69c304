"""CPU: the receive path's packet-level semantics against the reference's own
test fixtures (tests/golden/rx_fixtures.json): the oracle's per-packet
verdicts (oracle/packets.py) and the receive-contract mirror
(netstack_amd/rx.py) on IsValid, HandlePacket's fragment checks, reassembly
and the transmit-side fragmenter.  The checksum sums themselves are GPU work
(tests/test_gpu_rx_contract.py); nothing here calls the engine."""
import struct

import pytest

import rxcases as R


@pytest.fixture(scope="module")
def fx(oracle_mod):
    return R.fixtures()


def _pk(b: bytes):
    from netstack_amd.buffer import NewVectorisedView, View
    from netstack_amd.packet import PacketBuffer

    return PacketBuffer(Data=NewVectorisedView(len(b), [View(bytearray(b))]))


def test_invalid_fragments_counts_match_the_reference(fx):
    """TestInvalidFragments (ipv4_test.go:360-481): every case's packets,
    injected in order, give the reference's MalformedPacketsReceived and
    MalformedFragmentsReceived counts through the mirror's network layer."""
    from netstack_amd.rx import ReceivePath

    for case in fx["invalid_fragments"]:
        rp = ReceivePath(engine=object())  # the network layer never calls the engine
        for p in case["packets"]:
            assert rp.network(_pk(bytes.fromhex(p))) is None
        assert rp.stats.IPMalformedPacketsReceived == case["malformed_ip"], case["name"]
        assert rp.stats.IPMalformedFragmentsReceived == case["malformed_fragments"], case["name"]


def test_invalid_fragments_per_packet_verdicts(fx):
    """The per-packet checks (what one device pass can decide) agree with the
    mirror: a packet is MALFORMED in oracle/packets.py iff, arriving alone,
    HandlePacket drops it as malformed; a valid fragment is UNCHECKED."""
    import packets as P

    from netstack_amd.rx import ReceivePath

    seen = set()
    for case in fx["invalid_fragments"]:
        for p in case["packets"]:
            b = bytes.fromhex(p)
            rp = ReceivePath(engine=object())
            rp.network(_pk(b))
            v, _, _ = P.verify(b"", [b], len(b))
            assert (v == P.MALFORMED) == (rp.stats.IPMalformedPacketsReceived == 1), (case["name"], p)
            if v != P.MALFORMED:
                assert v == P.UNCHECKED, case["name"]  # fragments and a truncated-TCP-less packet
            seen.add(v)
    assert seen == {P.MALFORMED, P.UNCHECKED}


def test_fragment_edge_verdicts():
    """ipv4.go:355-373 on the edges: no payload with MF or an offset is
    malformed; at the highest offset (65528) 8 bytes end at 0xffff (kept),
    9 bytes wrap (malformed); a last fragment (offset, no MF) is kept."""
    import packets as P

    def frag(field, size, mf=False):
        h = bytearray(20)
        struct.pack_into(">BBHHHBBH4s4s", h, 0, 0x45, 0, 20 + size, 7, (0x2000 if mf else 0) | field, 64, 6, 0,
                         b"\x0a\0\0\1", b"\x0a\0\0\2")
        return bytes(h) + bytes(range(size))

    cases = [(frag(0, 0, True), P.MALFORMED), (frag(5, 0), P.MALFORMED), (frag(0x1FFF, 8), P.UNCHECKED),
             (frag(0x1FFF, 9), P.MALFORMED), (frag(0x1FFF, 9, True), P.MALFORMED), (frag(3, 100), P.UNCHECKED),
             (frag(0, 100, True), P.UNCHECKED), (frag(0x1FFE, 16), P.UNCHECKED), (frag(0x1FFE, 17), P.MALFORMED)]
    for b, want in cases:
        assert P.verify(b"", [b], len(b))[0] == want, b[:8].hex()


def test_reassembler_holes_and_process(fx):
    """TestUpdateHoles (reassembler_test.go:28-111) and
    TestFragmentationProcess (fragmentation_test.go:50-98) on the mirror's
    reassembler."""
    from netstack_amd.buffer import NewVectorisedView, View
    from netstack_amd.rx import _Reassembler

    for c in fx["holes"]:
        r = _Reassembler()
        for first, last, more in c["in"]:
            r.process(first, last, more, NewVectorisedView(0, []))
        assert [list(h) for h in r.holes] == c["want"]
    for c in fx["process"]:
        rs = {}
        for (ident, first, last, more, pieces), (done, want) in zip(c["in"], c["out"]):
            views = [View(bytearray(p.encode())) for p in pieces]
            r = rs.setdefault(ident, _Reassembler())
            vv, ok = r.process(first, last, more, NewVectorisedView(sum(map(len, views)), views))
            assert ok
            assert (vv is not None) == done
            if done:
                del rs[ident]
                assert [bytes(v).decode() for v in vv.Views()] == want and vv.Size() == sum(map(len, want))


def test_fragmentation_table_shapes(fx):
    """TestFragmentation's table (ipv4_test.go:257-320): the restated
    writePacketFragments gives the reference's fragment counts, every
    fragment a valid IPv4 header summing to 0xffff within the MTU, and the
    fragments reassemble (through the mirror) to the source payload."""
    import random

    import oracle as O

    from netstack_amd.buffer import NewVectorisedView, View
    from netstack_amd.packet import PacketBuffer
    from netstack_amd.rx import ReceivePath

    rnd = random.Random(257)
    for row in fx["fragmentation"]:
        sizes = R.view_sizes(row["views"])
        rest = bytes(rnd.getrandbits(8) for _ in range(row["hdr_length"]))
        views = [bytes(rnd.getrandbits(8) for _ in range(s)) for s in sizes]
        total = 20 + len(rest) + sum(sizes)
        ip = bytearray(20)
        struct.pack_into(">BBHHHBBH4s4s", ip, 0, 0x45, 0, total, 1, 0, 42, 6, 0, b"\x10\0\0\1", b"\x10\0\0\2")
        frags = R.write_packet_fragments(bytes(ip) + rest, views, row["mtu"])
        assert len(frags) == row["expected_frags"], row["name"]
        rp = ReceivePath(engine=object())
        got = None
        for h, d in frags:
            wire = h + b"".join(d)
            assert len(wire) <= row["mtu"] and O.c_checksum(h[:20], 0) == 0xFFFF, row["name"]
            pk = PacketBuffer(Data=NewVectorisedView(len(wire), [View(bytearray(wire))]))
            r = rp._ipv4(pk)
            if r is not None:
                got = b"".join(bytes(v) for v in r[3].Data.Views())[:r[3].Data.Size()]
        assert got == rest + b"".join(views), row["name"]
        assert rp.stats.IPMalformedPacketsReceived == 0


def test_fill_writes_only_the_ip_checksum_of_a_fragment():
    """A fragment on transmit gets its IPv4 header checksum only
    (writePacketFragments, ipv4.go:159-160): oracle.fill leaves the
    transport bytes as they are."""
    import packets as P

    seg = R.build_segment(b"\x0a\0\0\2", b"\x0a\0\0\1", 4096, 1235, 790, 1, 0x10, 30000, bytes(range(256)) * 8)
    frags = R.write_packet_fragments(bytes(seg[:20]), [bytes(seg[20:])], 800, set_checksums=False)
    for h, d in frags:
        out, net, tr = P.fill(h, d, sum(map(len, d)))
        assert tr == 0 and out[:10] == h[:10] and out[12:] == h[12:]
        assert (~net) & 0xFFFF == struct.unpack_from(">H", out, 10)[0]


def test_transport_step_trusts_the_link_verdict():
    """Contract step 3 without the engine: VALID and INVALID verdicts decide
    csumValid with no sum taken, and INVALID is counted where tcp
    HandlePacket counts it (endpoint.go:2108-2114), at every level."""
    from netstack_amd.rx import RX_CHECKSUM_INVALID, RX_CHECKSUM_VALID, ReceivePath

    seg = R.build_segment(b"\x0a\0\0\2", b"\x0a\0\0\1", 4096, 1235, 790, 1, 0x10, 30000, b"\x01\x02\x03")
    good, bad = _pk(bytes(seg)), _pk(bytes(seg))
    good.RXChecksum, bad.RXChecksum = RX_CHECKSUM_VALID, RX_CHECKSUM_INVALID
    rp = ReceivePath(engine=object())
    segs = [rp.network(good), rp.network(bad)]
    out = rp.transport(segs)
    assert [o[2] for o in out] == [bytes(seg[20:])]
    s = rp.stats
    assert (s.TCPChecksumErrors, s.EndpointChecksumErrors, s.TCPValidSegmentsReceived) == (1, 1, 1)


def test_reassembly_clears_a_fragment_verdict():
    """Contract step 2: a reassembled packet never carries a fragment's
    verdict (were a link to mark a fragment VALID, the reassembled segment
    would still be verified)."""
    from netstack_amd.rx import RX_CHECKSUM_UNKNOWN, RX_CHECKSUM_VALID, ReceivePath

    seg = R.build_segment(b"\x0a\0\0\2", b"\x0a\0\0\1", 4096, 1235, 790, 1, 0x10, 30000, bytes(2000))
    frags = R.write_packet_fragments(bytes(seg[:20]), [bytes(seg[20:])], 600)
    rp = ReceivePath(engine=object())
    last = None
    for h, d in frags:
        pk = _pk(h + b"".join(d))
        pk.RXChecksum = RX_CHECKSUM_VALID
        last = rp.network(pk)
    assert last is not None and last[2].RXChecksum == RX_CHECKSUM_UNKNOWN


def _choices():
    import json
    import os

    with open(os.path.join(os.path.dirname(__file__), "golden", "rx_choices.json")) as f:
        return json.load(f)["ipv4_header_past_first_view"]


def test_ipv4_header_past_the_first_view_is_malformed():
    """tests/golden/rx_choices.json: an IPv4 header longer than
    Data.First() — where the reference reslices into the view's spare
    capacity or panics (network/ipv4/ipv4.go:348) — is MALFORMED in the
    oracle, with no sums; the same header within its view verifies."""
    import packets as P

    cases = _choices()
    assert len(cases) == 4
    for c in cases:
        views = [bytes.fromhex(v) for v in c["views"]]
        assert P.verify(b"", views, c["size"]) == (c["verdict"], c["ipv4_sum"], c["transport_sum"]), c["name"]


def test_ipv6_receive_packets_verify(fx):
    """The IPv6 packets network/ipv6's tests inject (ipv6_test.go:40-225
    testReceiveICMP/testReceiveUDP, ndp_test.go:75-372 NDP hop-limit and RA
    validation — odd-length and 8-B ICMPv6 among them) get the fixture's
    verdict from both restatements, as one view, in the link's BufConfig
    views (TUN and Ethernet), and the link's sums as the Python oracle's."""
    import packets as P

    rows = R.ipv6_rows(fx)
    assert len(rows) == 46 and {r[2] for r in rows} == {P.VALID, P.INVALID, P.UNCHECKED}
    _both_restatements(rows)


def test_receive_control_packets_verify(fx):
    """TestIPv4ReceiveControl / TestIPv6ReceiveControl (network/ip_test.go:
    293-398, :534-650): ICMP errors cut 10 B short, at the inner header, at
    the 'extra info', at the ICMP header, to nothing.  An ICMP message under
    8 B is dropped before any checksum (MALFORMED), a cut ICMPv6 message
    fails its checksum (INVALID), a non-echo ICMPv4 one is never checked
    (UNCHECKED); every packet the reference hands on is VALID or UNCHECKED."""
    import packets as P

    rows = R.control_rows(fx)
    assert len(rows) == 18 and {r[2] for r in rows} == {P.VALID, P.INVALID, P.UNCHECKED, P.MALFORMED}
    _both_restatements(rows)


def _both_restatements(rows):
    """packets.verify on the packet as one view; packets.verify_frame and the
    C oracle_rx_ring on TUN and Ethernet rings (first view 128): the row's
    verdict, and the same sums from both."""
    import numpy as np

    import oracle as O
    import packets as P
    from pktgen import ethernet

    for name, b, want in rows:
        assert P.verify(b"", [b] if b else [], len(b))[0] == want, name
    for link_hdr in (0, 14):
        frames = [ethernet(b) if link_hdr else b for _, b, _ in rows]
        stride = 128
        arena = np.random.default_rng(6).integers(0, 256, len(frames) * stride, dtype=np.uint8)
        lens = np.zeros(len(frames), dtype=np.uint32)
        for k, f in enumerate(frames):
            arena[k * stride:k * stride + len(f)] = np.frombuffer(f, dtype=np.uint8)
            lens[k] = len(f)
        v, s = O.c_rx_ring(arena, lens, stride, len(frames), link_hdr=link_hdr, first_view=128)
        for k, (name, _, want) in enumerate(rows):
            py = P.verify_frame(bytes(arena[k * stride:(k + 1) * stride]), int(lens[k]), 0, link_hdr, 128)
            assert py[0] == want and (int(v[k]), int(s[2 * k]), int(s[2 * k + 1])) == py, (name, link_hdr)


def test_fill_reproduces_the_reference_tests_checksums(fx):
    """The transmit restatement (packets.fill: sendUDP's and ICMPv6Checksum's
    rules) writes into each fixture packet, its checksum field zeroed, the
    very checksum the reference's own test computed for it (ipv6_test.go,
    ndp_test.go, ip_test.go; tests/rxcases.py fill_rows)."""
    import packets as P

    rows = R.fill_rows(fx)
    assert len(rows) == 23 + 4
    for name, zeroed, want in rows:
        assert P.fill(zeroed, [], 0)[0] == want, name

