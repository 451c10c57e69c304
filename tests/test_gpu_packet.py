"""GPU: tcpip.PacketBuffer batches through
ns_csum_packet_buffers, every packet against oracle/packets.py (the
reference's receive and transmit call sequences restated on the oracle):

* receive — recvmmsg batches as recvMMsgDispatcher builds them
  (link/fdbased/packet_dispatchers.go:258-317: BufConfig views, capped, the
  link header trimmed): IPv4/IPv6 TCP segments (segment.parse), ICMPv4 echo
  requests, ICMPv6, UDP and fragments (not verified by the reference),
  malformed packets, and corrupted members (tcp_test.go:3246-3254);
* transmit — Header Prependables holding IPv4/IPv6 + TCP/UDP/ICMP headers
  over payload views: every checksum field written as buildTCPHdr, sendUDP,
  the echo reply, ICMPv6Checksum and addIPHeader write it, byte for byte.
"""
import struct

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

from pktgen import BUF_CONFIG  # noqa: F401
from pktgen import frag_packet as _frag_packet
from pktgen import ip4 as _ip4
from pktgen import ip6 as _ip6
from pktgen import tcp_header as _tcp
from pktgen import valid_packet as _valid_packet
from pktgen import views_bufconfig as _views_bufconfig


def _rx_batch(rng, n):
    """A recvmmsg-like batch: mostly TCP (v4/v6) of 0..9000-B payloads,
    plus ICMPv4/v6, UDP, fragments, malformed packets; ~1/7 of the valid ones
    get one corrupted byte."""
    from netstack_amd.packet import PacketBuffer

    pkts = []
    for i in range(n):
        r = rng.random()
        kind = "tcp4" if r < 0.45 else "tcp6" if r < 0.65 else "icmp4" if r < 0.72 else \
            "icmp6" if r < 0.79 else "udp4" if r < 0.85 else "frag" if r < 0.88 else "bad"
        plen = int(rng.choice([0, 1, 7, int(rng.integers(0, 1460)), int(rng.integers(0, 9000))]))
        if kind == "frag":
            p = _frag_packet(rng, int(rng.integers(0, 6)), plen)
        elif kind == "bad":
            p = _valid_packet(rng, "tcp4", plen)
            how = int(rng.integers(0, 4))
            if how == 0:
                p = p[:int(rng.integers(1, 20))]                 # shorter than an IPv4 header
            elif how == 1:
                p[0] = 0x43                                      # IHL 12 < 20
            elif how == 2:
                struct.pack_into(">H", p, 2, len(p) + 1)         # TotalLength past the packet
            else:
                p[20 + 12] = 0x40                                # TCP data offset 16 < 20
        else:
            p = _valid_packet(rng, kind, plen)
            if rng.random() < 1 / 7 and len(p) > 0:
                k = int(rng.integers(0, len(p)))
                p[k] ^= int(rng.integers(1, 256))
        # trailing bytes past TotalLength (Data.CapLength) on some packets
        if rng.random() < 0.1:
            p += bytes(rng.integers(0, 256, int(rng.integers(1, 30)), dtype=np.uint8))
        pkts.append(PacketBuffer(Data=_views_bufconfig(bytes(p), int(rng.choice([0, 14])))))
    return pkts


def _oracle_rx(pk):
    import packets as P

    views = [bytes(v) for v in pk.Data.Views()]
    return P.verify(bytes(pk.Header.View()), views, pk.Data.Size())


@pytest.mark.parametrize("seed", range(4))
def test_verify_packet_buffers_recvmmsg_batches(engine, seed):
    from netstack_amd.packet import verify_packet_buffers

    rng = np.random.default_rng(3100 + seed)
    pkts = _rx_batch(rng, 400 if seed < 3 else 8)  # recvmmsg delivers <= 8 (packet_dispatchers.go:187)
    verdict, sums = verify_packet_buffers(pkts, engine)
    kinds = {0: 0, 1: 0, 2: 0, 3: 0}
    for i, pk in enumerate(pkts):
        want = _oracle_rx(pk)
        got = (int(verdict[i]), int(sums[2 * i]), int(sums[2 * i + 1]))
        assert got == want, (i, got, want)
        kinds[want[0]] += 1
    if seed < 3:
        assert all(kinds[k] > 0 for k in kinds), kinds  # every verdict occurs


@pytest.mark.parametrize("link_hdr", [0, 14])
def test_verify_minimum_sizes(engine, link_hdr):
    """The minimum-size rows (tests/pktgen.py MIN_SIZE; ICMPv6 8 B,
    network/ipv6/icmp.go:68) as the link hands them up in BufConfig views,
    plus longer messages whose transport first view is cut at every length
    up to the minimum + 2 (the gate is on Data.First(), not the message)."""
    from netstack_amd.buffer import NewVectorisedView, View
    from netstack_amd.packet import PacketBuffer, verify_packet_buffers
    from pktgen import MIN_SIZE, min_size_frames, min_size_verdict, short_message

    rng = np.random.default_rng(3200 + link_hdr)
    frames, want = min_size_frames(rng, 0)
    pkts = [PacketBuffer(Data=_views_bufconfig(f, link_hdr)) for f in frames]
    for kind, v6 in (("tcp", False), ("tcp", True), ("udp", True), ("icmp4", False), ("icmp6", True)):
        ipl = 40 if v6 else 20
        for cut in range(1, MIN_SIZE[kind] + 3):
            p = bytes(short_message(rng, kind, MIN_SIZE[kind] + 40, v6))
            pkts.append(PacketBuffer(Data=NewVectorisedView(len(p), [View(bytearray(p[:ipl + cut])),
                                                                     View(bytearray(p[ipl + cut:]))])))
            want.append(min_size_verdict(kind, cut) if cut < MIN_SIZE[kind] or kind != "icmp6" or cut % 2 == 0
                        else None)
    verdict, sums = verify_packet_buffers(pkts, engine)
    for i, pk in enumerate(pkts):
        w = _oracle_rx(pk)
        assert (int(verdict[i]), int(sums[2 * i]), int(sums[2 * i + 1])) == w, i
        if want[i] is not None:
            assert w[0] == want[i], i


def test_verify_single_corrupted_byte_fails(engine):
    """TestReceivedIncorrectChecksumIncrement (tcp_test.go:3246-3254): one
    flipped payload byte fails the segment, anywhere in any view."""
    from netstack_amd.packet import INVALID, VALID, PacketBuffer, verify_packet_buffers

    rng = np.random.default_rng(77)
    base = bytes(_valid_packet(rng, "tcp4", 3000))
    pkts = [PacketBuffer(Data=_views_bufconfig(base, 14))]
    for k in range(20, len(base), 97):
        p = bytearray(base)
        p[k] ^= 0x01
        pkts.append(PacketBuffer(Data=_views_bufconfig(bytes(p), 14)))
    verdict, _ = verify_packet_buffers(pkts, engine)
    assert verdict[0] == VALID and (verdict[1:] == INVALID).all()


def test_ipv4_header_past_the_first_view(engine):
    """tests/golden/rx_choices.json: an IPv4 header longer than
    Data.First() is MALFORMED with no sums taken (the reference reslices past
    the view or panics, network/ipv4/ipv4.go:348); a header within its view
    verifies.  The fixture, the oracle and the engine agree."""
    import json
    import os

    import packets as P

    from netstack_amd.buffer import NewVectorisedView, View
    from netstack_amd.packet import PacketBuffer, verify_packet_buffers

    with open(os.path.join(os.path.dirname(__file__), "golden", "rx_choices.json")) as f:
        cases = json.load(f)["ipv4_header_past_first_view"]
    pkts = [PacketBuffer(Data=NewVectorisedView(c["size"], [View(bytearray.fromhex(v)) for v in c["views"]]))
            for c in cases]
    verdict, sums = verify_packet_buffers(pkts, engine)
    for i, c in enumerate(cases):
        want = (c["verdict"], c["ipv4_sum"], c["transport_sum"])
        assert (int(verdict[i]), int(sums[2 * i]), int(sums[2 * i + 1])) == want, c["name"]
        assert _oracle_rx(pkts[i]) == want, c["name"]
    assert [int(v) for v in verdict] == [P.MALFORMED, P.MALFORMED, P.VALID, P.VALID]


def _tx_batch(rng, n):
    """Outbound PacketBuffers: Header = a Prependable into which the
    transport header and then the IP header were prepended (checksum fields
    zero, as Encode leaves them); Data = payload views of random shapes."""
    from netstack_amd.buffer import NewPrependable, NewVectorisedView, View
    from netstack_amd.packet import PacketBuffer
    from netstack_amd.proto import encode_udp

    pkts = []
    for i in range(n):
        kind = ["tcp4", "tcp6", "udp4", "udp6", "icmp4", "icmp6"][i % 6]
        plen = int(rng.choice([0, 1, 3, int(rng.integers(0, 1460)), int(rng.integers(0, 65000))]))
        payload = bytes(rng.integers(0, 256, plen, dtype=np.uint8))
        cuts = sorted(int(x) for x in rng.integers(0, plen + 1, int(rng.integers(0, 5))))
        views = [View(bytearray(payload[a:b])) for a, b in zip([0] + cuts, cuts + [plen])]
        v6 = kind.endswith("6")
        src = bytes(rng.integers(0, 256, 16 if v6 else 4, dtype=np.uint8))
        dst = bytes(rng.integers(0, 256, 16 if v6 else 4, dtype=np.uint8))
        if kind.startswith("tcp"):
            t, proto = _tcp(rng, int(rng.integers(0, 11))), 6
        elif kind.startswith("udp"):
            t, proto = encode_udp(int(rng.integers(1, 65536)), int(rng.integers(1, 65536)), 8 + plen), 17
        elif kind == "icmp4":
            t, proto = bytearray(8), 1
            struct.pack_into(">HH", t, 4, int(rng.integers(0, 65536)), int(rng.integers(0, 65536)))
        else:
            t, proto = bytearray(24), 58
            t[0] = 136  # a neighbour advertisement-sized message
            t[4:24] = bytes(rng.integers(0, 256, 20, dtype=np.uint8))
        hdr = NewPrependable(int(rng.integers(0, 40)) + 40 + len(t))
        hdr.Prepend(len(t))[:] = t
        ip = _ip6(proto, src, dst, len(t) + plen) if v6 else _ip4(proto, src, dst, len(t) + plen,
                                                                   int(rng.integers(0, 65536)))
        hdr.Prepend(len(ip))[:] = ip
        pkts.append(PacketBuffer(Data=NewVectorisedView(plen, views), Header=hdr))
    return pkts


@pytest.mark.parametrize("seed", range(3))
def test_fill_packet_buffers_matches_reference_writes(engine, seed):
    import packets as P

    from netstack_amd.packet import VALID, PacketBuffer, fill_packet_buffers, verify_packet_buffers
    from netstack_amd.buffer import NewVectorisedView, View

    rng = np.random.default_rng(4200 + seed)
    pkts = _tx_batch(rng, 300)
    want = [P.fill(bytes(pk.Header.View()), [bytes(v) for v in pk.Data.Views()], pk.Data.Size()) for pk in pkts]
    sums = fill_packet_buffers(pkts, engine)
    for i, pk in enumerate(pkts):
        assert bytes(pk.Header.View()) == want[i][0], i
        assert (int(sums[2 * i]), int(sums[2 * i + 1])) == want[i][1:], i
    # what was sent verifies on receive (TCP: VALID; the rest per the reference)
    rx = []
    for pk in pkts:
        wire = bytes(pk.Header.View()) + b"".join(bytes(v) for v in pk.Data.Views())
        rx.append(PacketBuffer(Data=NewVectorisedView(len(wire), [View(bytearray(wire))])))
    verdict, _ = verify_packet_buffers(rx, engine)
    for i, pk in enumerate(pkts):
        w = _oracle_rx(rx[i])
        assert int(verdict[i]) == w[0]
        if i % 6 in (0, 1):  # TCP v4/v6 (ICMPv6's per-view restart makes odd payload cuts differ, as in Go)
            assert verdict[i] == VALID, i


def test_fill_rejects_a_field_outside_header(engine):
    """A transport checksum field that does not lie in Header cannot be
    written: NS_EINVAL (a ValueError here), and nothing is written."""
    from netstack_amd.buffer import NewPrependableFromView, NewVectorisedView, View
    from netstack_amd.packet import PacketBuffer, fill_packet_buffers

    rng = np.random.default_rng(5)
    ip = _ip4(6, b"\x0a\0\0\1", b"\x0a\0\0\2", 20 + 10)
    tcp = _tcp(rng)
    pk = PacketBuffer(Data=NewVectorisedView(30, [View(bytearray(bytes(tcp) + bytes(10)))]),
                      Header=NewPrependableFromView(View(bytearray(ip))))
    before = bytes(pk.Header.View())
    with pytest.raises(ValueError):
        fill_packet_buffers([pk], engine)
    assert bytes(pk.Header.View()) == before
    # the IPv4 header itself (its checksum field) reaching into Data: Header
    # holds only its first 10 bytes, or nothing at all
    for cut in (10, 0):
        wire = bytes(ip) + bytes(tcp) + bytes(10)
        data = bytearray(wire[cut:])
        pk = PacketBuffer(Data=NewVectorisedView(len(data), [View(data)]),
                          Header=NewPrependableFromView(View(bytearray(wire[:cut]))))
        with pytest.raises(ValueError):
            fill_packet_buffers([pk], engine)
        assert bytes(data) == wire[cut:]


@pytest.mark.parametrize("big", [False, True])
def test_acquired_stage_is_read_in_place(engine, big):
    """Pointers into an ns_csum_stage_acquire buffer are read in place (the
    Go shim's path): chains and a VV batch whose bytes all lie in one stage,
    small (zero-copy pass) and above 1 MiB (DMA pipeline), against the
    oracle; the stage returns to the pool and is reused."""
    import ctypes

    import oracle as O

    from netstack_amd import _lib

    rng = np.random.default_rng(11 + big)
    nbytes = (6 << 20) if big else 200_000
    st = engine.stage_acquire(nbytes)
    try:
        st[:] = rng.integers(0, 256, nbytes, dtype=np.uint8)
        base = st.ctypes.data
        nch = 300
        pieces, want = [], []
        for c in range(nch):
            k = int(rng.integers(1, 6))
            init = int(rng.integers(0, 65536))
            x = init
            odd = False
            for j in range(k):
                L = int(rng.integers(0, 3000))
                o = int(rng.integers(0, nbytes - L))
                restart = j == 0 or bool(rng.random() < 0.5)
                fl = (_lib.NS_PIECE_RESTART if restart else 0) | (_lib.NS_PIECE_END if j == k - 1 else 0)
                pieces.append(_lib.NsPiece(base + o, L, init if j == 0 else 0, fl, 0))
                b = bytes(st[o:o + L])
                if restart:
                    odd = False
                if L:
                    x, odd = O.py_calculate_checksum(b, odd, x) if L < 64 else \
                        O.c_calculate_checksum(b, odd, x)
            want.append(x)
        out = np.zeros(nch, dtype=np.uint16)
        arr = (_lib.NsPiece * len(pieces))(*pieces)
        _lib.check(_lib.lib().ns_csum_chains(engine._h, arr, len(pieces),
                                             out.ctypes.data_as(ctypes.POINTER(ctypes.c_uint16)), nch),
                   "ns_csum_chains")
        assert out.tolist() == want
        # a VectorisedView batch over views inside the stage
        views = [st[a:a + 1500] for a in range(0, min(nbytes, 1 << 20) - 1500, 1501)][:200]
        segs = [(int(o), int(s), int(i)) for o, s, i in zip(rng.integers(0, 100_000, 50),
                                                            rng.integers(0, 60_000, 50),
                                                            rng.integers(0, 65536, 50))]
        got = engine.vv_batch(views, segs)
        vb = [bytes(v) for v in views]
        assert got.tolist() == [O.c_checksum_vv_with_offset(vb, i, o, s) for o, s, i in segs]
    finally:
        engine.stage_release(st)
    st2 = engine.stage_acquire(nbytes)
    engine.stage_release(st2)


def test_fill_reproduces_the_reference_tests_checksums(engine):
    """ns_csum_packet_buffers (NS_PKB_FILL) writes into each fixture packet of
    tests/rxcases.py fill_rows, its checksum field zeroed, the checksum the
    reference's own test computed (ICMPv6Checksum over NDP messages and
    ICMPv6 errors, UDP's ^CalculateChecksum over an 8-B datagram)."""
    import rxcases

    from netstack_amd.buffer import NewPrependableFromView, NewVectorisedView, View
    from netstack_amd.packet import PacketBuffer, fill_packet_buffers

    rows = rxcases.fill_rows(rxcases.fixtures())
    pkts = [PacketBuffer(Data=NewVectorisedView(0, []), Header=NewPrependableFromView(View(bytearray(z))))
            for _, z, _ in rows]
    fill_packet_buffers(pkts, engine)
    for (name, _, want), pk in zip(rows, pkts):
        assert bytes(pk.Header.View()) == want, name

