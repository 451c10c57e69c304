"""GPU: a receive ring verified on the device (ns_csum_rx_ring, the receive
mirror of ns_csum_tcp_tx).  Every slot's verdict and sums
against oracle/packets.py verify_frame — recvMMsgDispatcher.dispatch
(link/fdbased/packet_dispatchers.go:258-317), IPv4/IPv6 HandlePacket and
IsValid (network/ipv4/ipv4.go:341-394, header/ipv4.go:280-296, network/ipv6/
ipv6.go:168-188), segment.parse (transport/tcp/segment.go:145-181) and
handleICMP restated on the CPU — and against ns_csum_packet_buffers
(NS_PKB_VERIFY) over the same packets as the link delivers them in BufConfig
views.  Slot bytes past each frame are random, so nothing outside a packet
may leak into its sums.
"""
import struct

import numpy as np
import pytest

from pktgen import ethernet, random_packet, valid_packet, views_bufconfig

pytestmark = pytest.mark.gpu


def _ring(frames, stride, frame_at=0, ring_off=0, seed=0, lens=None):
    """The arena: ring_off random bytes, then one slot of `stride` random
    bytes per frame with the frame written at frame_at.  lens[k] = bytes
    recvmmsg wrote into slot k (frame_at + the frame) unless given."""
    rng = np.random.default_rng(seed)
    n = len(frames)
    arena = rng.integers(0, 256, ring_off + n * stride + 64, dtype=np.uint8)
    out_lens = np.zeros(max(n, 1), dtype=np.uint32)
    for k, f in enumerate(frames):
        at = ring_off + k * stride + frame_at
        f = bytes(f)[:max(stride - frame_at, 0)]
        arena[at:at + len(f)] = np.frombuffer(f, dtype=np.uint8)
        out_lens[k] = frame_at + len(f)
    if lens is not None:
        out_lens[:n] = np.asarray(lens, dtype=np.uint32)
    return arena, out_lens


def _run(engine, arena, lens, ring, stream=None):
    import torch

    dev = torch.device("cuda", 0)
    a = torch.from_numpy(arena).to(dev)
    ln = torch.from_numpy(lens.view(np.int32)).to(dev)
    verdict, sums = engine.rx_ring(a, ring, ln, stream=stream)
    torch.cuda.synchronize()
    n = ring["n"]
    return verdict[:n].cpu().numpy(), sums[:2 * n].cpu().numpy().view(np.uint16)


def _oracle(arena, lens, ring):
    import packets as P

    out = []
    off, stride = ring.get("ring_off", 0), ring["stride"]
    for k in range(ring["n"]):
        slot = bytes(arena[off + k * stride: off + (k + 1) * stride])
        out.append(P.verify_frame(slot, int(lens[k]), ring.get("frame_at", 0), ring.get("link_hdr", 0),
                                  ring.get("first_view", 0)))
    return out


def _check(engine, frames, stride, frame_at=0, link_hdr=0, first_view=0, ring_off=0, lens=None, seed=0):
    arena, ln = _ring(frames, stride, frame_at, ring_off, seed, lens)
    ring = dict(ring_off=ring_off, stride=stride, n=len(frames), frame_at=frame_at, link_hdr=link_hdr,
                first_view=first_view)
    verdict, sums = _run(engine, arena, ln, ring)
    want = _oracle(arena, ln, ring)
    for k, w in enumerate(want):
        got = (int(verdict[k]), int(sums[2 * k]), int(sums[2 * k + 1]))
        assert got == w, (k, got, w, bytes(frames[k][:48]).hex())
    return [w[0] for w in want]


def _frames(rng, n, link_hdr, max_payload=9000):
    pk = [random_packet(rng, max_payload) for _ in range(n)]
    return pk, ([ethernet(p) for p in pk] if link_hdr else [bytes(p) for p in pk])


@pytest.mark.parametrize("link_hdr,first_view,frame_at", [(0, 0, 0), (0, 128, 0), (14, 128, 0), (14, 128, 10),
                                                           (14, 0, 0), (0, 200, 4)])
@pytest.mark.parametrize("seed", range(2))
def test_ring_matches_oracle(engine, link_hdr, first_view, frame_at, seed):
    rng = np.random.default_rng(5100 + seed)
    _, frames = _frames(rng, 300, link_hdr)
    stride = (max(len(f) for f in frames) + frame_at + 15) // 16 * 16
    got = _check(engine, frames, stride, frame_at, link_hdr, first_view, seed=seed)
    assert {0, 1, 2, 3} <= set(got)  # every verdict occurs


@pytest.mark.parametrize("link_hdr", [0, 14])
def test_ring_matches_packet_buffers(engine, link_hdr):
    """The same packets through ns_csum_packet_buffers (NS_PKB_VERIFY) as the
    link hands them up (BufConfig views, link header trimmed): identical
    verdicts and sums."""
    from netstack_amd.packet import PacketBuffer, verify_packet_buffers

    rng = np.random.default_rng(5200 + link_hdr)
    pk, frames = _frames(rng, 400, link_hdr)
    stride = (max(len(f) for f in frames) + 15) // 16 * 16
    arena, ln = _ring(frames, stride)
    ring = dict(stride=stride, n=len(frames), link_hdr=link_hdr, first_view=128)
    verdict, sums = _run(engine, arena, ln, ring)
    # ns_csum_packet_buffers has no EtherType: give it only IP-typed frames
    pkts = [PacketBuffer(Data=views_bufconfig(bytes(p), link_hdr)) for p in pk]
    v2, s2 = verify_packet_buffers(pkts, engine)
    assert (verdict == np.asarray(v2)).all()
    assert (sums == np.asarray(s2, dtype=np.uint16)).all()


def test_reference_packet_fixtures(engine):
    """tests/golden/rx_fixtures.json (the reference's own packets:
    TestInvalidFragments, TestUpdateHoles, TestFragmentationProcess, ...) in
    TUN and Ethernet rings."""
    import rxcases

    import packets as P

    fx = rxcases.fixtures()
    pk = [bytes.fromhex(h) for case in fx["invalid_fragments"] for h in case["packets"]]
    # TestReceivedIncorrectChecksumIncrement's segment (tcp_test.go:3232-3259),
    # intact and with its payload byte corrupted
    c = fx["incorrect_checksum"]
    seg = rxcases.build_segment(bytes.fromhex(c["src"]), bytes.fromhex(c["dst"]), c["src_port"], c["dst_port"],
                                c["seq"], c["ack"], c["flags"], c["window"], bytes.fromhex(c["payload"]),
                                ttl=c["ttl"])
    bad = bytearray(seg)
    bad[40 + c["corrupt_payload_byte"]] = c["corrupt_value"]
    pk += [bytes(seg), bytes(bad)]
    # testBrokenUpWrite's data (tcp_test.go:2214-2216) in one segment and as
    # writePacketFragments' fragments (ipv4.go:119-212)
    big = rxcases.build_segment(bytes.fromhex(c["src"]), bytes.fromhex(c["dst"]), 1, 2, 3, 4, 0x18, 5,
                                bytes(i & 0xFF for i in range(4000)))
    pk.append(bytes(big))
    pk += [h + b"".join(d) for h, d in rxcases.write_packet_fragments(bytes(big[:20]), [bytes(big[20:])], 1500)]
    assert len(pk) >= 20
    stride = (max(len(p) for p in pk) + 14 + 15) // 16 * 16
    got = _check(engine, pk, stride)
    assert got[-6:-4] == [P.VALID, P.INVALID] and got[-4] == P.VALID and set(got[-3:]) == {P.UNCHECKED}
    _check(engine, [ethernet(p, 0x0800) for p in pk], stride, link_hdr=14, first_view=128)


@pytest.mark.parametrize("link_hdr,first_view", [(0, 0), (0, 128), (14, 128), (14, 0)])
def test_ipv6_and_control_fixtures(engine, link_hdr, first_view):
    """tests/golden/rx_fixtures.json ipv6_receive — the IPv6 packets
    network/ipv6's tests inject (ipv6_test.go testReceiveICMP/testReceiveUDP,
    ndp_test.go's NDP hop-limit and RA validation: 8-B, 15-B and 64-B ICMPv6
    messages, an 8-B UDP), intact and with a flipped checksum bit — and
    receive_control — network/ip_test.go's IPv4/IPv6 ReceiveControl ICMP
    errors at every cut, down to empty packets — in a ring and through
    ns_csum_packet_buffers: the fixture's verdicts, the oracle's sums."""
    import rxcases

    from netstack_amd.packet import PacketBuffer, verify_packet_buffers

    fx = rxcases.fixtures()
    rows = rxcases.ipv6_rows(fx) + rxcases.control_rows(fx)
    frames = [ethernet(b) if link_hdr else b for _, b, _ in rows]
    got = _check(engine, frames, 128, link_hdr=link_hdr, first_view=first_view, seed=4)
    assert got == [w for _, _, w in rows]
    pkts = [PacketBuffer(Data=views_bufconfig(b, link_hdr)) for _, b, _ in rows]
    v2, _ = verify_packet_buffers(pkts, engine)
    assert list(v2) == got


@pytest.mark.parametrize("link_hdr,first_view", [(0, 0), (0, 128), (14, 128), (0, 64), (14, 78)])
def test_fuzzed_header_fields(engine, link_hdr, first_view):
    """Every header field the receive rules read set to its boundaries or a
    random value (pktgen.fuzz_fields: version/IHL, TotalLength, fragment
    field, protocol, IPv6 PayloadLength and NextHeader, TCP data offset, ICMP
    type, the checksum field): the ring's verdicts and sums equal the
    oracle's, and ns_csum_packet_buffers gives the same over the link's
    views."""
    from pktgen import fuzzed_packets

    from netstack_amd.packet import PacketBuffer, verify_packet_buffers

    rng = np.random.default_rng(6100 + link_hdr + first_view)
    pk = fuzzed_packets(rng, 3000)
    frames = [ethernet(p) if link_hdr else p for p in pk]
    stride = (max(len(f) for f in frames) + 15) // 16 * 16
    got = _check(engine, frames, stride, link_hdr=link_hdr, first_view=first_view, seed=6)
    assert {0, 1, 2, 3} <= set(got)
    if first_view in (0, 128):  # the views ns_csum_packet_buffers is given are BufConfig's (or one)
        ip = [k for k, p in enumerate(pk) if p and (p[0] >> 4) in (4, 6)]
        pkts = [PacketBuffer(Data=views_bufconfig(pk[k], link_hdr)) if first_view else
                PacketBuffer(Data=_one_view(pk[k])) for k in ip]
        v2, _ = verify_packet_buffers(pkts, engine)
        assert list(v2) == [got[k] for k in ip]


def _one_view(b: bytes):
    from netstack_amd.buffer import NewVectorisedView, View

    return NewVectorisedView(len(b), [View(bytearray(b))])


@pytest.mark.parametrize("link_hdr,first_view,frame_at", [(0, 0, 0), (0, 128, 0), (14, 128, 0), (14, 128, 10),
                                                           (14, 0, 4), (0, 64, 2)])
@pytest.mark.parametrize("cap", [80, 128, 192, 256])
def test_short_frame_rings(engine, link_hdr, first_view, frame_at, cap):
    """Rings of short slots (80-256 B, the strides the 4-lane group shape
    takes, rx_ring.hip rx_batch_units4): random packets and fuzzed headers
    cut to the slot, every verdict and sum equal to the oracle's."""
    from pktgen import fuzzed_packets

    rng = np.random.default_rng(6300 + cap + link_hdr + frame_at)
    pk = [random_packet(rng, cap) for _ in range(500)] + fuzzed_packets(rng, 500, max_payload=cap)
    frames = [ethernet(p) if link_hdr else bytes(p) for p in pk]
    stride = cap
    lens = [min(len(f) + frame_at, stride) for f in frames]
    got = _check(engine, frames, stride, frame_at, link_hdr, first_view, lens=lens, seed=cap)
    assert {1, 3} <= set(got)


@pytest.mark.parametrize("link_hdr,first_view", [(0, 0), (0, 128), (0, 64), (14, 128), (14, 0), (14, 78)])
def test_minimum_sizes(engine, link_hdr, first_view):
    """Every transport message from 0 to its minimum + 2 bytes (TCP 20, UDP 8,
    ICMPv4 8, ICMPv6 8 — ICMPv6MinimumSize, network/ipv6/icmp.go:68; the
    table and its reference lines in tests/pktgen.py MIN_SIZE), intact and
    with a changed byte: MALFORMED under the minimum, the checksum's verdict
    from it, as the oracle and the reference give them."""
    from pktgen import min_size_frames

    rng = np.random.default_rng(5900 + link_hdr + first_view)
    frames, want = min_size_frames(rng, link_hdr)
    got = _check(engine, frames, 128, link_hdr=link_hdr, first_view=first_view, seed=3)
    assert got == want


def test_first_view_decides_the_tcp_header_check(engine):
    """segment.parse checks DataOffset against the FIRST view (segment.go:160):
    a 60-B IPv4 header and a 60-B TCP header fit BufConfig's 128-B first view
    on a TUN link but not on Ethernet (128 - 14 = 114 B), where the packet is
    malformed; as one view it verifies."""
    import packets as P

    rng = np.random.default_rng(7)
    p = bytearray(valid_packet(rng, "tcp4", 600))
    # rebuild with IHL 15 and a 60-B TCP header, checksums refilled by the oracle
    from pktgen import ip4
    from netstack_amd.tcp import TCPFields, encode_tcp

    t = encode_tcp(TCPFields(1, 2, 3, 4, 60, 0x18, 100), bytes(40))
    payload = bytes(rng.integers(0, 256, 600, dtype=np.uint8))
    ip = ip4(6, b"\x0a\0\0\1", b"\x0a\0\0\2", 60 + 600, ihl=60)
    hdr, _, _ = P.fill(bytes(ip + t), [payload], 600)
    p = hdr + payload
    assert _check(engine, [p], 1024, link_hdr=0, first_view=128) == [P.VALID]
    assert _check(engine, [ethernet(p)], 1024, link_hdr=14, first_view=128) == [P.MALFORMED]
    assert _check(engine, [ethernet(p)], 1024, link_hdr=14, first_view=0) == [P.VALID]


def test_lengths_and_link_edges(engine):
    """Slot lengths at every edge: 0, the link header alone (dropped), one
    byte past it, exactly the stride, longer than the stride (MALFORMED and
    counted by ns_csum_sync), odd lengths; non-IP EtherTypes (UNCHECKED) and
    an EtherType that disagrees with the version nibble (IsValid: MALFORMED)."""
    import packets as P
    import torch

    rng = np.random.default_rng(11)
    good = bytes(valid_packet(rng, "tcp4", 101))  # odd length
    g6 = bytes(valid_packet(rng, "tcp6", 57))
    stride = 256
    frames = [ethernet(good), ethernet(good), ethernet(good), ethernet(good), ethernet(good),
              ethernet(good, 0x0806), ethernet(g6, 0x0800), ethernet(good, 0x86DD), ethernet(g6),
              ethernet(good)[:15], ethernet(g6) + bytes(stride)]
    lens = [len(frames[0]), 0, 14, 15, stride + 1, len(frames[5]), len(frames[6]), len(frames[7]), len(frames[8]),
            15, stride]
    arena, ln = _ring(frames, stride, lens=lens)
    ring = dict(stride=stride, n=len(frames), link_hdr=14, first_view=128)
    eng = engine
    eng.sync()
    verdict, sums = _run(eng, arena, ln, ring)
    want = _oracle(arena, ln, ring)
    assert [int(v) for v in verdict] == [w[0] for w in want]
    assert [(int(sums[2 * k]), int(sums[2 * k + 1])) for k in range(len(frames))] == [w[1:] for w in want]
    assert [w[0] for w in want] == [P.VALID, P.MALFORMED, P.MALFORMED, P.MALFORMED, P.MALFORMED,
                                   P.UNCHECKED, P.MALFORMED, P.MALFORMED, P.VALID, P.MALFORMED, P.VALID]
    assert eng.sync() == 1  # the slot longer than its stride
    torch.cuda.synchronize()


@pytest.mark.parametrize("kind", ["tcp4", "tcp6", "icmp6"])
def test_largest_packets(engine, kind):
    """IP packets at their header-given maximum (IPv4 TotalLength 65,535;
    IPv6 40 + PayloadLength 65,535) in 64-KiB+ slots: more lines than one load
    batch, every byte summed once."""
    import packets as P

    from pktgen import ip4, ip6, tcp_header

    rng = np.random.default_rng(13)
    v6 = kind.endswith("6")
    t = tcp_header(rng) if kind.startswith("tcp") else bytearray([128, 0, 0, 0, 0, 0, 0, 0])
    proto = 6 if kind.startswith("tcp") else 58
    plen = 65535 - len(t) - (0 if v6 else 20)
    src, dst = bytes(range(16 if v6 else 4)), bytes(range(1, 17 if v6 else 5))
    ip = ip6(proto, src, dst, len(t) + plen) if v6 else ip4(proto, src, dst, len(t) + plen)
    payload = bytes(rng.integers(0, 256, plen, dtype=np.uint8))
    hdr, _, _ = P.fill(bytes(ip + t), [payload], plen)
    p = hdr + payload
    bad = bytearray(p)
    bad[len(bad) // 2] ^= 0x40
    stride = (len(p) + 15) // 16 * 16 + 32
    assert _check(engine, [p, bytes(bad), p], stride) == [P.VALID, P.INVALID, P.VALID]


@pytest.mark.parametrize("stride", [64, 80, 1504, 2048])
def test_small_and_common_strides(engine, stride):
    rng = np.random.default_rng(17 + stride)
    frames = []
    for _ in range(200):
        p = random_packet(rng, max_payload=stride)
        frames.append(bytes(p)[:stride])
    got = _check(engine, frames, stride, ring_off=stride * 3)
    assert len(got) == 200


@pytest.mark.parametrize("stride,link_hdr,frame_at", [(1536, 0, 0), (2048, 14, 10), (1536, 14, 120), (1664, 14, 2)])
def test_line_aligned_slots(engine, stride, link_hdr, frame_at):
    """Rings of 128-B-aligned slots whose packets start in the slot's first
    line load line 0 nontemporal too (no line is shared between slots); a
    frame starting past the first line (frame_at + link >= 128) keeps the
    default shape.  The same verdicts and sums as the oracle either way."""
    rng = np.random.default_rng(19 + stride + frame_at)
    _, frames = _frames(rng, 300, link_hdr, max_payload=stride - frame_at - 80)
    got = _check(engine, frames, stride, frame_at, link_hdr, 128 if link_hdr else 0, ring_off=stride * 2)
    assert {0, 1} <= set(got)


def test_header_fuzz(engine):
    """Random byte flips in the first 80 bytes of valid packets (every
    header field the receive path reads), as TUN and Ethernet frames."""
    rng = np.random.default_rng(19)
    frames = []
    for i in range(600):
        p = random_packet(rng, max_payload=1500)
        for _ in range(int(rng.integers(1, 4))):
            k = int(rng.integers(0, min(80, len(p)))) if len(p) else 0
            if len(p):
                p[k] = int(rng.integers(0, 256))
        frames.append(bytes(p))
    stride = (max(len(f) for f in frames) + 14 + 15) // 16 * 16
    _check(engine, frames, stride, first_view=128)
    _check(engine, [ethernet(f) for f in frames], stride, link_hdr=14, first_view=128, frame_at=0)


def test_two_streams_and_no_outputs_but_verdict(engine):
    """Two rings on two streams at once, one with verdicts only."""
    import torch

    rng = np.random.default_rng(23)
    _, f1 = _frames(rng, 200, 0, 3000)
    _, f2 = _frames(rng, 200, 14, 3000)
    s1 = (max(len(f) for f in f1) + 15) // 16 * 16
    s2 = (max(len(f) for f in f2) + 15) // 16 * 16
    a1, l1 = _ring(f1, s1, seed=1)
    a2, l2 = _ring(f2, s2, seed=2)
    dev = torch.device("cuda", 0)
    st = [torch.cuda.Stream(dev), torch.cuda.Stream(dev)]
    t1, t2 = torch.from_numpy(a1).to(dev), torch.from_numpy(a2).to(dev)
    n1, n2 = torch.from_numpy(l1.view(np.int32)).to(dev), torch.from_numpy(l2.view(np.int32)).to(dev)
    torch.cuda.synchronize()
    r1 = dict(stride=s1, n=200, first_view=128)
    r2 = dict(stride=s2, n=200, link_hdr=14, first_view=128)
    v1, sm1 = engine.rx_ring(t1, r1, n1, stream=st[0])
    v2 = torch.empty(200, dtype=torch.uint8, device=dev)
    import ctypes

    from netstack_amd import _lib

    r = _lib.NsRxRing(0, s2, 200, 0, 14, 128, 0)
    _lib.check(_lib.lib().ns_csum_rx_ring(engine._h, t2.data_ptr(), t2.numel(), ctypes.byref(r), n2.data_ptr(),
                                          None, v2.data_ptr(), st[1].cuda_stream), "ns_csum_rx_ring")
    torch.cuda.synchronize()
    w1, w2 = _oracle(a1, l1, r1), _oracle(a2, l2, r2)
    assert [int(x) for x in v1.cpu()] == [w[0] for w in w1]
    assert [int(x) for x in v2.cpu()] == [w[0] for w in w2]
    s = sm1.cpu().numpy().view(np.uint16)
    assert [(int(s[2 * k]), int(s[2 * k + 1])) for k in range(200)] == [w[1:] for w in w1]


def test_invalid_geometry(engine):
    import torch

    dev = torch.device("cuda", 0)
    a = torch.zeros(1 << 16, dtype=torch.uint8, device=dev)
    ln = torch.zeros(16, dtype=torch.int32, device=dev)
    bad = [dict(stride=1500, n=16), dict(stride=0, n=16), dict(stride=1 << 24, n=1), dict(stride=1504, n=16, ring_off=8),
           dict(stride=1504, n=16, link_hdr=6), dict(stride=1504, n=16, frame_at=3),
           dict(stride=1504, n=16, first_view=127), dict(stride=1504, n=16, link_hdr=14, first_view=64),
           dict(stride=1504, n=16, flags=1), dict(stride=1504, n=16, frame_at=1504)]
    for r in bad:
        with pytest.raises(ValueError):
            engine.rx_ring(a, r, ln)
    from netstack_amd._lib import ChecksumError

    with pytest.raises(ChecksumError):  # NS_ERANGE: the ring past the arena
        engine.rx_ring(a, dict(stride=4096, n=17), torch.zeros(17, dtype=torch.int32, device=dev))
    engine.rx_ring(a, dict(stride=4096, n=16, link_hdr=14, first_view=78), ln)  # 78 - 14 = 64: accepted
    torch.cuda.synchronize()


@pytest.mark.slow
@pytest.mark.parametrize("v6", [False, True])
def test_full_size_ring(engine, v6):
    """BASELINE cfg2's shape as a receive ring (1M x 1500-B IPv4/TCP, or
    IPv6/TCP, packets at stride 1504, every 997th with one corrupted byte):
    exactly those fail; every IPv4 header sums to 0xffff (IPv6: no IP sum,
    0); 256 random slots against the oracle."""
    import torch

    from netstack_amd import workloads as W

    n = 1 << 20
    dev = torch.device("cuda", 0)
    make = W.rx_ring_batch_v6 if v6 else W.rx_ring_batch
    arena, lens, bad = make(n, 9, dev, corrupt_every=997)
    ring = dict(stride=W.RX_STRIDE, n=n)
    verdict, sums = engine.rx_ring(arena, ring, lens)
    torch.cuda.synchronize()
    v = verdict.cpu().numpy()
    want = np.ones(n, dtype=np.uint8)
    want[bad] = 0
    assert (v == want).all()
    s = sums.cpu().numpy().view(np.uint16)
    assert (s[0::2] == (0 if v6 else 0xFFFF)).all()
    rng = np.random.default_rng(29)
    pick = np.sort(rng.choice(n, 256, replace=False))
    a = arena.view(n, W.RX_STRIDE)[torch.from_numpy(pick).to(dev)].cpu().numpy()
    import packets as P

    for i, k in enumerate(pick):
        got = (int(v[k]), int(s[2 * k]), int(s[2 * k + 1]))
        assert got == P.verify_frame(bytes(a[i]), W.RX_PKT), k


@pytest.mark.parametrize("frame_at", [0, 2, 4, 10])
def test_padded_frames_and_chunk_edges(engine, frame_at):
    """Frames carrying bytes past their transport's end (Ethernet padding,
    CapLength) of every size, next to unpadded ones in the same waves, with
    the transport's end at every offset inside its 16-B chunk: the kernel
    sums lines past line 1 whole, corrects the chunk holding the end, and
    re-reads a wave with a padded frame beyond line 1 with the range check
    (rx_ring.hip F = 1).  Every slot against the oracle."""
    rng = np.random.default_rng(41 + frame_at)
    frames = []
    for i in range(400):
        kind = ("tcp4", "tcp6", "icmp4", "icmp6")[i % 4]
        plen = int(rng.integers(100, 2600)) if i % 3 else int(rng.integers(0, 120))
        p = bytearray(valid_packet(rng, kind, plen))
        if rng.random() < 0.15:  # a corrupted byte
            k = int(rng.integers(0, len(p)))
            p[k] ^= 0x21
        pad = int(rng.choice([0, 0, 0, 1, 2, 15, 16, 17, 31, 100, 300, 1000]))
        p += bytes(rng.integers(0, 256, pad, dtype=np.uint8))
        frames.append(bytes(p))
    stride = (max(len(f) for f in frames) + frame_at + 15) // 16 * 16
    got = _check(engine, frames, stride, frame_at=frame_at, first_view=128 if frame_at % 4 == 0 else 0)
    assert {0, 1} <= set(got)
