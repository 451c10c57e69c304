"""Test infrastructure: packet builders shared by the receive-path GPU tests
(tests/test_gpu_packet.py, tests/test_gpu_rx_ring.py).  Checksums of the
packets they build are filled by the oracle's transmit restatement
(oracle/packets.py fill), so a "valid" packet is what a peer running the
reference would send.  Not part of the product."""
import struct

import numpy as np

BUF_CONFIG = [128, 256, 256, 512, 1024, 2048, 4096, 8192, 16384, 32768]  # packet_dispatchers.go:30


def views_bufconfig(pkt: bytes, link_hdr: int):
    """recvMMsgDispatcher: the frame (link header + packet) read into
    BufConfig views, the last used one capped (capViews), then
    Data.TrimFront(hdrSize)."""
    from netstack_amd.buffer import NewVectorisedView, View

    frame = bytes(link_hdr) + pkt
    views, c = [], 0
    for s in BUF_CONFIG:
        views.append(View(bytearray(frame[c:c + s])))
        c += s
        if c >= len(frame):
            break
    vv = NewVectorisedView(len(frame), views)
    vv.TrimFront(link_hdr)
    return vv


def ip4(proto, src, dst, payload_len, ident=0, frag=0, ihl=20, tlen=None):
    from netstack_amd.proto import IPv4Fields, encode_ipv4

    h = encode_ipv4(IPv4Fields(IHL=ihl, TotalLength=tlen if tlen is not None else ihl + payload_len, ID=ident,
                               TTL=64, Protocol=proto, SrcAddr=src, DstAddr=dst))
    if frag:
        struct.pack_into(">H", h, 6, frag)
    return h


def ip6(proto, src, dst, payload_len):
    h = bytearray(40)
    h[0] = 0x60
    struct.pack_into(">HBB", h, 4, payload_len & 0xFFFF, proto, 64)
    h[8:24] = src
    h[24:40] = dst
    return h


def tcp_header(rng, opts_words=0):
    from netstack_amd.tcp import TCPFields, encode_tcp

    off = 20 + 4 * opts_words
    return encode_tcp(TCPFields(int(rng.integers(1, 65536)), int(rng.integers(1, 65536)),
                                int(rng.integers(0, 2**32)), int(rng.integers(0, 2**32)), off, 0x18,
                                int(rng.integers(0, 65536))), bytes(rng.integers(0, 256, 4 * opts_words,
                                                                                 dtype=np.uint8)))


def valid_packet(rng, kind, plen):
    """A well-formed packet of `kind` with correct checksums (filled by the
    oracle's transmit restatement) — the bytes a peer would send."""
    import packets as P

    from netstack_amd.proto import encode_udp

    payload = bytes(rng.integers(0, 256, plen, dtype=np.uint8))
    v6 = kind.endswith("6")
    src, dst = (bytes(rng.integers(0, 256, 16, dtype=np.uint8)), bytes(rng.integers(0, 256, 16, dtype=np.uint8))) \
        if v6 else (bytes(rng.integers(0, 256, 4, dtype=np.uint8)), bytes(rng.integers(0, 256, 4, dtype=np.uint8)))
    if kind.startswith("tcp"):
        t = tcp_header(rng, int(rng.integers(0, 4)))
        proto = 6
    elif kind.startswith("udp"):
        t = encode_udp(int(rng.integers(1, 65536)), int(rng.integers(1, 65536)), 8 + plen)
        proto = 17
    elif kind == "icmp4":
        t = bytearray(8)
        t[0] = 8  # echo request
        struct.pack_into(">HH", t, 4, int(rng.integers(0, 65536)), int(rng.integers(0, 65536)))
        proto = 1
    else:  # icmp6: echo request
        t = bytearray(8)
        t[0] = 128
        proto = 58
    ip = ip6(proto, src, dst, len(t) + plen) if v6 else ip4(proto, src, dst, len(t) + plen,
                                                               int(rng.integers(0, 65536)))
    hdr, _, _ = P.fill(bytes(ip + t), [payload], plen)
    if kind == "icmp4":  # fill() wrote an echo-reply style sum: valid for the request too
        pass
    return bytearray(hdr + payload)


def frag_packet(rng, how, plen):
    """IPv4 fragments of every kind HandlePacket tells apart
    (network/ipv4/ipv4.go:355-385; FragmentOffset() = field << 3 in a uint16):
    0 MF with a TCP header and payload (reassembled: UNCHECKED); 1 the last
    fragment (no MF, an offset; UNCHECKED); 2 MF and no payload (MALFORMED,
    :357-363); 3 an offset with no payload (MALFORMED); 4 the highest offset
    with `last = offset + size - 1` wrapping past 0xffff (MALFORMED,
    :365-373); 5 the same offset with exactly 8 bytes, last = 0xffff (no wrap:
    UNCHECKED)."""
    if how in (0, 1):
        p = valid_packet(rng, "tcp4", plen)
        struct.pack_into(">H", p, 6, 0x2000 if how == 0 else int(rng.integers(1, 0x2000)))
        return p
    src, dst = bytes(rng.integers(0, 256, 4, dtype=np.uint8)), bytes(rng.integers(0, 256, 4, dtype=np.uint8))
    size = 0 if how in (2, 3) else int(rng.integers(9, 3000)) if how == 4 else 8
    frag = {2: 0x2000 | int(rng.integers(0, 0x2000)), 3: int(rng.integers(1, 0x2000)),
            4: 0x1FFF | (0x2000 if rng.random() < 0.5 else 0), 5: 0x1FFF}[how]
    p = ip4(6, src, dst, size, int(rng.integers(0, 65536)), frag=frag)
    p += bytes(rng.integers(0, 256, size, dtype=np.uint8))
    # the IPv4 header checksum as addIPHeader writes it (the reference does not check it on receive)
    import oracle as O

    struct.pack_into(">H", p, 10, 0)
    struct.pack_into(">H", p, 10, (~O.c_checksum(bytes(p[:20]), 0)) & 0xFFFF)
    return p


def random_packet(rng, max_payload: int = 9000) -> bytearray:
    """One received IP packet of a recvmmsg-like mix: mostly TCP (v4/v6),
    plus ICMPv4/v6, UDP, fragments of every kind and malformed packets; ~1/7
    of the valid ones carry one corrupted byte, ~1/10 trailing bytes past
    their TotalLength (Data.CapLength)."""
    r = rng.random()
    kind = "tcp4" if r < 0.45 else "tcp6" if r < 0.65 else "icmp4" if r < 0.72 else \
        "icmp6" if r < 0.79 else "udp4" if r < 0.85 else "frag" if r < 0.88 else "bad" if r < 0.96 else "short"
    plen = int(rng.choice([0, 1, 7, int(rng.integers(0, 1460)), int(rng.integers(0, max_payload))]))
    if kind == "short":  # a message around its protocol's minimum size
        k = ("tcp", "udp", "icmp4", "icmp6")[int(rng.integers(0, 4))]
        p = short_message(rng, k, int(rng.integers(0, MIN_SIZE[k] + 3)),
                          None if k.startswith("icmp") else bool(rng.integers(0, 2)))
    elif kind == "frag":
        p = frag_packet(rng, int(rng.integers(0, 6)), plen)
    elif kind == "bad":
        p = valid_packet(rng, "tcp4", plen)
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
        p = valid_packet(rng, kind, plen)
        if rng.random() < 1 / 7 and len(p) > 0:
            k = int(rng.integers(0, len(p)))
            p[k] ^= int(rng.integers(1, 256))
    if rng.random() < 0.1:
        p += bytes(rng.integers(0, 256, int(rng.integers(1, 30)), dtype=np.uint8))
    return bytearray(p)


def ethernet(pkt: bytes, etype: int | None = None) -> bytes:
    """An Ethernet frame around an IP packet (header.Ethernet: dst, src,
    EtherType); the type follows the version nibble unless given."""
    if etype is None:
        etype = 0x86DD if pkt and (pkt[0] >> 4) == 6 else 0x0800
    return bytes(range(1, 13)) + struct.pack(">H", etype) + bytes(pkt)


# The receive path's minimum sizes, each checked against the transport's FIRST
# VIEW (Data.First() after the IP trim) before any checksum is taken:
#   tcp   TCPMinimumSize 20   stack/nic.go:851 (DeliverTransportPacket),
#                             header/tcp.go:169; segment.go:159 (DataOffset)
#   udp   UDPMinimumSize 8    stack/nic.go:851, header/udp.go:56
#   icmp4 ICMPv4MinimumSize 8 network/ipv4/icmp.go:60, header/icmpv4.go:32
#   icmp6 ICMPv6MinimumSize 8 network/ipv6/icmp.go:68, header/icmpv6.go:35
# and the network headers' against the packet's first view:
#   ip4   IPv4MinimumSize 20  stack/nic.go:774, header/ipv4.go:83, :281
#   ip6   IPv6MinimumSize 40  stack/nic.go:774, header/ipv6.go:68, :208
MIN_SIZE = {"tcp": 20, "udp": 8, "icmp4": 8, "icmp6": 8}
_HDR = {"tcp": 20, "udp": 8, "icmp4": 8, "icmp6": 8}
_PROTO = {"tcp": 6, "udp": 17, "icmp4": 1, "icmp6": 58}


def short_message(rng, kind: str, length: int, v6: bool | None = None) -> bytearray:
    """An IP packet whose transport message is exactly `length` bytes:
    `kind` in tcp/udp/icmp4/icmp6 (IPv4 unless v6 or icmp6).  From the
    protocol's minimum size on it is a well-formed message with correct
    checksums (oracle/packets.py fill, a 20-B TCP header, an ICMP echo
    request); below it, the first `length` bytes of one, with the IP length
    fields saying `length`."""
    import packets as P

    v6 = kind == "icmp6" if v6 is None else v6
    alen = 16 if v6 else 4
    src = bytes(rng.integers(0, 256, alen, dtype=np.uint8))
    dst = bytes(rng.integers(0, 256, alen, dtype=np.uint8))
    proto, hl = _PROTO[kind], _HDR[kind]
    if kind == "tcp":
        t = tcp_header(rng, 0)
    elif kind == "udp":
        from netstack_amd.proto import encode_udp

        t = encode_udp(int(rng.integers(1, 65536)), int(rng.integers(1, 65536)), length)
    else:
        t = bytearray(8)
        t[0] = 128 if kind == "icmp6" else 8  # echo request
        struct.pack_into(">HH", t, 4, int(rng.integers(0, 65536)), int(rng.integers(0, 65536)))
    ip = ip6(proto, src, dst, length) if v6 else ip4(proto, src, dst, length, int(rng.integers(0, 65536)))
    if length < hl:
        return bytearray(ip + t[:length])
    payload = bytes(rng.integers(0, 256, length - hl, dtype=np.uint8))
    hdr, _, _ = P.fill(bytes(ip + t), [payload], length - hl)
    return bytearray(hdr + payload)


def min_size_verdict(kind: str, first_len: int, valid: int = 1) -> int:
    """The reference's verdict for a message of `kind` whose first view holds
    `first_len` transport bytes: MALFORMED (3) under the minimum size; at or
    above it UNCHECKED (2) for UDP (no receive checksum), else `valid` (the
    checksum's outcome, 1 for the well-formed messages above)."""
    if first_len < MIN_SIZE[kind]:
        return 3
    return 2 if kind == "udp" else valid


def short_messages(rng, extra: int = 2):
    """Every (kind, ip version, length) with length 0 .. minimum + extra:
    [(kind, v6, length, packet)] — the rows of the minimum-size table."""
    out = []
    for kind in ("tcp", "udp", "icmp4", "icmp6"):
        for v6 in ((False,) if kind == "icmp4" else (True,) if kind == "icmp6" else (False, True)):
            for length in range(0, MIN_SIZE[kind] + extra + 1):
                out.append((kind, v6, length, short_message(rng, kind, length, v6)))
    return out


def min_size_frames(rng, link_hdr: int):
    """The minimum-size rows as a receive batch: every short_messages row
    (TUN packets, or Ethernet frames when link_hdr) plus, for each row at or
    above its minimum, a copy with its last byte changed (the checksum's
    INVALID side).  Returns (frames, the reference's verdicts)."""
    frames, want = [], []
    for kind, _, length, p in short_messages(rng):
        frames.append(p)
        want.append(min_size_verdict(kind, length))
        if length >= MIN_SIZE[kind]:
            q = bytearray(p)
            q[-1] ^= int(rng.integers(1, 256))
            frames.append(q)
            want.append(min_size_verdict(kind, length, valid=0))
    if link_hdr:
        frames = [ethernet(bytes(f)) for f in frames]
    return [bytes(f) for f in frames], want


def fuzz_fields(rng, p: bytearray) -> bytearray:
    """One header field of a packet set to a boundary or random value: the
    fields the receive rules read (IPv4 version/IHL, TotalLength, flags and
    fragment offset, protocol; IPv6 PayloadLength and NextHeader; the TCP
    data offset, the ICMP type, the transport checksum field).  Checksums are
    left as they were, so most results are INVALID or MALFORMED, and the
    boundaries sit where a rule changes its mind."""
    p = bytearray(p)
    if len(p) < 1:
        return p
    n = len(p)
    v6 = (p[0] >> 4) == 6
    ipl = 40 if v6 else 4 * (p[0] & 15)
    pick = lambda *vals: int(vals[int(rng.integers(0, len(vals)))])  # noqa: E731
    f = int(rng.integers(0, 6))
    if not v6 and f == 0:
        p[0] = pick(0x40, 0x44, 0x45, 0x46, 0x4F, 0x60, 0x00, int(rng.integers(0, 256)))
    elif not v6 and f == 1 and n >= 4:
        struct.pack_into(">H", p, 2, pick(0, 19, 20, ipl, ipl + 7, ipl + 8, ipl + 19, ipl + 20, n - 1, n, n + 1,
                                          0xFFFF, int(rng.integers(0, 65536))) & 0xFFFF)
    elif not v6 and f == 2 and n >= 8:
        struct.pack_into(">H", p, 6, pick(0x2000, 0x1FFF, 0x3FFF, 0x4000, 0x0001, 0x2001, int(rng.integers(0, 65536))))
    elif v6 and f in (0, 1) and n >= 6:
        struct.pack_into(">H", p, 4, pick(0, 7, 8, 19, 20, n - 41, n - 40, n - 39, 0xFFFF,
                                          int(rng.integers(0, 65536))) & 0xFFFF)
    elif f == 3 and n > (6 if v6 else 9):
        p[6 if v6 else 9] = pick(1, 6, 17, 58, 0, 44, int(rng.integers(0, 256)))
    elif f == 4 and n > ipl + 12:
        proto = p[6] if v6 else p[9]
        if proto == 6:
            p[ipl + 12] = pick(0x00, 0x40, 0x50, 0x60, 0xF0, 0x80, int(rng.integers(0, 256)))
        else:
            p[ipl] = pick(0, 3, 8, 128, 129, 133, 136, int(rng.integers(0, 256)))
    elif n > ipl + 18:
        proto = p[6] if v6 else p[9]
        at = ipl + (16 if proto == 6 else 6 if proto == 17 else 2)
        p[at + int(rng.integers(0, 2))] ^= 1 << int(rng.integers(0, 8))
    return p


def fuzzed_packets(rng, count: int, max_payload: int = 3000):
    """valid_packet / random_packet bytes, each with one field fuzzed."""
    out = []
    for _ in range(count):
        if rng.random() < 0.7:
            kind = ("tcp4", "tcp6", "icmp4", "icmp6", "udp4")[int(rng.integers(0, 5))]
            p = valid_packet(rng, kind, int(rng.choice([0, 1, 7, 8, 20, int(rng.integers(0, max_payload))])))
        else:
            p = random_packet(rng, max_payload)
        out.append(bytes(fuzz_fields(rng, p)))
    return out
