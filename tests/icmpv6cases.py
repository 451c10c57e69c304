"""The ICMPv6 checksum validation cases of the reference's own tests, as data:
TestICMPChecksumValidationSimple, ...WithPayload and
...WithPayloadMultipleViews (tcpip/network/ipv6/icmp_test.go:367-899).

Each case builds one ICMPv6 message as the test's handleIPv6Payload does, in
two forms:
- the transmit split, which the test checksums with
  ICMPv6Checksum(pkt, lladdr1, lladdr0, vv) (icmp_test.go:495, 671, 849);
- the receive split, which icmp.go:79-82 checksums: h = the first view after
  the IPv6 header, payload = the remaining views.

The reference asserts two things for every case. The message injected with a
zero checksum field counts as Invalid (icmp_test.go:524-531, 701-708,
879-886). The message with the field set counts as received (:534-541,
711-718, 889-896). Since ICMPv6Checksum zeroes h[2:4] itself
(icmpv6.go:214-219), the receive check `h.Checksum() != want` (icmp.go:82)
passes for the second message exactly when the receive split gives the
transmit split's value, and fails for the first one exactly when that value
is not 0.
"""
from __future__ import annotations

import struct

# icmp_test.go:33-39 and header.LinkLocalAddr (ipv6.go:271-291)
LINK_ADDR0 = bytes([0x02, 0x02, 0x03, 0x04, 0x05, 0x06])
LINK_ADDR1 = bytes([0x0A, 0x0B, 0x0C, 0x0D, 0x0E, 0x0F])


def link_local(mac: bytes) -> bytes:
    a = bytearray(16)
    a[0], a[1] = 0xFE, 0x80
    a[8], a[9], a[10], a[11], a[12] = mac[0] ^ 2, mac[1], mac[2], 0xFF, 0xFE
    a[13], a[14], a[15] = mac[3], mac[4], mac[5]
    return bytes(a)


LLADDR0 = link_local(LINK_ADDR0)
LLADDR1 = link_local(LINK_ADDR1)

# header constants (icmpv6.go:32-110, ndp_*.go, ipv6.go)
IPV6_MIN = 40
ICMPV6_HEADER = 4
ICMPV6_MIN = 8
ICMPV6_PAYLOAD_OFFSET = 8
NDP_RA_MIN = 12
NDP_NS_MIN = 20
NDP_NA_MIN = 20
NDP_TARGET_LLA = 8
NDP_HOP_LIMIT = 255
ICMPV6_PROTOCOL = 58

# (name, type, size) of TestICMPChecksumValidationSimple (icmp_test.go:368-462)
SIMPLE = [
    ("DstUnreachable", 1, ICMPV6_MIN),
    ("PacketTooBig", 2, ICMPV6_MIN),
    ("TimeExceeded", 3, ICMPV6_MIN),
    ("ParamProblem", 4, ICMPV6_MIN),
    ("EchoRequest", 128, 8),
    ("EchoReply", 129, 8),
    ("RouterSolicit", 133, ICMPV6_MIN),
    ("RouterAdvert", 134, ICMPV6_HEADER + NDP_RA_MIN),
    ("NeighborSolicit", 135, ICMPV6_HEADER + NDP_NS_MIN),
    ("NeighborAdvert", 136, ICMPV6_HEADER + NDP_NA_MIN + NDP_TARGET_LLA),
    ("RedirectMsg", 137, ICMPV6_MIN),
]

SIMPLE_BODY = 64
ERROR_BODY = IPV6_MIN + SIMPLE_BODY
# (name, type, size, payload size) of ...WithPayload (:567-635) and
# ...WithPayloadMultipleViews (:744-812): the same six rows
WITH_PAYLOAD = [
    ("DstUnreachable", 1, ICMPV6_MIN, ERROR_BODY),
    ("PacketTooBig", 2, ICMPV6_MIN, ERROR_BODY),
    ("TimeExceeded", 3, ICMPV6_MIN, ERROR_BODY),
    ("ParamProblem", 4, ICMPV6_MIN, ERROR_BODY),
    ("EchoRequest", 128, 8, SIMPLE_BODY),
    ("EchoReply", 129, 8, SIMPLE_BODY),
]


def ipv6_header(payload_len: int, next_header: int, hop_limit: int, src: bytes, dst: bytes) -> bytes:
    """IPv6.Encode (ipv6.go:197-204) with TrafficClass = FlowLabel = 0."""
    return struct.pack(">IHBB", 6 << 28, payload_len & 0xFFFF, next_header, hop_limit) + src + dst


def payload_bytes(size: int) -> bytes:
    """simpleBody / errorICMPBody (:548-565, :725-742)."""
    simple = bytes(range(SIMPLE_BODY))
    if size == SIMPLE_BODY:
        return simple
    assert size == ERROR_BODY
    return ipv6_header(SIMPLE_BODY, 10, 20, LLADDR0, LLADDR1) + simple


def cases():
    """[(label, tx_h, tx_views, rx_h, rx_views)]; src = lladdr1, dst = lladdr0."""
    out = []
    for name, typ, size in SIMPLE:
        pkt = bytearray(size)
        pkt[0] = typ
        out.append((f"simple/{name}", bytes(pkt), [], bytes(pkt), []))
    for name, typ, size, psize in WITH_PAYLOAD:
        pkt = bytearray(size + psize)
        pkt[0] = typ
        pkt[ICMPV6_PAYLOAD_OFFSET:ICMPV6_PAYLOAD_OFFSET + psize] = payload_bytes(psize)
        out.append((f"payload/{name}", bytes(pkt), [], bytes(pkt), []))
    for name, typ, size, psize in WITH_PAYLOAD:
        pkt = bytearray(size)
        pkt[0] = typ
        body = payload_bytes(psize)
        out.append((f"views/{name}", bytes(pkt), [body], bytes(pkt), [body]))
    return out


def with_checksum(h: bytes, value: int) -> bytes:
    b = bytearray(h)
    struct.pack_into(">H", b, 2, value & 0xFFFF)
    return bytes(b)


def oracle_checksum(O, h: bytes, src: bytes, dst: bytes, views) -> int:
    """ICMPv6Checksum (icmpv6.go:202-221) on the C oracle."""
    x = O.c_checksum(src, 0)
    x = O.c_checksum(dst, x)
    x = O.c_checksum(struct.pack(">I", len(h) + sum(len(v) for v in views)), x)
    x = O.c_checksum(bytes([0, 0, 0, ICMPV6_PROTOCOL]), x)
    for v in views:
        x = O.c_checksum(v, x)
    hz = bytearray(h)
    hz[2:4] = b"\0\0"
    return (~O.c_checksum(bytes(hz), x)) & 0xFFFF
