"""Batched per-protocol checksum callers (SURVEY.md §8(a) rows a7-a9 and
§8(f) ranks 3-4), mirrored from google/netstack and computed in one device
pass per batch through ``ns_csum_chains``:

* IPv4 header: ``IPv4.CalculateChecksum`` (header/ipv4.go:251-253),
  ``addIPHeader`` (network/ipv4/ipv4.go:217-238), ``IPv4.EncodePartial``
  (ipv4.go:273-277).
* UDP transmit: ``sendUDP`` (transport/udp/endpoint.go:794-815) — note its
  per-view restart ``xsum = Checksum(v, xsum)`` loop.
* ICMP: ``ICMPv4Checksum`` (header/icmpv4.go:155-169) and ``ICMPv6Checksum``
  (header/icmpv6.go:202-221).
* TCP incremental update: ``TCP.EncodePartial`` (header/tcp.go:295-314).

Field encoding and view slicing happen on the host; every sum is a chain of
restart/continue pieces evaluated by the gfx950 kernel.
"""
from __future__ import annotations

import struct
from dataclasses import dataclass

from .engine import default_engine

IPV4_MINIMUM_SIZE = 20
IPV4_TOTAL_LEN_OFFSET = 2
IPV4_CHECKSUM_OFFSET = 10
UDP_MINIMUM_SIZE = 8
UDP_CHECKSUM_OFFSET = 6
UDP_PROTOCOL_NUMBER = 17
ICMPV6_PROTOCOL_NUMBER = 58


def _views_of(vv):
    return [v.memory if hasattr(v, "memory") else memoryview(v) for v in vv.Views()]


def _restart_all(bufs):
    return [(bytes(b), True) for b in bufs]


# ---- IPv4 ------------------------------------------------------------------
@dataclass
class IPv4Fields:
    """header.IPv4Fields (ipv4.go) — what Encode writes."""

    IHL: int = IPV4_MINIMUM_SIZE
    TOS: int = 0
    TotalLength: int = 0
    ID: int = 0
    Flags: int = 0
    FragmentOffset: int = 0
    TTL: int = 64
    Protocol: int = 6
    Checksum: int = 0
    SrcAddr: bytes = bytes(4)
    DstAddr: bytes = bytes(4)


def encode_ipv4(f: IPv4Fields) -> bytearray:
    """header.IPv4.Encode (ipv4.go:256-267)."""
    b = bytearray(f.IHL)
    b[0] = (4 << 4) | ((f.IHL // 4) & 0xF)
    b[1] = f.TOS & 0xFF
    struct.pack_into(">HHH", b, 2, f.TotalLength & 0xFFFF, f.ID & 0xFFFF,
                     ((f.Flags & 0x7) << 13) | (f.FragmentOffset >> 3 & 0x1FFF))
    b[8] = f.TTL & 0xFF
    b[9] = f.Protocol & 0xFF
    struct.pack_into(">H", b, IPV4_CHECKSUM_OFFSET, f.Checksum & 0xFFFF)
    b[12:16] = bytes(f.SrcAddr)[:4]
    b[16:20] = bytes(f.DstAddr)[:4]
    return b


def ipv4_calculate_checksums(headers, engine=None) -> list[int]:
    """[IPv4(h).CalculateChecksum() for h in headers] (ipv4.go:251-253):
    Checksum(b[:HeaderLength()], 0), one device pass."""
    eng = engine or default_engine()
    chains = [[(bytes(h[: (h[0] & 0xF) * 4]), True)] for h in headers]
    return [int(x) for x in eng.chains(chains)]


def add_ip_headers(headers, engine=None) -> None:
    """addIPHeader's checksum step for a batch of encoded headers
    (network/ipv4/ipv4.go:236: ip.SetChecksum(^ip.CalculateChecksum())).
    `headers` are bytearrays whose checksum field is the value to include
    (zero after Encode)."""
    sums = ipv4_calculate_checksums(headers, engine)
    for h, s in zip(headers, sums):
        struct.pack_into(">H", h, IPV4_CHECKSUM_OFFSET, (~s) & 0xFFFF)


def ipv4_encode_partial(headers, partials, total_lengths, engine=None) -> None:
    """IPv4.EncodePartial (ipv4.go:273-277) over a batch: set TotalLength,
    checksum := Checksum(b[2:4], partial), SetChecksum(^checksum)."""
    eng = engine or default_engine()
    chains = []
    for h, p, tl in zip(headers, partials, total_lengths):
        struct.pack_into(">H", h, IPV4_TOTAL_LEN_OFFSET, tl & 0xFFFF)
        chains.append([("init", p), (bytes(h[IPV4_TOTAL_LEN_OFFSET:IPV4_TOTAL_LEN_OFFSET + 2]), True)])
    for h, s in zip(headers, eng.chains(chains)):
        struct.pack_into(">H", h, IPV4_CHECKSUM_OFFSET, (~int(s)) & 0xFFFF)


# ---- UDP -------------------------------------------------------------------
def encode_udp(src_port: int, dst_port: int, length: int, checksum: int = 0) -> bytearray:
    """header.UDP.Encode (udp.go:110-116)."""
    return bytearray(struct.pack(">HHHH", src_port & 0xFFFF, dst_port & 0xFFFF, length & 0xFFFF,
                                 checksum & 0xFFFF))


def _pseudo(protocol, src, dst, total_len):
    return [(bytes(src), True), (bytes(dst), True), (struct.pack(">H", total_len & 0xFFFF), True),
            (bytes([0, protocol & 0xFF]), True)]


def send_udp_batch(datagrams, tx_checksum_offload: bool = False, engine=None) -> list[bytearray]:
    """sendUDP's header + checksum (udp/endpoint.go:800-815) for a batch of
    (vv, local_addr, remote_addr, src_port, dst_port): returns the encoded
    UDP headers with the checksum field set.  Note the per-view restart:
    ``for v in data.Views(): xsum = Checksum(v, xsum)``."""
    eng = engine or default_engine()
    hdrs, chains = [], []
    for vv, src, dst, sp, dp in datagrams:
        length = UDP_MINIMUM_SIZE + vv.Size()
        h = encode_udp(sp, dp, length)
        hdrs.append(h)
        ch = _pseudo(UDP_PROTOCOL_NUMBER, src, dst, length)
        ch += _restart_all(_views_of(vv))
        ch.append((bytes(h[:UDP_MINIMUM_SIZE]), True))   # udp.CalculateChecksum(xsum)
        chains.append(ch)
    if not tx_checksum_offload and chains:
        for h, s in zip(hdrs, eng.chains(chains)):
            struct.pack_into(">H", h, UDP_CHECKSUM_OFFSET, (~int(s)) & 0xFFFF)
    return hdrs


# ---- ICMP ------------------------------------------------------------------
def icmpv4_checksums(items, engine=None) -> list[int]:
    """[ICMPv4Checksum(h, vv) for (h, vv) in items] (icmpv4.go:155-169): the
    payload views restart per view, then ^Checksum(h with h[2:4] zeroed)."""
    eng = engine or default_engine()
    chains = []
    for h, vv in items:
        hz = bytearray(h)
        hz[2:4] = b"\0\0"
        chains.append(_restart_all(_views_of(vv)) + [(bytes(hz), True)])
    return [(~int(s)) & 0xFFFF for s in eng.chains(chains)]


def icmpv6_checksums(items, engine=None) -> list[int]:
    """[ICMPv6Checksum(h, src, dst, vv) ...] (icmpv6.go:202-221): IPv6
    pseudo-header (src, dst, u32 upper-layer length, {0,0,0,58}), payload
    views restarting per view, then ^Checksum(h with h[2:4] zeroed)."""
    eng = engine or default_engine()
    chains = []
    for h, src, dst, vv in items:
        hz = bytearray(h)
        hz[2:4] = b"\0\0"
        ch = [(bytes(src), True), (bytes(dst), True),
              (struct.pack(">I", (len(h) + vv.Size()) & 0xFFFFFFFF), True),
              (bytes([0, 0, 0, ICMPV6_PROTOCOL_NUMBER]), True)]
        ch += _restart_all(_views_of(vv))
        ch.append((bytes(hz), True))
        chains.append(ch)
    return [(~int(s)) & 0xFFFF for s in eng.chains(chains)]


# ---- TCP incremental update --------------------------------------------------
def tcp_encode_partial(headers, partials, lengths, seqnums, acknums, flags, rcvwnds,
                       engine=None) -> None:
    """TCP.EncodePartial (tcp.go:295-314) over a batch of headers, in place:
    checksum := Checksum({length, uint16(flags)}, partial); encodeSubset;
    checksum = Checksum(b[4:12], checksum); checksum = Checksum(b[14:16],
    checksum); SetChecksum(^checksum)."""
    eng = engine or default_engine()
    chains = []
    for h, p, ln, sq, ak, fl, wn in zip(headers, partials, lengths, seqnums, acknums, flags, rcvwnds):
        struct.pack_into(">IIBBH", h, 4, sq & 0xFFFFFFFF, ak & 0xFFFFFFFF, h[12], fl & 0xFF, wn & 0xFFFF)
        chains.append([("init", p), (struct.pack(">HH", ln & 0xFFFF, fl & 0xFF), True),
                       (bytes(h[4:12]), True), (bytes(h[14:16]), True)])
    for h, s in zip(headers, eng.chains(chains)):
        struct.pack_into(">H", h, 16, (~int(s)) & 0xFFFF)
