"""Batched TCP transmit and receive checksums — the callers of the hot path
(SURVEY.md §8(f) ranks 1-3), mirrored from google/netstack:

* TX: ``sendTCPBatch`` (tcpip/transport/tcp/connect.go:668-702) cuts a GSO
  payload into MSS segments and calls ``buildTCPHdr`` (:634-666) for each:
  ``xsum = PseudoHeaderChecksum(6, src, dst, hdrLen+size)``,
  ``xsum = ChecksumVVWithOffset(data, xsum, off, size)``,
  ``tcp.SetChecksum(^tcp.CalculateChecksum(xsum))`` (tcp.go:259-262).
* RX: ``segment.parse`` (tcp/segment.go:166-181) verifies
  ``ChecksumVV(payload, CalculateChecksum(PseudoHeaderChecksum(...))) == 0xffff``.

Here every segment's whole checksum — pseudo-header fields, payload views and
the TCP header itself — is one chain of ``ns_csum_chains``, and all segments
of a batch go to the GPU in ONE device pass.  The host only encodes header
fields (tcp.go:276-291) and slices views (the view walk of checksum.go:72-96);
it performs no checksum arithmetic.
"""
from __future__ import annotations

import struct
from dataclasses import dataclass, field

from .buffer import VectorisedView, View
from .engine import default_engine

PROTOCOL_NUMBER = 6          # header.TCPProtocolNumber
TCP_MINIMUM_SIZE = 20        # header.TCPMinimumSize
TCP_CHECKSUM_OFFSET = 16     # header.TCPChecksumOffset (tcp.go:34)


@dataclass
class TCPFields:
    """header.TCPFields (tcp.go) — the fields Encode writes."""

    SrcPort: int = 0
    DstPort: int = 0
    SeqNum: int = 0
    AckNum: int = 0
    DataOffset: int = TCP_MINIMUM_SIZE
    Flags: int = 0
    WindowSize: int = 0
    Checksum: int = 0
    UrgentPointer: int = 0


def encode_tcp(f: TCPFields, opts: bytes = b"") -> bytearray:
    """header.TCP.Encode (tcp.go:276-291) + the option copy of buildTCPHdr
    (connect.go:652)."""
    b = bytearray(f.DataOffset)
    struct.pack_into(">HHIIBBHHH", b, 0, f.SrcPort & 0xFFFF, f.DstPort & 0xFFFF,
                     f.SeqNum & 0xFFFFFFFF, f.AckNum & 0xFFFFFFFF, (f.DataOffset // 4) << 4,
                     f.Flags & 0xFF, f.WindowSize & 0xFFFF, f.Checksum & 0xFFFF,
                     f.UrgentPointer & 0xFFFF)
    b[TCP_MINIMUM_SIZE:TCP_MINIMUM_SIZE + len(opts)] = opts
    return b


def _clip(vv: VectorisedView, off: int, size: int):
    """The view walk of ChecksumVVWithOffset (checksum.go:72-96): the byte
    ranges of vv in [off, off+size), empty views skipped."""
    out = []
    for v in vv.Views():
        m = v.memory if isinstance(v, View) else memoryview(v)
        if len(m) == 0:
            continue
        if off >= len(m):
            off -= len(m)
            continue
        m = m[off:]
        m = m[: min(len(m), size)]
        out.append(m)
        size -= len(m)
        if size == 0:
            break
        off = 0
    return out


def _pseudo_pieces(src: bytes, dst: bytes, total_len: int, protocol: int = PROTOCOL_NUMBER):
    """PseudoHeaderChecksum (checksum.go:112-122) as four restart pieces."""
    return [(bytes(src), True), (bytes(dst), True),
            (struct.pack(">H", total_len & 0xFFFF), True), (bytes([0, protocol & 0xFF]), True)]


@dataclass
class PacketDescriptor:
    """stack.PacketDescriptor (stack/route.go:174-178): header bytes + the
    payload range it carries."""

    Hdr: bytearray = field(default_factory=bytearray)
    Off: int = 0
    Size: int = 0


@dataclass
class NetworkHeaderParams:
    """stack.NetworkHeaderParams (stack/registration.go) plus the IPv4 id
    counter addIPHeader draws from (ipv4.go:221-225): ``ID`` is the counter's
    value before this batch; each packet longer than 68 B takes the next id."""

    TTL: int = 64
    TOS: int = 0
    ID: int = 0


IPV4_MINIMUM_SIZE = 20
IPV4_MAXIMUM_HEADER_SIZE = 60


def _ipv4_header(params: NetworkHeaderParams, length: int, src: bytes, dst: bytes) -> bytearray:
    """addIPHeader's Encode (network/ipv4/ipv4.go:217-235), checksum left 0."""
    ident = 0
    if length > IPV4_MAXIMUM_HEADER_SIZE + 8:
        params.ID = (params.ID + 1) & 0xFFFFFFFF
        ident = params.ID
    b = bytearray(IPV4_MINIMUM_SIZE)
    struct.pack_into(">BBHHHBBH4s4s", b, 0, 0x45, params.TOS & 0xFF, length & 0xFFFF, ident & 0xFFFF,
                     0, params.TTL & 0xFF, PROTOCOL_NUMBER, 0, bytes(src), bytes(dst))
    return b


def send_tcp_batch(data: VectorisedView, mss: int, local_addr: bytes, remote_addr: bytes,
                   src_port: int, dst_port: int, flags: int, seq: int, ack: int, rcv_wnd: int,
                   opts: bytes = b"", tx_checksum_offload: bool = False,
                   gso_needs_csum: bool = False, ipv4: NetworkHeaderParams | None = None,
                   engine=None) -> list[PacketDescriptor]:
    """sendTCPBatch + buildTCPHdr (connect.go:634-702) for one GSO payload:
    returns the n PacketDescriptors with fully encoded, checksummed TCP
    headers.  All n checksums come from one device pass.

    With ``ipv4`` set, the IPv4 network endpoint's WritePackets step is fused
    in (network/ipv4/ipv4.go:271-285 -> addIPHeader :217-238, SURVEY §8(f)
    rank 3): every Hdr gets its 20-B IPv4 header prepended, and the n IPv4
    header checksums ride in the same device pass as the n TCP checksums."""
    if rcv_wnd > 0xFFFF:
        rcv_wnd = 0xFFFF
    eng = engine or default_engine()
    n = (data.Size() + mss - 1) // mss
    hdr_len = TCP_MINIMUM_SIZE + len(opts)
    descs, chains = [], []
    size, off = data.Size(), 0
    for _ in range(n):
        psize = min(mss, size)
        size -= psize
        h = encode_tcp(TCPFields(src_port, dst_port, seq, ack, hdr_len, flags, rcv_wnd), opts)
        length = hdr_len + psize
        d = PacketDescriptor(h, off, psize)
        descs.append(d)
        if gso_needs_csum:
            # CHECKSUM_PARTIAL: only the pseudo-header sum goes in (connect.go:655-660)
            chains.append(_pseudo_pieces(local_addr, remote_addr, length))
        elif not tx_checksum_offload:
            payload = _clip(data, off, psize)
            ch = _pseudo_pieces(local_addr, remote_addr, length)
            ch += [(p, k == 0) for k, p in enumerate(payload)] or [(b"", True)]
            ch.append((bytes(h), True))        # tcp.CalculateChecksum(xsum): Checksum(tcp[:DataOffset], xsum)
            chains.append(ch)
        off += psize
        seq = (seq + psize) & 0xFFFFFFFF
    ntcp = len(chains)
    ips = []
    if ipv4 is not None:
        for d in descs:
            ip = _ipv4_header(ipv4, IPV4_MINIMUM_SIZE + len(d.Hdr) + d.Size, local_addr, remote_addr)
            ips.append(ip)
            chains.append([(bytes(ip), True)])          # ip.CalculateChecksum()
    if chains:
        sums = eng.chains(chains)
        for d, s in zip(descs, sums[:ntcp]):
            v = int(s) if gso_needs_csum else (~int(s)) & 0xFFFF
            struct.pack_into(">H", d.Hdr, TCP_CHECKSUM_OFFSET, v)  # tcp.SetChecksum
        for d, ip, s in zip(descs, ips, sums[ntcp:]):
            struct.pack_into(">H", ip, 10, (~int(s)) & 0xFFFF)     # ip.SetChecksum(^...)
            d.Hdr[0:0] = ip                                        # hdr.Prepend
    return descs


def verify_tcp_segments(segments, engine=None) -> list[bool]:
    """segment.parse's checksum verification (segment.go:174-180) for a batch
    of received segments in one device pass.  Each segment is
    (src_addr, dst_addr, vv) where vv holds the TCP header + payload (the IP
    header already trimmed, as the stack does before parse) and the TCP header
    lies in the first view.  Returns csumValid per segment."""
    eng = engine or default_engine()
    chains = []
    for src, dst, vv in segments:
        first = vv.First()
        h = bytes(first[:TCP_MINIMUM_SIZE]) if first is not None else b""
        offset = (h[12] >> 4) * 4 if len(h) >= 13 else TCP_MINIMUM_SIZE
        ch = _pseudo_pieces(src, dst, vv.Size())                 # :176
        ch.append((bytes(first[:offset]), True))                 # :177 h.CalculateChecksum(xsum)
        payload = _clip(vv, offset, vv.Size() - offset)          # :178 TrimFront(offset)
        ch += [(p, k == 0) for k, p in enumerate(payload)]       # :179 ChecksumVV(s.data, xsum)
        chains.append(ch)
    sums = eng.chains(chains)
    return [int(s) == 0xFFFF for s in sums]                     # :180
