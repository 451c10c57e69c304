"""The receive-side contract: how the engine's per-packet verdicts reach
``segment.parse`` ("Receive").  A host-side mirror of the
Go patch a maintainer applies (go/netstack-hipcsum.patch), so its semantics
are testable here.

The reference has one switch for "someone else verified the checksum": the
link-wide ``CapabilityRXChecksumOffload`` (stack/registration.go:324-327),
with which ``segment.parse`` trusts *every* segment of the link
(transport/tcp/segment.go:166-173).  The engine's verdicts are per packet, and
an IPv4 fragment's transport checksum cannot be checked before reassembly
(network/ipv4/ipv4.go:355-385).  A link that advertised the bit would deliver
corrupted fragmented TCP unchecked, so the engine's link never advertises it.
Instead:

1. The link verifies each recvmmsg batch in one device pass
   (``verify_packet_buffers``) and records each packet's verdict in a new
   ``PacketBuffer.RXChecksum`` field: ``VALID`` -> ``RX_CHECKSUM_VALID``,
   ``INVALID`` -> ``RX_CHECKSUM_INVALID``, anything else (``UNCHECKED``:
   fragments, UDP, ...; ``MALFORMED``) -> ``RX_CHECKSUM_UNKNOWN``, the zero
   value.  It drops nothing: the stack's own checks drop malformed packets
   and count them as the reference does.
2. IPv4 ``HandlePacket`` resets the field to ``RX_CHECKSUM_UNKNOWN`` when it
   replaces ``Data`` with a reassembled payload (a fragment's verdict never
   describes the reassembled segment).
3. ``segment.parse``: the link capability still wins (unchanged); otherwise
   ``RX_CHECKSUM_VALID`` / ``RX_CHECKSUM_INVALID`` set ``csumValid`` without
   summing, and ``RX_CHECKSUM_UNKNOWN`` is verified as the reference verifies
   it (segment.go:174-180) — here by the engine, in one pass per delivered
   batch.  ``HandlePacket`` then counts ``ChecksumErrors`` exactly where the
   reference does (transport/tcp/endpoint.go:2108-2114): only for segments
   that reach a TCP endpoint, and at every level (stack, endpoint).

A link-side drop of INVALID packets would not be equivalent: the link cannot
reach the endpoint's own ``ReceiveErrors.ChecksumErrors``, and it would count
segments that the reference never parses (no endpoint, or not TCP).

Only IPv4/IPv6 + TCP are followed past the network layer; the rest of the
stack (demux, endpoints, ICMP) is out of scope.
"""
from __future__ import annotations

import heapq
import struct
from dataclasses import dataclass

from .buffer import NewVectorisedView, VectorisedView
from .packet import INVALID, VALID, PacketBuffer, verify_packet_buffers
from .tcp import verify_tcp_segments

RX_CHECKSUM_UNKNOWN = 0  # the zero value: the stack verifies the packet itself
RX_CHECKSUM_VALID = 1
RX_CHECKSUM_INVALID = 2


def rx_checksum_of(verdict: int) -> int:
    """The link's mapping of an NS_PKB_* verdict to PacketBuffer.RXChecksum."""
    if verdict == VALID:
        return RX_CHECKSUM_VALID
    if verdict == INVALID:
        return RX_CHECKSUM_INVALID
    return RX_CHECKSUM_UNKNOWN


@dataclass
class Stats:
    """The tcpip.Stats counters the receive path touches (tcpip.go:684-708,
    980-981)."""

    MalformedRcvdPackets: int = 0
    IPMalformedPacketsReceived: int = 0
    IPMalformedFragmentsReceived: int = 0
    IPPacketsDelivered: int = 0
    TCPInvalidSegmentsReceived: int = 0
    TCPChecksumErrors: int = 0
    TCPValidSegmentsReceived: int = 0
    EndpointChecksumErrors: int = 0  # e.stats.ReceiveErrors.ChecksumErrors


class _Reassembler:
    """fragmentation's reassembler for one datagram: the hole list
    (reassembler.go:62-79), the fragments kept only if they filled a hole
    (:91-95), and fragHeap.reassemble (frag_heap.go:57-77)."""

    def __init__(self):
        self.holes = [[0, 0xFFFF, False]]
        self.deleted = 0
        self.heap = []
        self.seq = 0

    def process(self, first: int, last: int, more: bool, vv: VectorisedView):
        used = False
        for h in list(self.holes):
            if h[2] or first > h[1] or last < h[0]:
                continue
            used = True
            self.deleted += 1
            h[2] = True
            if first > h[0]:
                self.holes.append([h[0], first - 1, False])
            if last < h[1] and more:
                self.holes.append([last + 1, h[1], False])
        if used:
            heapq.heappush(self.heap, (first, self.seq, vv.Clone(None)))
            self.seq += 1
        if self.deleted < len(self.holes):
            return None, True
        off, _, cur = heapq.heappop(self.heap)
        if off != 0:
            return None, False
        views, size = list(cur.Views()), cur.Size()
        while self.heap:
            off, _, cur = heapq.heappop(self.heap)
            if off < size:
                cur.TrimFront(size - off)
            elif off > size:
                return None, False
            size += cur.Size()
            views += cur.Views()
        return NewVectorisedView(size, views), True


class ReceivePath:
    """A link (recvmmsg batches) feeding IPv4/IPv6 HandlePacket and TCP
    HandlePacket/segment.parse, with the contract above.  ``deliver``
    returns the TCP segments a connected endpoint would enqueue:
    (src, dst, segment bytes) for every segment whose checksum holds."""

    def __init__(self, engine=None):
        self.engine = engine
        self.stats = Stats()
        self._frags: dict[tuple, _Reassembler] = {}

    # -- link: one device pass per batch --------------------------------------
    def link_verify(self, pkts) -> None:
        verdict, _ = verify_packet_buffers(pkts, self.engine)
        for pk, v in zip(pkts, verdict):
            pk.RXChecksum = rx_checksum_of(int(v))

    # -- network layer ---------------------------------------------------------
    def _ipv4(self, pk: PacketBuffer):
        """IPv4 HandlePacket (network/ipv4/ipv4.go:341-394) up to the
        transport dispatch: returns (proto, src, dst, pk) or None."""
        first = pk.Data.First()
        h = bytes(first) if first is not None else b""
        size = pk.Data.Size()
        hlen = (h[0] & 0xF) * 4 if h else 0
        tlen = struct.unpack_from(">H", h, 2)[0] if len(h) >= 4 else 0
        # IsValid (header/ipv4.go:280-296); `hlen > len(h)` is this repo's choice
        # where ipv4.go:348 reslices past the view or panics (DESIGN.md §7,
        # tests/golden/rx_choices.json)
        if len(h) < 20 or hlen < 20 or hlen > tlen or tlen > size or hlen > len(h):
            self.stats.IPMalformedPacketsReceived += 1
            return None
        src, dst, proto, ident = h[12:16], h[16:20], h[9], struct.unpack_from(">H", h, 4)[0]
        pk.Data.TrimFront(hlen)
        pk.Data.CapLength(tlen - hlen)
        more = bool(h[6] & 0x20)
        foff = ((((h[6] & 0x1F) << 8) | h[7]) << 3) & 0xFFFF
        if more or foff:
            if pk.Data.Size() == 0:
                self.stats.IPMalformedPacketsReceived += 1
                self.stats.IPMalformedFragmentsReceived += 1
                return None
            last = (foff + pk.Data.Size() - 1) & 0xFFFF
            if last < foff:
                self.stats.IPMalformedPacketsReceived += 1
                self.stats.IPMalformedFragmentsReceived += 1
                return None
            key = (ident, proto, src, dst)  # hash.IPv4FragmentHash's inputs
            r = self._frags.setdefault(key, _Reassembler())
            data, ok = r.process(foff, last, more, pk.Data)
            if not ok:
                del self._frags[key]
                self.stats.IPMalformedPacketsReceived += 1
                self.stats.IPMalformedFragmentsReceived += 1
                return None
            if data is None:
                return None
            del self._frags[key]
            pk.Data = data
            pk.RXChecksum = RX_CHECKSUM_UNKNOWN  # contract step 2
        self.stats.IPPacketsDelivered += 1
        return proto, src, dst, pk

    def _ipv6(self, pk: PacketBuffer):
        """IPv6 HandlePacket (network/ipv6/ipv6.go:168-184)."""
        first = pk.Data.First()
        h = bytes(first) if first is not None else b""
        if len(h) < 40 or struct.unpack_from(">H", h, 4)[0] > pk.Data.Size() - 40:  # IsValid
            return None
        pk.Data.TrimFront(40)
        pk.Data.CapLength(struct.unpack_from(">H", h, 4)[0])
        self.stats.IPPacketsDelivered += 1
        return h[6], h[8:24], h[24:40], pk

    def network(self, pk: PacketBuffer):
        """HandlePacket of the network layer, then the transport dispatch's
        TCP checks: returns (src, dst, pk) for a TCP segment that reaches
        segment.parse's checksum step, else None (counted where the
        reference counts it)."""
        first = pk.Data.First()
        ver = (bytes(first[:1])[0] >> 4) if first is not None and len(first) else 0
        if ver not in (4, 6):
            return None
        if len(first) < (20 if ver == 4 else 40):  # NIC.DeliverNetworkPacket (nic.go:774-777)
            self.stats.MalformedRcvdPackets += 1
            return None
        r = self._ipv4(pk) if ver == 4 else self._ipv6(pk)
        if r is None or r[0] != 6:
            return None
        _, src, dst, pk = r
        tf = pk.Data.First()
        if tf is None or len(tf) < 20:  # stack DeliverTransportPacket (nic.go:851-854)
            self.stats.MalformedRcvdPackets += 1
            return None
        off = (bytes(tf[12:13])[0] >> 4) * 4
        if off < 20 or off > len(tf):  # segment.parse (segment.go:158-161)
            self.stats.MalformedRcvdPackets += 1
            self.stats.TCPInvalidSegmentsReceived += 1
            return None
        return bytes(src), bytes(dst), pk

    def transport(self, segs):
        """segment.parse's checksum step (contract step 3) and tcp
        HandlePacket's counting (endpoint.go:2098-2123) for the batch's
        segments: the link's verdict is trusted, the rest verified in one
        device pass."""
        unknown = [k for k, s in enumerate(segs) if s[2].RXChecksum == RX_CHECKSUM_UNKNOWN]
        checked = verify_tcp_segments([(segs[k][0], segs[k][1], segs[k][2].Data) for k in unknown],
                                      self.engine) if unknown else []
        valid = [s[2].RXChecksum == RX_CHECKSUM_VALID for s in segs]
        for k, ok in zip(unknown, checked):
            valid[k] = ok
        out = []
        for (src, dst, pk), ok in zip(segs, valid):
            if not ok:
                self.stats.MalformedRcvdPackets += 1
                self.stats.TCPChecksumErrors += 1
                self.stats.EndpointChecksumErrors += 1
                continue
            self.stats.TCPValidSegmentsReceived += 1
            out.append((src, dst, b"".join(bytes(v) for v in pk.Data.Views())[:pk.Data.Size()]))
        return out

    def deliver(self, pkts):
        """One recvmmsg batch through the link, the network layer and TCP."""
        self.link_verify(pkts)
        segs = [s for s in (self.network(pk) for pk in pkts) if s is not None]
        return self.transport(segs)
