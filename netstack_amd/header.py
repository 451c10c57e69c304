"""Mirror of google/netstack ``tcpip/header`` checksum entry points
(tcpip/header/checksum.go) — same names, argument meaning and results — with
every sum computed by the gfx950 engine through the C ABI.

Reference functions mirrored (all results un-complemented, like Go):

=========================  ===============================  =====================
Go (checksum.go)           here                             C ABI
=========================  ===============================  =====================
Checksum :52-55            Checksum(buf, initial)           ns_csum_checksum
ChecksumVV :61-63          ChecksumVV(vv, initial)          ns_csum_vv_with_offset
ChecksumVVWithOffset       ChecksumVVWithOffset(vv, ...)    ns_csum_vv_with_offset
:69-98
ChecksumCombine :104-107   ChecksumCombine(a, b)            ns_csum_combine
PseudoHeaderChecksum       PseudoHeaderChecksum(p, s, d, l) ns_csum_pseudo_header
:112-122
(new) sendTCPBatch's n x   ChecksumVVBatch(vv, descs)       ns_csum_vv_batch
ChecksumVVWithOffset
(connect.go:668-702)
(callers' per-view loop,   ChecksumViews(views, initial)    ns_csum_views_restart
udp/endpoint.go:811-813)
=========================  ===============================  =====================

Error behaviour: where Go panics (a negative ``off``/``size`` slice bound),
these raise ``ValueError``; a HIP failure raises ``ChecksumError``.  There is
no host fallback.
"""
from __future__ import annotations

from .buffer import VectorisedView, View
from .engine import combine, default_engine


def _mem(v):
    if isinstance(v, View):
        return v.memory
    return v


def Checksum(buf, initial: int = 0) -> int:
    """header.Checksum (checksum.go:52-55): RFC 1071 sum of `buf` seeded with
    `initial` (which must cover an even number of bytes)."""
    return default_engine().checksum(_mem(buf), initial)


def ChecksumVVWithOffset(vv: VectorisedView, initial: int, off: int, size: int) -> int:
    """header.ChecksumVVWithOffset (checksum.go:69-98)."""
    return default_engine().vv_with_offset([_mem(v) for v in vv.Views()], initial, off, size)


def ChecksumVV(vv: VectorisedView, initial: int) -> int:
    """header.ChecksumVV (checksum.go:61-63)."""
    return ChecksumVVWithOffset(vv, initial, 0, vv.Size())


def ChecksumCombine(a: int, b: int) -> int:
    """header.ChecksumCombine (checksum.go:104-107)."""
    return combine(a, b)


def PseudoHeaderChecksum(protocol: int, srcAddr: bytes, dstAddr: bytes, totalLen: int) -> int:
    """header.PseudoHeaderChecksum (checksum.go:112-122); addresses are the
    raw 4- or 16-byte tcpip.Address strings (tcpip.go:146)."""
    return default_engine().pseudo_header(protocol, srcAddr, dstAddr, totalLen)


def ChecksumVVBatch(vv: VectorisedView, descs) -> list[int]:
    """n x ChecksumVVWithOffset(vv, d.initial, d.Off, d.Size) in one device
    pass — the batch sendTCPBatch needs (connect.go:668-702, one descriptor
    per MSS segment, stack.PacketDescriptor route.go:174-178).

    `descs`: iterable of objects with Off/Size/initial attributes, or of
    (off, size, initial) tuples."""
    segs = []
    for d in descs:
        if isinstance(d, tuple):
            segs.append(d)
        else:
            segs.append((d.Off, d.Size, getattr(d, "initial", 0)))
    return [int(x) for x in default_engine().vv_batch([_mem(v) for v in vv.Views()], segs)]


def ChecksumViews(views, initial: int) -> int:
    """`xsum = initial; for v in views: xsum = Checksum(v, xsum)` — the
    per-view-restart loop of sendUDP (udp/endpoint.go:811-813) and
    ICMPv4Checksum / ICMPv6Checksum (icmpv4.go:158-160, icmpv6.go:210-212)."""
    return default_engine().views_restart([_mem(v) for v in views], initial)
