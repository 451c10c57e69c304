"""Mirror of google/netstack ``tcpip.PacketBuffer`` (tcpip/packet_buffer.go:
25-50) and the checksum steps of a batch of them, in one device pass through
``ns_csum_packet_buffers`` (include/netstack_csum.h):

* receive — ``verify_packet_buffers``: a recvmmsg batch as the link layer
  delivers it (``recvMMsgDispatcher.dispatch``, link/fdbased/
  packet_dispatchers.go:258-317: ``Data`` holds the IP packet over
  ``BufConfig`` views).  After IPv4/IPv6 ``HandlePacket``'s checks and trims
  (network/ipv4/ipv4.go:341-353, network/ipv6/ipv6.go:168-177): TCP
  ``segment.parse`` (transport/tcp/segment.go:174-180), the ICMPv4 echo check
  (network/ipv4/icmp.go:72-80), the ICMPv6 check (network/ipv6/icmp.go:76-84).
* transmit — ``fill_packet_buffers``: packets whose ``Header`` Prependable
  holds the IP and transport headers (``Data`` the payload) get the
  transport checksum of ``buildTCPHdr`` (transport/tcp/connect.go:653-663),
  ``sendUDP`` (transport/udp/endpoint.go:808-815), the ICMPv4 echo reply
  (network/ipv4/icmp.go:96-100) or ``ICMPv6Checksum`` (header/icmpv6.go:
  202-221), and the IPv4 header checksum of ``addIPHeader``
  (network/ipv4/ipv4.go:236), written into ``Header``.

The host reads header fields and cuts the packets into pieces (in
csum_api.cpp); every sum is computed by the gfx950 kernel.
"""
from __future__ import annotations

import ctypes
from dataclasses import dataclass, field

import numpy as np

from . import _lib
from .buffer import Prependable, VectorisedView, View
from .engine import _u8, default_engine

INVALID = _lib.NS_PKB_INVALID
VALID = _lib.NS_PKB_VALID
UNCHECKED = _lib.NS_PKB_UNCHECKED
MALFORMED = _lib.NS_PKB_MALFORMED


@dataclass
class PacketBuffer:
    """tcpip.PacketBuffer (packet_buffer.go:25-50)."""

    Data: VectorisedView = field(default_factory=VectorisedView)
    Header: Prependable = field(default_factory=Prependable)
    LinkHeader: View | None = None
    NetworkHeader: View | None = None
    TransportHeader: View | None = None
    # New with the receive contract (netstack_amd/rx.py):
    # the link's verdict on the transport checksum, 0 = not verified.
    RXChecksum: int = 0

    def Clone(self) -> "PacketBuffer":  # packet_buffer.go:55-58
        return PacketBuffer(self.Data.Clone(None), self.Header, self.LinkHeader, self.NetworkHeader,
                            self.TransportHeader, self.RXChecksum)


def _marshal(pkts):
    """ns_pkt_buf table over the packets' own bytes (no copies: the Header's
    View and the Data views are passed by address) + keep-alive list."""
    keep = []
    tab = (_lib.NsPktBuf * max(len(pkts), 1))()
    for i, pk in enumerate(pkts):
        hv = pk.Header.View()
        h = np.frombuffer(hv.memory, dtype=np.uint8) if len(hv) else np.zeros(0, np.uint8)
        views = [_u8(v.memory if isinstance(v, View) else v) for v in pk.Data.Views()]
        vt = (_lib.NsView * max(len(views), 1))(*[_lib.NsView(a.ctypes.data if a.size else None, a.size)
                                                   for a in views])
        keep += [h, views, vt]
        tab[i].hdr = h.ctypes.data if h.size else None
        tab[i].hdr_len = h.size
        tab[i].data = ctypes.cast(vt, ctypes.c_void_p)
        tab[i].ndata = len(views)
        tab[i].flags = 0
        tab[i].data_size = pk.Data.Size()
    return tab, keep


def _run(pkts, op, engine):
    eng = engine or default_engine()
    n = len(pkts)
    sums = np.zeros(2 * max(n, 1), dtype=np.uint16)
    verdict = np.zeros(max(n, 1), dtype=np.uint8)
    tab, keep = _marshal(pkts)
    _lib.check(_lib.lib().ns_csum_packet_buffers(
        eng._h, tab, n, op, sums.ctypes.data_as(ctypes.POINTER(ctypes.c_uint16)),
        verdict.ctypes.data_as(ctypes.POINTER(ctypes.c_uint8))), "ns_csum_packet_buffers")
    del keep
    return sums[:2 * n], verdict[:n]


def verify_packet_buffers(pkts, engine=None):
    """Receive-side verdicts for a batch (one device pass): returns
    (verdicts, sums) — verdicts[i] in {VALID, INVALID, UNCHECKED, MALFORMED};
    sums[2i] the IPv4 header sum (0xffff when intact; 0 for IPv6), sums[2i+1]
    the transport chain's un-complemented sum."""
    sums, verdict = _run(pkts, _lib.NS_PKB_VERIFY, engine)
    return verdict, sums


def fill_packet_buffers(pkts, engine=None):
    """Transmit side: writes every packet's transport and IPv4 header
    checksums into its Header (one device pass); returns the sums."""
    sums, _ = _run(pkts, _lib.NS_PKB_FILL, engine)
    return sums
