"""ORACLE — TEST INFRASTRUCTURE ONLY.  Not part of the product.

The checksum steps of google/netstack's receive and transmit paths for ONE
tcpip.PacketBuffer, restated call for call from the reference on top of the
checksum.go restatement in oracle.py (its C binding, for speed; both are
pinned by the reference's KATs).  tests/test_gpu_packet.py compares
ns_csum_packet_buffers (netstack_amd.packet) with these, packet by packet.

A packet is (hdr, views, size): the used bytes of its Header Prependable, its
Data views, and Data.Size() (the views' total may exceed it after
CapLength).  Nothing here is ever imported by netstack_amd.
"""
from __future__ import annotations

import struct

from oracle import c_checksum, c_checksum_vv_with_offset, c_pseudo_header, c_views_restart

INVALID, VALID, UNCHECKED, MALFORMED = 0, 1, 2, 3


def _cap(views, size):
    """VectorisedView.CapLength (view.go:82-103) on a list of byte strings."""
    out, left = [], size
    for v in views:
        if left <= 0:
            break
        out.append(bytes(v[:left]))
        left -= min(len(v), left)
    return out


def _trim_front(views, count):
    """VectorisedView.TrimFront (view.go:69-79)."""
    views = list(views)
    while count > 0 and views:
        if count < len(views[0]):
            views[0] = views[0][count:]
            return views
        count -= len(views[0])
        views.pop(0)
    return views


def _size(views):
    return sum(len(v) for v in views)


def _checksum_vv(views, initial):
    """ChecksumVV (checksum.go:61-63)."""
    return c_checksum_vv_with_offset(views, initial, 0, _size(views))


def _icmpv6_checksum(h: bytearray, src: bytes, dst: bytes, payload_views) -> int:
    """header.ICMPv6Checksum (icmpv6.go:202-221)."""
    xsum = c_checksum(src, 0)
    xsum = c_checksum(dst, xsum)
    xsum = c_checksum(struct.pack(">I", (len(h) + _size(payload_views)) & 0xFFFFFFFF), xsum)
    xsum = c_checksum(bytes([0, 0, 0, 58]), xsum)
    for v in payload_views:
        xsum = c_checksum(v, xsum)
    h2, h3 = h[2], h[3]
    h[2] = h[3] = 0
    xsum = (~c_checksum(bytes(h), xsum)) & 0xFFFF
    h[2], h[3] = h2, h3
    return xsum


def verify(hdr: bytes, views, size: int, net_proto: int | None = None):
    """The receive path for a packet as the link layer delivers it (Data =
    the IP packet): returns (verdict, ipv4 header sum, transport sum) — the
    sums as ns_csum_packet_buffers reports them (0 where none is taken).
    net_proto: the network protocol an Ethernet link picked by EtherType (4,
    6, or 0 for anything else); None: a headerless link, which picks it by the
    version nibble (packet_dispatchers.go:283-296)."""
    data = _cap(([bytes(hdr)] if len(hdr) else []) + [bytes(v) for v in views], size)
    first = data[0] if data else b""
    if not first:
        return MALFORMED, 0, 0
    ver = first[0] >> 4
    if net_proto is not None:
        if net_proto not in (4, 6):
            return UNCHECKED, 0, 0  # not IP: nothing the reference checksums
        if ver != net_proto:
            return MALFORMED, 0, 0  # IsValid's version check (header/ipv4.go:292, ipv6.go:218)
    if ver == 4:
        # IPv4 HandlePacket (network/ipv4/ipv4.go:341-353) + IsValid (header/ipv4.go:280-296)
        if len(first) < 20:
            return MALFORMED, 0, 0
        hlen = (first[0] & 0xF) * 4
        tlen = (first[2] << 8) | first[3]
        # `hlen > len(first)` is not in IsValid: there ipv4.go:348 reslices
        # headerView past its length (spare capacity) or panics.  This repo
        # makes it MALFORMED, i.e. RXChecksumUnknown for the stack (DESIGN.md
        # §7; pinned by tests/golden/rx_choices.json).
        if hlen < 20 or hlen > tlen or tlen > _size(data) or hlen > len(first):
            return MALFORMED, 0, 0
        net = c_checksum(first[:hlen], 0)  # IPv4.CalculateChecksum (ipv4.go:251-253), reported only
        src, dst, proto = first[12:16], first[16:20], first[9]
        more = first[6] & 0x20
        foff = ((((first[6] & 0x1F) << 8) | first[7]) << 3) & 0xFFFF  # FragmentOffset() (header/ipv4.go:167-169)
        data = _cap(_trim_front(data, hlen), tlen - hlen)
        if more or foff:
            # ipv4.go:355-373: a fragment without payload, or one whose
            # uint16 `last = offset + size - 1` wraps below its offset, is
            # dropped as malformed; any other goes to reassembly (:375-385),
            # and its transport checksum is checked only after that.
            size = _size(data)
            if size == 0 or ((foff + (size & 0xFFFF) - 1) & 0xFFFF) < foff:
                return MALFORMED, net, 0
            return UNCHECKED, net, 0
    elif ver == 6:
        # IPv6 HandlePacket (network/ipv6/ipv6.go:168-177) + IsValid (header/ipv6.go:207-222)
        if len(first) < 40:
            return MALFORMED, 0, 0
        plen = (first[4] << 8) | first[5]
        if plen > _size(data) - 40:
            return MALFORMED, 0, 0
        net = 0
        src, dst, proto = first[8:24], first[24:40], first[6]
        data = _cap(_trim_front(data, 40), plen)
    else:
        return MALFORMED, 0, 0
    tfirst = data[0] if data else b""
    if proto == 6:
        # stack DeliverTransportPacket: First() >= TCPMinimumSize; segment.parse
        # (transport/tcp/segment.go:145-181)
        if len(tfirst) < 20:
            return MALFORMED, net, 0
        off = (tfirst[12] >> 4) * 4
        if off < 20 or off > len(tfirst):
            return MALFORMED, net, 0
        xsum = c_pseudo_header(6, src, dst, _size(data) & 0xFFFF)  # :176
        xsum = c_checksum(tfirst[:off], xsum)                      # :177
        xsum = _checksum_vv(_trim_front(data, off), xsum)          # :178-179
        return (VALID if xsum == 0xFFFF else INVALID), net, xsum   # :180
    if proto == 1 and ver == 4:
        # handleICMP (network/ipv4/icmp.go:60-80): echo requests only
        if len(tfirst) < 8:
            return MALFORMED, net, 0
        if tfirst[0] != 8:
            return UNCHECKED, net, 0
        want = (tfirst[2] << 8) | tfirst[3]
        z = [bytearray(v) for v in data]
        z[0][2] = z[0][3] = 0  # h.SetChecksum(0)
        s = _checksum_vv([bytes(v) for v in z], 0)
        got = (~s) & 0xFFFF
        return (VALID if got == want else INVALID), net, s
    if proto == 58 and ver == 6:
        # handleICMP (network/ipv6/icmp.go:62-84): len(v) < ICMPv6MinimumSize
        # (= 8, header/icmpv6.go:35) is dropped at :68-71
        if len(tfirst) < 8:
            return MALFORMED, net, 0
        h = bytearray(tfirst)
        want = (h[2] << 8) | h[3]
        got = _icmpv6_checksum(h, src, dst, data[1:])
        return (VALID if got == want else INVALID), net, (~got) & 0xFFFF
    if proto == 17 and len(tfirst) < 8:
        # stack DeliverTransportPacket: First() >= UDPMinimumSize (stack/nic.go:
        # 851, header/udp.go:56); UDP takes no checksum on receive otherwise
        return MALFORMED, net, 0
    return UNCHECKED, net, 0


def fill(hdr: bytes, views, size: int):
    """The transmit path: Header holds the IP header and the transport header,
    Data the payload.  Returns (new header bytes, ipv4 header sum, transport
    sum) with the checksum fields written as the reference writes them."""
    h = bytearray(hdr)
    data = _cap([bytes(v) for v in views], size)
    total = len(h) + _size(data)
    ver = h[0] >> 4
    if ver == 4:
        hlen = (h[0] & 0xF) * 4
        src, dst, proto = bytes(h[12:16]), bytes(h[16:20]), h[9]
    else:
        hlen = 40
        src, dst, proto = bytes(h[8:24]), bytes(h[24:40]), h[6]
    t0, tl = hlen, total - hlen
    rest = [bytes(h[t0:])] + data  # everything after the IP header, as views
    tr = 0
    # an IPv4 fragment (MF or an offset) gets only its IP header checksum, as
    # writePacketFragments writes it (network/ipv4/ipv4.go:159-160)
    frag = ver == 4 and ((h[6] & 0x20) or (((h[6] & 0x1F) << 8) | h[7]))
    if frag:
        pass
    elif proto == 6:
        # buildTCPHdr (transport/tcp/connect.go:653-663)
        thl = (h[t0 + 12] >> 4) * 4
        xsum = c_pseudo_header(6, src, dst, tl & 0xFFFF)
        payload = _trim_front(rest, thl)
        xsum = c_checksum_vv_with_offset(payload, xsum, 0, _size(payload))
        tr = c_checksum(bytes(h[t0:t0 + thl]), xsum)   # tcp.CalculateChecksum (tcp.go:259-262)
        struct.pack_into(">H", h, t0 + 16, (~tr) & 0xFFFF)
    elif proto == 17:
        # sendUDP (transport/udp/endpoint.go:808-815)
        xsum = c_pseudo_header(17, src, dst, tl & 0xFFFF)
        xsum = c_views_restart([v for v in _trim_front(rest, 8) if True], xsum)
        tr = c_checksum(bytes(h[t0:t0 + 8]), xsum)     # udp.CalculateChecksum (udp.go:104-107)
        struct.pack_into(">H", h, t0 + 6, (~tr) & 0xFFFF)
    elif proto == 1 and ver == 4:
        # echo reply (network/ipv4/icmp.go:96-100): pkt = the ICMP bytes in Header
        pkt = h[t0:]
        pkt[2] = pkt[3] = 0
        tr = c_checksum(bytes(pkt), _checksum_vv(data, 0))
        struct.pack_into(">H", h, t0 + 2, (~tr) & 0xFFFF)
    elif proto == 58 and ver == 6:
        icm = h[t0:]
        v = _icmpv6_checksum(icm, src, dst, data)
        tr = (~v) & 0xFFFF
        struct.pack_into(">H", h, t0 + 2, v)
    net = 0
    if ver == 4:
        # addIPHeader (network/ipv4/ipv4.go:236): ip.SetChecksum(^ip.CalculateChecksum()),
        # over the header as encoded (the checksum field as it was)
        net = c_checksum(bytes(hdr[:hlen]), 0)
        struct.pack_into(">H", h, 10, (~net) & 0xFFFF)
    return bytes(h), net, tr


BUF_CONFIG = (128, 256, 256, 512, 1024, 2048, 4096, 8192, 16384, 32768)  # packet_dispatchers.go:30


def frame_views(frame: bytes, first_view: int = 128):
    """The views recvMMsgDispatcher hands up for a frame of len(frame) bytes
    (allocateViews + capViews, packet_dispatchers.go:214-245): BufConfig's
    buffers (the first one first_view bytes; 0: the frame as one view),
    the last one capped."""
    sizes = ((first_view,) + BUF_CONFIG[1:]) if first_view else (max(len(frame), 1),)
    out, at = [], 0
    for sz in sizes:
        if at >= len(frame):
            break
        out.append(bytes(frame[at:at + sz]))
        at += sz
    return out


def verify_frame(slot: bytes, rlen: int, frame_at: int = 0, link_hdr: int = 0, first_view: int = 0):
    """One slot of a receive ring (ns_csum_rx_ring): recvmmsg wrote rlen bytes
    into `slot`, the link frame starting at frame_at; recvMMsgDispatcher.
    dispatch (packet_dispatchers.go:258-317) then drops a frame of no more
    than link_hdr bytes, picks the network protocol (EtherType with an
    Ethernet header, else the version nibble), trims the link header off
    Data and delivers; verify() does the rest."""
    if rlen > len(slot):
        return MALFORMED, 0, 0  # longer than its slot: counted by the engine
    frame = bytes(slot[frame_at:rlen]) if rlen > frame_at else b""
    if len(frame) <= link_hdr:
        return MALFORMED, 0, 0
    views = frame_views(frame, first_view)
    size = len(frame) - link_hdr
    net_proto = None
    if link_hdr:
        et = (frame[12] << 8) | frame[13]
        net_proto = 4 if et == 0x0800 else 6 if et == 0x86DD else 0
        views = _trim_front(views, link_hdr)
    return verify(b"", views, size, net_proto)
