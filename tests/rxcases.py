"""Test infrastructure for the receive-path cases (tests/test_rx_contract.py,
tests/test_gpu_rx_contract.py): the reference's packet-level fixtures
(tests/golden/rx_fixtures.json) and the two packet builders its tests use,
restated on the oracle.  Not part of the product."""
from __future__ import annotations

import json
import os
import struct

import oracle as O

HERE = os.path.dirname(os.path.abspath(__file__))


def fixtures():
    with open(os.path.join(HERE, "golden", "rx_fixtures.json")) as f:
        return json.load(f)


def view_sizes(spec):
    return [spec["repeat"]] * spec["count"] if isinstance(spec, dict) else list(spec)


def _ipv4_set_checksum(h: bytearray, hl: int) -> None:
    """ip.SetChecksum(0); ip.SetChecksum(^ip.CalculateChecksum())."""
    struct.pack_into(">H", h, 10, 0)
    struct.pack_into(">H", h, 10, (~O.c_checksum(bytes(h[:hl]), 0)) & 0xFFFF)


def build_segment(src: bytes, dst: bytes, src_port: int, dst_port: int, seq: int, ack: int, flags: int,
                  window: int, payload: bytes, ttl: int = 65, ident: int = 0) -> bytearray:
    """testing/context BuildSegmentWithAddrs (context.go:317-356): one IPv4 +
    TCP packet with both checksums set."""
    buf = bytearray(40 + len(payload))
    buf[40:] = payload
    struct.pack_into(">BBHHHBBH4s4s", buf, 0, 0x45, 0, len(buf), ident, 0, ttl, 6, 0, src, dst)
    _ipv4_set_checksum(buf, 20)
    struct.pack_into(">HHIIBBHHH", buf, 20, src_port, dst_port, seq & 0xFFFFFFFF, ack & 0xFFFFFFFF, 5 << 4,
                     flags, window, 0, 0)
    xsum = O.c_pseudo_header(6, src, dst, len(buf) - 20)
    xsum = O.c_checksum(payload, xsum)
    xsum = O.c_checksum(bytes(buf[20:40]), xsum)  # t.CalculateChecksum(xsum)
    struct.pack_into(">H", buf, 36, (~xsum) & 0xFFFF)
    return buf


def _cap(views, n):
    out = []
    for v in views:
        if n <= 0:
            break
        out.append(bytes(v[:n]))
        n -= min(len(v), n)
    return out


def _trim(views, n):
    views = list(views)
    while n > 0 and views:
        if n < len(views[0]):
            views[0] = views[0][n:]
            return views
        n -= len(views[0])
        views.pop(0)
    return views


def write_packet_fragments(hdr: bytes, data, mtu: int, set_checksums: bool = True):
    """IPv4 writePacketFragments (network/ipv4/ipv4.go:119-212) on bytes:
    `hdr` is pkt.Header's used bytes (the IP header first), `data` the
    payload views.  Returns [(header bytes, data views)] per fragment; the IP
    header checksums are written as :159-160 writes them, or left 0 for the
    engine to fill (set_checksums=False)."""
    ip = bytearray(hdr)
    hl = (ip[0] & 0xF) * 4
    if len(ip) + sum(len(v) for v in data) <= mtu:  # WritePacket sends it whole (ipv4.go:260-265)
        if set_checksums:
            _ipv4_set_checksum(ip, hl)
        return [(bytes(ip), [bytes(v) for v in data])]
    flags = ip[6] >> 5
    offset = (((ip[6] & 0x1F) << 8) | ip[7]) << 3
    payload_len = struct.unpack_from(">H", ip, 2)[0] - hl  # ip.PayloadLength()
    inner = (mtu - hl) & ~7
    n = (payload_len + inner - 1) // inner
    outer = inner + hl
    data = [bytes(v) for v in data]
    first_hdr = ip  # pkt.Header's bytes, the first fragment's IP header in place
    out = []
    for i in range(n):
        h = first_hdr if i == 0 else bytearray(first_hdr[:hl])
        rest = sum(len(v) for v in data)
        if i != n - 1:
            total, fl = outer, flags | 0x1  # IPv4FlagMoreFragments
        else:
            total, fl = hl + rest, flags
        struct.pack_into(">H", h, 2, total)
        struct.pack_into(">H", h, 6, (fl << 13) | (offset >> 3))
        if set_checksums:
            _ipv4_set_checksum(h, hl)
        else:
            struct.pack_into(">H", h, 10, 0)
        offset += inner
        if i > 0:
            piece = _cap(data, inner)
            out.append((bytes(h), piece))
            data = _trim(data, sum(len(v) for v in piece))
            continue
        if outer >= len(first_hdr):
            npl = outer - len(first_hdr)
            out.append((first_hdr, _cap(data, npl)))
            data = _trim(data, npl)
        else:
            out.append((first_hdr[:outer], []))
            data = [bytes(first_hdr[outer:])] + data
    return [(bytes(h), d) for h, d in out]


def ipv6_rows(fx):
    """tests/golden/rx_fixtures.json ipv6_receive, each packet intact and
    with its checksum field's low bit flipped (ICMPv6 -> INVALID, as
    handleICMP counts it, network/ipv6/icmp.go:79-82; UDP stays UNCHECKED)."""
    import packets as P

    rows = []
    for c in fx["ipv6_receive"]:
        b = bytes.fromhex(c["packet"])
        at = 40 + (6 if b[6] == 17 else 2)
        bad = bytearray(b)
        bad[at + 1] ^= 1
        rows.append((c["name"], b, c["verdict"]))
        rows.append((c["name"] + "/bad", bytes(bad), P.UNCHECKED if b[6] == 17 else P.INVALID))
    return rows



def control_rows(fx):
    """tests/golden/rx_fixtures.json receive_control: TestIPv4ReceiveControl's
    and TestIPv6ReceiveControl's ICMP errors at each case's cut, with the
    verdict each owes (network/ip_test.go:293-398, :534-650)."""
    return [(c["name"], bytes.fromhex(c["packet"]), c["verdict"]) for c in fx["receive_control"]]


def fill_rows(fx):
    """The packets of rx_fixtures.json whose checksum the reference's own
    tests computed (ipv6_test.go / ndp_test.go: ICMPv6Checksum over the
    message, UDP's ^CalculateChecksum over the pseudo-header; ip_test.go
    TestIPv6ReceiveControl's uncut ICMPv6 errors), each with that field
    zeroed: (name, zeroed packet, the packet as the test built it)."""
    rows = []
    for c in fx["ipv6_receive"] + [c for c in fx["receive_control"] if c["name"].startswith("ipv6/") and c["verdict"] == 1]:
        b = bytes.fromhex(c["packet"])
        at = 40 + (6 if b[6] == 17 else 2)
        z = bytearray(b)
        z[at:at + 2] = b"\0\0"
        rows.append((c["name"], bytes(z), b))
    return rows
