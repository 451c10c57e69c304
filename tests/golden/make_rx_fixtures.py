"""Generate tests/golden/rx_fixtures.json (run: python tests/golden/make_rx_fixtures.py).

Packet-level cases of the reference's own tests, kept as DATA (inputs and the
reference's expected outcomes), to pin the receive path's verdict semantics
(IsValid, HandlePacket's fragment checks, reassembly, checksum errors) beyond
the checksum arithmetic that kat.json pins:

invalid_fragments — network/ipv4/ipv4_test.go:360-455 TestInvalidFragments:
    the packets (bytes) of each case and the expected
    Stats.IP.MalformedPacketsReceived / MalformedFragmentsReceived.  The byte
    arrays are read out of the reference's test file at generation time.
holes             — network/fragmentation/reassembler_test.go:28-98
    TestUpdateHoles: fragments (first, last, more) -> the hole list.
process           — network/fragmentation/fragmentation_test.go:50-78
    TestFragmentationProcess: (id, first, last, more, pieces) -> (done,
    reassembled pieces).
fragmentation     — network/ipv4/ipv4_test.go:257-270 TestFragmentation: the
    table of (mtu, hdrLength, extraLength, payload view sizes,
    expectedFrags) shapes.
incorrect_checksum — transport/tcp/tcp_test.go:3232-3259
    TestReceivedIncorrectChecksumIncrement: the segment BuildSegment makes
    (testing/context/context.go:311-356: TestAddr -> StackAddr, IPv4 TTL 65,
    TCP TestPort -> the endpoint's port, ACK, seq 790, window 30000, payload
    {1, 2, 3}) with its first payload byte overwritten with 0x4; expected:
    ChecksumErrors + 1 (stack and endpoint).  The endpoint's port and the
    ack number are chosen by the test at run time; fixed values stand in.
ipv6_receive      — the IPv6 packets network/ipv6's tests inject and expect to
    pass the checksum: ipv6_test.go:40-67 testReceiveICMP (a 32-B
    NeighborAdvert) and :71-125 testReceiveUDP (an 8-B UDP, 5555 -> 80) as
    TestReceiveOnAllNodesMulticastAddr (:129-155) and
    TestReceiveOnSolicitedNodeAddr (:160-225) send them; ndp_test.go:75-184
    TestHopLimitValidation (each NDP type at its table size, lladdr0 ->
    lladdr1, hop limit 254 and 255) and :189-372 TestRouterAdvertValidation
    (its seven RAs to ff02::1, 15-B NDPPayloadTooSmall among them);
    stack/ndp_test.go:361-420 TestDADFail's NS from :: and NA.  Each
    row: the packet, the verdict the receive path owes it (VALID; UNCHECKED
    for UDP) and what the reference's test then expects — the drops these
    tests count (hop limit, code, source, RA size) all come after the
    checksum check (network/ipv6/icmp.go:79-102), so none of them changes
    the verdict.  The checksums are computed here as those tests compute
    them (ICMPv6Checksum / PseudoHeaderChecksum over the message with a zero
    checksum field).
receive_control   — network/ip_test.go:293-398 TestIPv4ReceiveControl and
    :534-650 TestIPv6ReceiveControl: an ICMP error (outer header, ICMP
    header with ident 0xdead / sequence 0xbeef, the inner header, 8 payload
    bytes i & 0xff) cut short by each case's trunc, and the case's
    expectedCount.  The verdict each row owes follows from the rules these
    packets meet first: the IP header against the packet (IsValid), the
    8-B ICMP minimum (ipv4/icmp.go:60, ipv6/icmp.go:68), then for ICMPv6
    the checksum (set over the untruncated message, so a cut one is
    INVALID) and for a non-echo ICMPv4 none (UNCHECKED).  Every row the
    reference counts (expectedCount 1) is VALID or UNCHECKED.

Nothing here is reference source: the file holds values only.
"""
from __future__ import annotations

import json
import os
import re

HERE = os.path.dirname(os.path.abspath(__file__))
REF = "/root/reference/tcpip/network/ipv4/ipv4_test.go"


def invalid_fragments():
    text = open(REF).read()
    body = text[text.index("func TestInvalidFragments"):]
    body = body[:body.index("for _, tc := range testCases")]
    cases = []
    # each case: {"name", [][]byte{ {...}, ... }, malformedIP, malformedFrag}
    for m in re.finditer(r'"([a-z0-9_]+)",\s*\[\]\[\]byte\{(.*?)\n\t\t\t\},\s*(\d+),\s*(\d+),', body, re.S):
        name, arrays, mip, mfr = m.group(1), m.group(2), int(m.group(3)), int(m.group(4))
        pkts = [bytes(int(x, 0) for x in a.split(",") if x.strip()).hex()
                for a in re.findall(r"\{([0-9a-fx,\s]+)\}", arrays)]
        cases.append({"name": name, "packets": pkts, "malformed_ip": mip, "malformed_fragments": mfr,
                      "source": "network/ipv4/ipv4_test.go:360-455"})
    assert len(cases) == 8, len(cases)
    return cases


def holes():
    M = 0xFFFF
    src = "network/fragmentation/reassembler_test.go:28-98"
    return [
        {"in": [], "want": [[0, M, False]], "source": src},
        {"in": [[0, 1, True]], "want": [[0, M, True], [2, M, False]], "source": src},
        {"in": [[1, 2, True]], "want": [[0, M, True], [0, 0, False], [3, M, False]], "source": src},
        {"in": [[1, 2, False]], "want": [[0, M, True], [0, 0, False]], "source": src},
        {"in": [[0, 1, False]], "want": [[0, M, True]], "source": src},
        {"in": [[0, 1, True], [2, 3, False]], "want": [[0, M, True], [2, M, True]], "source": src},
        {"in": [[0, 2, True], [2, 3, False]], "want": [[0, M, True], [3, M, True]], "source": src},
    ]


def process():
    src = "network/fragmentation/fragmentation_test.go:50-78"
    return [
        {"in": [[0, 0, 1, True, ["01"]], [0, 2, 3, False, ["23"]]],
         "out": [[False, []], [True, ["01", "23"]]], "source": src},
        {"in": [[0, 0, 1, True, ["01"]], [1, 0, 1, True, ["ab"]], [1, 2, 3, False, ["cd"]],
                [0, 2, 3, False, ["23"]]],
         "out": [[False, []], [False, []], [True, ["ab", "cd"]], [True, ["01", "23"]]], "source": src},
    ]


def fragmentation():
    src = "network/ipv4/ipv4_test.go:257-270"
    many = {"repeat": 7, "count": 1000}
    rows = [
        ("NoFragmentation", 2000, 0, 20, [1000], 1),
        ("NoFragmentationWithBigHeader", 2000, 16, 20, [1000], 1),
        ("Fragmented", 800, 0, 20, [1000], 2),
        ("FragmentedWithGsoNil", 800, 0, 20, [1000], 2),
        ("FragmentedWithManyViews", 300, 0, 20, many, 25),
        ("FragmentedWithManyViewsAndPrependableBytes", 300, 0, 20 + 55, many, 25),
        ("FragmentedWithBigHeader", 800, 20, 20, [1000], 2),
        ("FragmentedWithBigHeaderAndPrependableBytes", 800, 20, 20 + 66, [1000], 2),
        ("FragmentedWithMTUSmallerThanHeaderAndPrependableBytes", 300, 1000, 20 + 77, [500], 6),
    ]
    return [{"name": n, "mtu": mtu, "hdr_length": hl, "extra_length": el, "views": v, "expected_frags": k,
             "source": src} for (n, mtu, hl, el, v, k) in rows]


def incorrect_checksum():
    return {"src": "0a000002", "dst": "0a000001", "ttl": 65, "src_port": 4096, "dst_port": 1235,
            "flags": 0x10, "seq": 790, "ack": 0x12345679, "window": 30000, "payload": "010203",
            "corrupt_payload_byte": 0, "corrupt_value": 4, "checksum_errors": 1,
            "source": "transport/tcp/tcp_test.go:3232-3259, testing/context/context.go:311-356"}


def _sum16(b: bytes, acc: int = 0) -> int:
    if len(b) % 2:
        b += b"\0"
    for i in range(0, len(b), 2):
        acc += b[i] << 8 | b[i + 1]
    while acc > 0xFFFF:
        acc = (acc & 0xFFFF) + (acc >> 16)
    return acc


def _ipv6(src: bytes, dst: bytes, proto: int, hop: int, msg: bytearray, at: int) -> str:
    """msg's checksum field (offset at) set from the pseudo-header, then the
    40-B IPv6 header (IPv6Fields: PayloadLength, NextHeader, HopLimit)."""
    pseudo = _sum16(src + dst + len(msg).to_bytes(4, "big") + bytes([0, 0, 0, proto]))
    c = ~_sum16(bytes(msg), pseudo) & 0xFFFF
    msg[at:at + 2] = c.to_bytes(2, "big")
    h = bytes([0x60, 0, 0, 0]) + len(msg).to_bytes(2, "big") + bytes([proto, hop]) + src + dst
    return (h + bytes(msg)).hex()


def ipv6_receive():
    addr1 = b"\x0a" + bytes(14) + b"\x01"
    addr2 = b"\x0a" + bytes(14) + b"\x02"
    all_nodes = b"\xff\x02" + bytes(13) + b"\x01"
    snmc = b"\xff\x02" + bytes(9) + b"\x01\xff" + addr2[-3:]

    def lladdr(mac):  # header/ipv6.go:271-290 LinkLocalAddr
        return b"\xfe\x80" + bytes(6) + bytes([mac[0] ^ 2, mac[1], mac[2], 0xFF, 0xFE, mac[3], mac[4], mac[5]])

    ll0, ll1 = lladdr(b"\x02\x02\x03\x04\x05\x06"), lladdr(b"\x0a\x0b\x0c\x0d\x0e\x0f")
    rows = []
    for dname, dst in (("all_nodes", all_nodes), ("solicited_node", snmc)):
        na = bytearray(32)
        na[0] = 136
        rows.append({"name": f"receive_icmp_{dname}", "packet": _ipv6(addr1, dst, 58, 255, na, 2), "verdict": 1,
                     "reference": "ICMP.V6PacketsReceived.NeighborAdvert + 1",
                     "source": "network/ipv6/ipv6_test.go:40-67,129-225"})
        u = bytearray((5555).to_bytes(2, "big") + (80).to_bytes(2, "big") + (8).to_bytes(2, "big") + bytes(2))
        rows.append({"name": f"receive_udp_{dname}", "packet": _ipv6(addr1, dst, 17, 255, u, 6), "verdict": 2,
                     "reference": "UDP.PacketsReceived + 1", "source": "network/ipv6/ipv6_test.go:71-125,129-225"})
    for tname, typ, size in (("RouterSolicit", 133, 8), ("RouterAdvert", 134, 4 + 12), ("NeighborSolicit", 135, 24),
                             ("NeighborAdvert", 136, 32), ("RedirectMsg", 137, 8)):
        for hop in (254, 255):
            m = bytearray(size)
            m[0] = typ
            rows.append({"name": f"hop_limit_{tname}_{hop}", "packet": _ipv6(ll0, ll1, 58, hop, m, 2), "verdict": 1,
                         "reference": f"ICMP.V6PacketsReceived.{tname} + 1" if hop == 255
                         else "ICMP.V6PacketsReceived.Invalid + 1 (hop limit, after the checksum)",
                         "source": "network/ipv6/ndp_test.go:75-184"})
    ra = bytes(12)
    opts = bytes([2, 1]) + bytes(6) + bytes([255, 1]) + bytes(6) + bytes([3, 4]) + bytes(30)
    zero_len = bytes([2, 0]) + opts[2:]
    for name, src, hop, code, payload, ok in (("OK", ll0, 255, 0, ra, True), ("NonLinkLocalSourceAddr", addr1, 255, 0, ra, False),
                                              ("HopLimitNot255", ll0, 254, 0, ra, False), ("NonZeroCode", ll0, 255, 1, ra, False),
                                              ("NDPPayloadTooSmall", ll0, 255, 0, ra[:11], False),
                                              ("OKWithOptions", ll0, 255, 0, ra + opts, True),
                                              ("OptionWithZeroLength", ll0, 255, 0, ra + zero_len, False)):
        m = bytearray([134, code, 0, 0]) + payload
        rows.append({"name": f"router_advert_{name}", "packet": _ipv6(src, all_nodes, 58, hop, m, 2), "verdict": 1,
                     "reference": "ICMP.V6PacketsReceived.RouterAdvert + 1" if ok
                     else "ICMP.V6PacketsReceived.Invalid + 1 (after the checksum)",
                     "source": "network/ipv6/ndp_test.go:189-372"})
    # stack/ndp_test.go:361-420 TestDADFail: a DAD probe (NS from the
    # unspecified address to the target's solicited-node group) and an
    # NA with the S and O flags, both for addr1
    any6 = bytes(16)
    snmc1 = b"\xff\x02" + bytes(9) + b"\x01\xff" + addr1[-3:]
    ns = bytearray(24)
    ns[0], ns[8:24] = 135, addr1
    rows.append({"name": "dad_rx_solicit", "packet": _ipv6(any6, snmc1, 58, 255, ns, 2), "verdict": 1,
                 "reference": "ICMP.V6PacketsReceived.NeighborSolicit + 1 (DAD fails)",
                 "source": "stack/ndp_test.go:361-420"})
    na = bytearray(32)
    na[0], na[4], na[8:24] = 136, 0x60, addr1
    rows.append({"name": "dad_rx_advert", "packet": _ipv6(addr1, all_nodes, 58, 255, na, 2), "verdict": 1,
                 "reference": "ICMP.V6PacketsReceived.NeighborAdvert + 1 (DAD fails)",
                 "source": "stack/ndp_test.go:361-420"})
    assert len(rows) == 4 + 10 + 7 + 2
    return rows


def receive_control():
    rows = []
    src4, local4, remote4 = bytes([10, 0, 0, 0xbb]), bytes([10, 0, 0, 1]), bytes([10, 0, 0, 2])

    def ipv4(total, proto, frag, src, dst):  # IPv4Fields: IHL 20, TTL 20, no checksum
        return bytes([0x45, 0]) + total.to_bytes(2, "big") + bytes(2) + (frag >> 3).to_bytes(2, "big") + \
            bytes([20, proto, 0, 0]) + src + dst

    # (name, expectedCount, inner fragment offset, code, trunc, verdict)
    for name, count, fo, code, trunc, verdict in (
            ("FragmentationNeeded", 1, 0, 4, 0, 2), ("Truncated (10 bytes missing)", 0, 0, 4, 10, 2),
            ("Truncated (missing IPv4 header)", 0, 0, 4, 28, 2),
            ("Truncated (missing 'extra info')", 0, 0, 4, 32, 3),
            ("Truncated (missing ICMP header)", 0, 0, 4, 36, 3), ("Port unreachable", 1, 0, 3, 0, 2),
            ("Non-zero fragment offset", 0, 100, 3, 0, 2), ("Zero-length packet", 0, 0, 3, 56, 3)):
        view = bytearray(56)
        view[0:20] = ipv4(56 - trunc, 1, 0, src4, local4)
        view[20:28] = bytes([3, code, 0, 0, 0xde, 0xad, 0xbe, 0xef])
        view[28:48] = ipv4(100, 10, fo, local4, remote4)
        for i in range(48, 56):
            view[i] = i & 0xFF
        rows.append({"name": "ipv4/" + name, "packet": bytes(view[:56 - trunc]).hex(), "verdict": verdict,
                     "expected_count": count, "source": "network/ip_test.go:293-398"})

    local6 = b"\x0a" + bytes(14) + b"\x01"
    remote6 = b"\x0a" + bytes(14) + b"\x02"
    outer6 = b"\x0a" + bytes(14) + b"\xaa"

    def ipv6(pl, nh, src, dst):  # IPv6Fields: hop limit 20
        return bytes([0x60, 0, 0, 0]) + (pl & 0xFFFF).to_bytes(2, "big") + bytes([nh, 20]) + src + dst

    for name, count, fo, typ, code, trunc, verdict in (
            ("PacketTooBig", 1, None, 2, 0, 0, 1), ("Truncated (10 bytes missing)", 0, None, 2, 0, 10, 0),
            ("Truncated (missing IPv6 header)", 0, None, 2, 0, 48, 0),
            ("Truncated PacketTooBig (missing 'extra info')", 0, None, 2, 0, 52, 3),
            ("Truncated (missing ICMP header)", 0, None, 2, 0, 56, 3), ("Port unreachable", 1, None, 1, 4, 0, 1),
            ("Truncated DstUnreachable (missing 'extra info')", 0, None, 1, 4, 52, 3),
            ("Fragmented, zero offset", 1, 0, 1, 4, 0, 1), ("Non-zero fragment offset", 0, 100, 1, 4, 0, 1),
            ("Zero-length packet", 0, None, 1, 4, 96, 3)):
        data_at = 88 + (8 if fo is not None else 0)
        view = bytearray(data_at + 8)
        view[0:40] = ipv6(len(view) - 40 - trunc, 58, outer6, local6)
        view[40:48] = bytes([typ, code, 0, 0, 0xde, 0xad, 0xbe, 0xef])
        view[48:88] = ipv6(100, 10 if fo is None else 44, local6, remote6)
        if fo is not None:  # IPv6FragmentFields: NextHeader 10, M, Identification 0x12345678
            view[88:96] = bytes([10, 0]) + ((fo << 3) | 1).to_bytes(2, "big") + (0x12345678).to_bytes(4, "big")
        for i in range(data_at, len(view)):
            view[i] = i & 0xFF
        msg = bytes(view[40:])  # ICMPv6Checksum over the whole message, before the cut
        pseudo = _sum16(outer6 + local6 + len(msg).to_bytes(4, "big") + bytes([0, 0, 0, 58]))
        view[42:44] = (~_sum16(msg, pseudo) & 0xFFFF).to_bytes(2, "big")
        pkt = bytes(view[:len(view) - trunc])
        if verdict == 0:  # a cut message no longer matches its checksum
            m = pkt[40:]
            ps = _sum16(outer6 + local6 + len(m).to_bytes(4, "big") + bytes([0, 0, 0, 58]))
            assert _sum16(m, ps) != 0xFFFF, name
        rows.append({"name": "ipv6/" + name, "packet": pkt.hex(), "verdict": verdict, "expected_count": count,
                     "source": "network/ip_test.go:534-650"})
    assert all(r["verdict"] in (1, 2) for r in rows if r["expected_count"])
    return rows


def main():
    out = {"invalid_fragments": invalid_fragments(), "holes": holes(), "process": process(),
           "fragmentation": fragmentation(), "incorrect_checksum": incorrect_checksum(),
           "ipv6_receive": ipv6_receive(), "receive_control": receive_control()}
    with open(os.path.join(HERE, "rx_fixtures.json"), "w") as f:
        json.dump(out, f, indent=1)
        f.write("\n")


if __name__ == "__main__":
    main()
