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


def main():
    out = {"invalid_fragments": invalid_fragments(), "holes": holes(), "process": process(),
           "fragmentation": fragmentation(), "incorrect_checksum": incorrect_checksum()}
    with open(os.path.join(HERE, "rx_fixtures.json"), "w") as f:
        json.dump(out, f, indent=1)
        f.write("\n")


if __name__ == "__main__":
    main()
