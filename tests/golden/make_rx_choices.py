"""Generate tests/golden/rx_choices.json (run: python tests/golden/make_rx_choices.py).

Receive-path cases where the reference's behaviour is not defined by its
packet bytes alone, and this repo made a choice.  Each case
holds the Data views as the link delivers them, the Data size, the verdict
and sums that oracle/packets.py and ns_csum_packet_buffers must give, and
what the reference does.

ipv4_header_past_first_view — IsValid (header/ipv4.go:280-296) checks hlen
    against TotalLength and the packet size, but not against the first
    view; HandlePacket then takes `headerView[:h.HeaderLength()]`
    (network/ipv4/ipv4.go:348), which reslices past the view's length into
    its spare capacity, or panics beyond the capacity.  Which one happens
    depends on the backing array, not on the packet.  The engine does not
    guess: the packet is MALFORMED (no sums taken).  In the Go receive
    contract (go/link/fdbased/csum_rx_hip.go) only VALID/INVALID set
    PacketBuffer.RXChecksum, so such a packet stays RXChecksumUnknown and
    the stack handles it exactly as without the engine.  fdbased's first
    view is 128 B minus the link header (BufConfig, packet_dispatchers.go:30)
    and an IPv4 header is at most 60 B, so that link never delivers one.

The packets are built here from fixed bytes; the TCP checksum is written by
the oracle's transmit restatement (oracle/packets.py fill), test
infrastructure.  Nothing here is reference source.
"""
from __future__ import annotations

import json
import os
import struct
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(HERE, "..", "..", "oracle"))

import packets as P  # noqa: E402


def _ipv4_tcp(ihl_words: int, payload: bytes) -> bytes:
    hlen = 4 * ihl_words
    ip = bytearray(hlen)
    ip[0] = 0x40 | ihl_words
    struct.pack_into(">HHHBB", ip, 2, hlen + 20 + len(payload), 0x1234, 0x4000, 64, 6)
    ip[12:20] = bytes([10, 0, 0, 1, 10, 0, 0, 2])
    ip[20:hlen] = b"\x01" * (hlen - 20)  # NOP options
    tcp = bytearray(20)
    struct.pack_into(">HHIIBBH", tcp, 0, 40000, 443, 790, 1, 5 << 4, 0x18, 30000)
    hdr, _, _ = P.fill(bytes(ip + tcp), [payload], len(payload))
    return hdr + payload


def cases():
    payload = bytes((7 * i + 3) & 0xFF for i in range(333))
    out = []
    for name, ihl, first in [
        ("ipv4_header_past_first_view", 6, 20),      # 24-B header, 20-B first view
        ("ipv4_max_header_past_first_view", 15, 40),  # 60-B header, 40-B first view
        ("ipv4_header_ends_with_first_view", 6, 24),  # control: the header fits its view
        ("ipv4_header_and_more_in_first_view", 15, 128),  # control: BufConfig's first view
    ]:
        pkt = _ipv4_tcp(ihl, payload)
        views = [pkt[:first], pkt[first:first + 200], pkt[first + 200:]]
        v, net, tr = P.verify(b"", views, len(pkt))
        out.append({"name": name, "views": [x.hex() for x in views], "size": len(pkt),
                    "verdict": v, "ipv4_sum": net, "transport_sum": tr,
                    "reference": "ipv4.go:348 reslices headerView past its length (spare capacity) or panics"
                    if first < 4 * ihl else "IsValid passes; segment.parse verifies the checksum"})
    assert [c["verdict"] for c in out] == [P.MALFORMED, P.MALFORMED, P.VALID, P.VALID], out
    return out


if __name__ == "__main__":
    with open(os.path.join(HERE, "rx_choices.json"), "w") as f:
        json.dump({"ipv4_header_past_first_view": cases()}, f, indent=1)
        f.write("\n")
