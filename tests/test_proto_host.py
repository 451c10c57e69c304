"""CPU: header field encoding of the caller mirrors (no checksum arithmetic
happens on the host; these check only the byte layout Encode writes)."""
import struct

from netstack_amd import proto, tcp


def test_encode_ipv4_layout():
    # the classic worked example: 4500 0073 0000 4000 4011 xxxx c0a8 0001 c0a8 00c7
    f = proto.IPv4Fields(20, 0, 0x73, 0, 2, 0, 0x40, 17, 0, bytes([192, 168, 0, 1]), bytes([192, 168, 0, 199]))
    h = proto.encode_ipv4(f)
    assert bytes(h).hex() == "450000730000400040110000c0a80001c0a800c7"
    f = proto.IPv4Fields(24, 0xB8, 1500, 0xBEEF, 1, 8 * 100, 1, 6, 0x1234, bytes(4), bytes(4))
    h = proto.encode_ipv4(f)
    assert h[0] == 0x46 and h[1] == 0xB8
    assert struct.unpack_from(">HHHBBH", h, 2) == (1500, 0xBEEF, (1 << 13) | 100, 1, 6, 0x1234)


def test_encode_udp_and_tcp_layout():
    assert bytes(proto.encode_udp(53, 1234, 40)).hex() == "003504d200280000"
    h = tcp.encode_tcp(tcp.TCPFields(1, 2, 3, 4, 24, 0x12, 5), bytes([2, 4, 5, 0xB4]))
    assert bytes(h).hex() == "000100020000000300000004601200050000000002040" + "5b4"
