"""The reference's ICMPv6 checksum validation cases (icmp_test.go:367-899,
restated in tests/icmpv6cases.py) on the C oracle: every message checksummed
by the transmit split validates under the receive split (icmp.go:79-82), and
the same message with a zero field does not.  tests/test_gpu_proto.py runs
the same cases through the engine."""
import icmpv6cases as C


def test_link_local_addresses():
    # header.LinkLocalAddr (ipv6.go:271-291): aa:bb:cc:dd:ee:ff => fe80::(aa^2)bb:ccff:fedd:eeff
    assert C.LLADDR0.hex() == "fe80000000000000" "000203fffe040506"
    assert C.LLADDR1.hex() == "fe80000000000000" "080b0cfffe0d0e0f"


def test_case_table_matches_the_reference_rows():
    cs = C.cases()
    assert len(cs) == 11 + 6 + 6
    sizes = {n: (len(tx), sum(map(len, v))) for n, tx, v, _, _ in cs}
    assert sizes["simple/NeighborAdvert"] == (32, 0)   # ICMPv6NeighborAdvertSize = 4 + 20 + 8
    assert sizes["simple/RouterAdvert"] == (16, 0)     # ICMPv6HeaderSize + NDPRAMinimumSize
    assert sizes["payload/DstUnreachable"] == (8 + 104, 0)
    assert sizes["views/EchoRequest"] == (8, 64)


def test_reference_cases_on_the_oracle():
    import oracle as O

    for label, tx_h, tx_v, rx_h, rx_v in C.cases():
        c = C.oracle_checksum(O, tx_h, C.LLADDR1, C.LLADDR0, tx_v)
        assert c != 0, label                           # the unset field is Invalid
        got = C.oracle_checksum(O, C.with_checksum(rx_h, c), C.LLADDR1, C.LLADDR0, rx_v)
        assert got == c, label                         # the set field is received
        # and the pure-Python restatement agrees
        x = O.py_pseudo_header(58, C.LLADDR1, C.LLADDR0, len(tx_h) + sum(map(len, tx_v)))
        for v in tx_v:
            x = O.py_checksum(v, x)
        hz = bytearray(tx_h)
        hz[2:4] = b"\0\0"
        assert (~O.py_checksum(bytes(hz), x)) & 0xFFFF == c, label
