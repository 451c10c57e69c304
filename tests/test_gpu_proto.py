"""GPU: the batched IPv4 / UDP / ICMP / TCP-EncodePartial callers
(netstack_amd/proto.py) against the oracle composed exactly as the reference
sequences do (ipv4.go:251-277, udp/endpoint.go:809-815, icmpv4.go:155-169,
icmpv6.go:202-221, tcp.go:295-314)."""
import struct

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

SRC = bytes([10, 0, 0, 1])
DST = bytes([10, 0, 0, 2])
SRC6 = bytes.fromhex("fe800000000000000000000000000001")
DST6 = bytes.fromhex("ff020000000000000000000000000001")


def _vv(rng, size):
    from netstack_amd.buffer import NewVectorisedView, View

    data = rng.integers(0, 256, size, dtype=np.uint8).tobytes()
    views, pos = [], 0
    while pos < size:
        s = int(rng.integers(0, 700))   # includes empty and odd-length views
        views.append(View(bytearray(data[pos:pos + s])))
        pos += s
    return NewVectorisedView(size, views), [bytes(v) for v in views]


def test_ipv4_header_checksums(engine):
    import oracle as O
    from netstack_amd import proto

    rng = np.random.default_rng(20)
    hdrs = []
    for i in range(500):
        ihl = 20 + 4 * int(rng.integers(0, 11))
        f = proto.IPv4Fields(ihl, int(rng.integers(0, 256)), int(rng.integers(0, 65536)), i,
                             int(rng.integers(0, 8)), 8 * int(rng.integers(0, 8192)),
                             int(rng.integers(0, 256)), int(rng.integers(0, 256)), 0,
                             rng.integers(0, 256, 4, dtype=np.uint8).tobytes(),
                             rng.integers(0, 256, 4, dtype=np.uint8).tobytes())
        h = proto.encode_ipv4(f)
        h[20:] = rng.integers(0, 256, ihl - 20, dtype=np.uint8).tobytes()  # options
        hdrs.append(h)
    want = [O.c_checksum(bytes(h), 0) for h in hdrs]
    assert proto.ipv4_calculate_checksums(hdrs) == want
    proto.add_ip_headers(hdrs)
    for h in hdrs:
        assert O.c_checksum(bytes(h), 0) == 0xFFFF     # a valid header sums to 0xffff


def test_ipv4_encode_partial(engine):
    import oracle as O
    from netstack_amd import proto

    rng = np.random.default_rng(21)
    hdrs, parts, tls, want = [], [], [], []
    for i in range(300):
        f = proto.IPv4Fields(20, 0, 0, i, 2, 0, 64, 17, 0, SRC, DST)
        h = proto.encode_ipv4(f)
        # partial = checksum of the header without total length and checksum
        p = O.c_checksum(bytes(h[:2]) + bytes(h[4:10]) + bytes(h[12:]), 0)
        tl = int(rng.integers(20, 65536))
        hdrs.append(h)
        parts.append(p)
        tls.append(tl)
        want.append((~O.c_checksum(struct.pack(">H", tl), p)) & 0xFFFF)
    proto.ipv4_encode_partial(hdrs, parts, tls)
    for h, tl, w in zip(hdrs, tls, want):
        assert struct.unpack_from(">HxxxxxxH", h, 2) == (tl, w)
        assert O.c_checksum(bytes(h), 0) == 0xFFFF


@pytest.mark.parametrize("src,dst", [(SRC, DST), (SRC6, DST6)])
def test_send_udp_batch(engine, src, dst):
    import oracle as O
    from netstack_amd import proto

    rng = np.random.default_rng(22)
    dgrams, views_list = [], []
    for i in range(200):
        vv, views = _vv(rng, int(rng.integers(0, 9000)))
        dgrams.append((vv, src, dst, 1000 + i, 53))
        views_list.append(views)
    hdrs = proto.send_udp_batch(dgrams)
    for (vv, s, d, sp, dp), views, h in zip(dgrams, views_list, hdrs):
        length = 8 + vv.Size()
        x = O.c_pseudo_header(17, s, d, length)
        for v in views:                                 # endpoint.go:811-813
            x = O.c_checksum(v, x)
        x = O.c_checksum(struct.pack(">HHHH", sp, dp, length & 0xFFFF, 0), x)
        assert bytes(h) == struct.pack(">HHHH", sp, dp, length & 0xFFFF, (~x) & 0xFFFF)
    off = proto.send_udp_batch(dgrams[:3], tx_checksum_offload=True)
    assert all(struct.unpack_from(">H", h, 6)[0] == 0 for h in off)


def test_icmpv4_checksums(engine):
    import oracle as O
    from netstack_amd import proto

    rng = np.random.default_rng(23)
    items, want = [], []
    for i in range(200):
        h = bytearray(rng.integers(0, 256, 8, dtype=np.uint8).tobytes())
        vv, views = _vv(rng, int(rng.integers(0, 3000)))
        items.append((h, vv))
        x = 0
        for v in views:
            x = O.c_checksum(v, x)
        hz = bytearray(h)
        hz[2:4] = b"\0\0"
        want.append((~O.c_checksum(bytes(hz), x)) & 0xFFFF)
    before = [bytes(h) for h, _ in items]
    assert proto.icmpv4_checksums(items) == want
    assert [bytes(h) for h, _ in items] == before     # h[2:4] restored (icmpv4.go:167)


def test_icmpv6_checksums(engine):
    import oracle as O
    from netstack_amd import proto

    rng = np.random.default_rng(24)
    items, want = [], []
    for i in range(200):
        hl = int(rng.choice([4, 8, 24]))
        h = bytearray(rng.integers(0, 256, hl, dtype=np.uint8).tobytes())
        vv, views = _vv(rng, int(rng.integers(0, 3000)))
        items.append((h, SRC6, DST6, vv))
        x = O.c_checksum(SRC6, 0)
        x = O.c_checksum(DST6, x)
        x = O.c_checksum(struct.pack(">I", hl + vv.Size()), x)
        x = O.c_checksum(bytes([0, 0, 0, 58]), x)
        for v in views:
            x = O.c_checksum(v, x)
        hz = bytearray(h)
        hz[2:4] = b"\0\0"
        want.append((~O.c_checksum(bytes(hz), x)) & 0xFFFF)
    assert proto.icmpv6_checksums(items) == want


def test_icmpv6_reference_validation_cases(engine):
    """icmp_test.go:367-899 (tests/icmpv6cases.py): the engine's ICMPv6Checksum
    equals the oracle's for the transmit split, the receive split of the
    message with the field set gives the same value (received), and no value
    is 0 (the unset field is Invalid)."""
    import icmpv6cases as C
    import oracle as O
    from netstack_amd import proto
    from netstack_amd.buffer import NewVectorisedView, View

    def vv(views):
        return NewVectorisedView(sum(map(len, views)), [View(bytearray(v)) for v in views])

    cs = C.cases()
    tx = proto.icmpv6_checksums([(bytearray(h), C.LLADDR1, C.LLADDR0, vv(v)) for _, h, v, _, _ in cs])
    want = [C.oracle_checksum(O, h, C.LLADDR1, C.LLADDR0, v) for _, h, v, _, _ in cs]
    assert tx == want
    assert all(c != 0 for c in tx)
    rx = proto.icmpv6_checksums([(bytearray(C.with_checksum(h, c)), C.LLADDR1, C.LLADDR0, vv(v))
                                 for (_, _, _, h, v), c in zip(cs, tx)])
    assert rx == tx


def test_tcp_encode_partial(engine):
    """tcp.go:295-314: the incremental update must equal a full recompute of
    the segment checksum when `partial` covers everything else."""
    import oracle as O
    from netstack_amd import proto, tcp

    rng = np.random.default_rng(25)
    hdrs, args, payloads = [], [], []
    for i in range(300):
        payload = rng.integers(0, 256, int(rng.integers(0, 2000)), dtype=np.uint8).tobytes()
        h = tcp.encode_tcp(tcp.TCPFields(1234, 80, 0, 0, 20, 0, 0))
        # partial checksum over pseudo-header (without length) + payload + the
        # header fields EncodePartial does not touch (tcp_test style)
        p = O.c_checksum(SRC + DST + bytes([0, 6]), 0)
        p = O.c_checksum(payload, p)
        p = O.c_checksum(bytes(h[0:4]) + bytes(h[12:13]) + b"\0" + bytes(h[18:20]), p)
        seq, ack = (int(v) for v in rng.integers(0, 2**32, 2, dtype=np.uint64))
        fl, wnd = int(rng.integers(0, 256)), int(rng.integers(0, 65536))
        hdrs.append(h)
        payloads.append(payload)
        args.append((p, 20 + len(payload), seq, ack, fl, wnd))
    proto.tcp_encode_partial(hdrs, *zip(*args))
    for h, payload, (p, ln, seq, ack, fl, wnd) in zip(hdrs, payloads, args):
        assert struct.unpack_from(">IIxBH", h, 4) == (seq, ack, fl, wnd)
        x = O.c_pseudo_header(6, SRC, DST, ln)
        x = O.c_checksum(payload, O.c_checksum(bytes(h), x))
        assert x == 0xFFFF
