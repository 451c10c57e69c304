"""GPU: the batched TCP callers (netstack_amd/tcp.py) against the oracle
composed exactly as the reference does (connect.go:634-702, segment.go:166-181),
plus the reference's protocol-level assertions (tcp_test.go testBrokenUpWrite
and TestReceivedIncorrectChecksumIncrement)."""
import struct

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

SRC = bytes([10, 0, 0, 1])
DST = bytes([10, 0, 0, 2])
SRC6 = bytes.fromhex("20010db8000000000000000000000001")
DST6 = bytes.fromhex("20010db8000000000000000000000002")


def _views(rng, data: bytes, shapes):
    from netstack_amd.buffer import NewVectorisedView, View

    out, pos = [], 0
    for s in shapes:
        if pos >= len(data):
            break
        out.append(View(bytearray(data[pos:pos + s])))
        pos += s
    if pos < len(data):
        out.append(View(bytearray(data[pos:])))
    return NewVectorisedView(len(data), out)


def _oracle_tx(views, src, dst, hdr: bytes, off, size):
    import oracle as O

    h = bytearray(hdr)
    h[16:18] = b"\0\0"
    x = O.c_pseudo_header(6, src, dst, len(h) + size)
    x = O.c_checksum_vv_with_offset(views, x, off, size)
    return (~O.c_checksum(bytes(h), x)) & 0xFFFF


@pytest.mark.parametrize("src,dst", [(SRC, DST), (SRC6, DST6)])
def test_send_tcp_batch_matches_reference_sequence(engine, src, dst):
    from netstack_amd import tcp

    rng = np.random.default_rng(10)
    for trial in range(8):
        size = int(rng.integers(0, 65536))
        data = rng.integers(0, 256, size, dtype=np.uint8).tobytes()
        shapes = [int(x) for x in rng.integers(1, 9000, 20)]
        vv = _views(rng, data, shapes)
        mss = int(rng.choice([536, 1448, 1460, 8948, 1]))  if trial else 1460
        opts = b"" if trial % 2 else bytes([1, 1, 8, 10]) + bytes(8)  # NOP NOP TS
        descs = tcp.send_tcp_batch(vv, mss, src, dst, 1234, 80, 0x18, 1000 + trial, 7777, 65535 * 4, opts)
        assert len(descs) == (size + mss - 1) // mss
        views = [bytes(v) for v in vv.Views()]
        for d in descs:
            want = _oracle_tx(views, src, dst, bytes(d.Hdr), d.Off, d.Size)
            assert struct.unpack_from(">H", d.Hdr, 16)[0] == want


def test_broken_up_write_segments_verify(engine):
    """tcp_test.go:2210-2270 testBrokenUpWrite: data[i] = byte(i), split into
    MSS-sized segments; every segment must verify at the receiver."""
    from netstack_amd import tcp
    from netstack_amd.buffer import NewVectorisedView, View

    max_payload = 100
    data = bytes(i & 0xFF for i in range(10 * max_payload))
    vv = NewVectorisedView(len(data), [View(bytearray(data))])
    descs = tcp.send_tcp_batch(vv, max_payload, SRC, DST, 1234, 80, 0x10, 789, 790, 30000)
    assert len(descs) == 10
    segs = []
    for d in descs:
        seg = bytes(d.Hdr) + data[d.Off:d.Off + d.Size]
        segs.append((SRC, DST, NewVectorisedView(len(seg), [View(bytearray(seg))])))
    assert tcp.verify_tcp_segments(segs) == [True] * 10


def test_verify_rx_batch_bufconfig_views_and_corruption(engine):
    """segment.parse over recvmmsg-shaped views (packet_dispatchers.go:30
    BufConfig 128,256,256,...), with one corrupted payload byte per odd
    segment (tcp_test.go:3232-3259 TestReceivedIncorrectChecksumIncrement)."""
    import oracle as O
    from netstack_amd import tcp
    from netstack_amd.buffer import NewVectorisedView, View

    rng = np.random.default_rng(11)
    segs, want = [], []
    for i in range(300):
        size = int(rng.integers(0, 9000))
        payload = bytearray(rng.integers(0, 256, size, dtype=np.uint8).tobytes())
        opts = bytes(4 * int(rng.integers(0, 11)))
        h = tcp.encode_tcp(tcp.TCPFields(1000 + i, 80, i, 5, 20 + len(opts), 0x10, 4096), opts)
        x = O.c_checksum(bytes(payload), O.c_checksum(bytes(h), O.c_pseudo_header(6, SRC, DST, len(h) + size)))
        struct.pack_into(">H", h, 16, (~x) & 0xFFFF)
        if i % 2 and size:
            payload[int(rng.integers(0, size))] ^= 0x5A
        seg = bytes(h) + bytes(payload)
        # BufConfig-shaped views; the TCP header sits inside the first 128 B
        shapes = [128, 256, 256, 512, 1024, 2048, 4096, 8192]
        views, pos = [], 0
        for s in shapes:
            if pos >= len(seg):
                break
            views.append(View(bytearray(seg[pos:pos + s])))
            pos += s
        vv = NewVectorisedView(len(seg), views)
        segs.append((SRC, DST, vv))
        # oracle, exactly as segment.go:176-180
        off = (seg[12] >> 4) * 4
        xs = O.c_pseudo_header(6, SRC, DST, len(seg))
        xs = O.c_checksum(seg[:off], xs)
        xs = O.c_checksum_vv_with_offset([bytes(v) for v in views], xs, off, len(seg) - off)
        want.append(xs == 0xFFFF)
    got = tcp.verify_tcp_segments(segs)
    assert got == want
    assert want.count(False) > 100  # the corrupted half fails


def test_gso_partial_and_offload_paths(engine):
    """connect.go:655-663: with GSO NeedsCsum only the pseudo-header sum is
    written; with TX checksum offload nothing is computed."""
    import oracle as O
    from netstack_amd import tcp
    from netstack_amd.buffer import NewVectorisedView, View

    data = bytes(range(256)) * 20
    vv = NewVectorisedView(len(data), [View(bytearray(data))])
    d = tcp.send_tcp_batch(vv, 1000, SRC, DST, 1, 2, 0x10, 0, 0, 100, gso_needs_csum=True)
    for x in d:
        assert struct.unpack_from(">H", x.Hdr, 16)[0] == O.c_pseudo_header(6, SRC, DST, 20 + x.Size)
    d = tcp.send_tcp_batch(vv, 1000, SRC, DST, 1, 2, 0x10, 0, 0, 100, tx_checksum_offload=True)
    assert all(struct.unpack_from(">H", x.Hdr, 16)[0] == 0 for x in d)


def test_chains_api_semantics(engine):
    """ns_csum_chains: restart vs continue pieces against the Go composition."""
    import oracle as O

    rng = np.random.default_rng(12)
    chains, want = [], []
    for _ in range(200):
        init = int(rng.integers(0, 65536))
        pieces = []
        x, odd = init, False
        k = int(rng.integers(1, 8))
        for j in range(k):
            b = rng.integers(0, 256, int(rng.integers(0, 300)), dtype=np.uint8).tobytes()
            restart = bool(rng.integers(0, 2))
            pieces.append((b, restart))
            if restart:
                x, odd = O.py_calculate_checksum(b, False, x)
            elif b:
                x, odd = O.py_calculate_checksum(b, odd, x)
        chains.append([("init", init)] + pieces)
        want.append(x)
    assert engine.chains(chains).tolist() == want


def test_send_tcp_batch_fused_ipv4_headers(engine):
    """WritePackets -> addIPHeader (network/ipv4/ipv4.go:217-238, 271-285)
    fused into the TX pass: the IPv4 header checksums verify (ipv4_test.go:
    140-142 style, header sums to 0xffff), ids advance only for packets > 68 B,
    and the TCP part equals the unfused result."""
    import oracle as O
    from netstack_amd import tcp
    from netstack_amd.buffer import NewVectorisedView, View

    data = bytes(np.random.default_rng(13).integers(0, 256, 20000, dtype=np.uint8))
    vv = NewVectorisedView(len(data), [View(bytearray(data[:7000])), View(bytearray(data[7000:]))])
    plain = tcp.send_tcp_batch(vv, 1448, SRC, DST, 5, 6, 0x18, 9, 10, 500)
    p = tcp.NetworkHeaderParams(TTL=63, TOS=0x10, ID=41)
    fused = tcp.send_tcp_batch(vv, 1448, SRC, DST, 5, 6, 0x18, 9, 10, 500, ipv4=p)
    assert p.ID == 41 + len(fused)
    for k, (a, b) in enumerate(zip(plain, fused)):
        ip = bytes(b.Hdr[:20])
        assert b.Hdr[20:] == a.Hdr and (b.Off, b.Size) == (a.Off, a.Size)
        assert O.c_checksum(ip, 0) == 0xFFFF
        assert struct.unpack_from(">HH", ip, 2) == (20 + len(a.Hdr) + a.Size, 42 + k)
        assert ip[8] == 63 and ip[1] == 0x10 and ip[9] == 6 and ip[12:16] == SRC and ip[16:20] == DST
    # a bare ACK (68 B or less) takes no id
    p2 = tcp.NetworkHeaderParams(ID=7)
    one = tcp.send_tcp_batch(NewVectorisedView(1, [View(bytearray(b"x"))]), 1448, SRC, DST, 1, 2, 0x10, 0, 0, 1,
                             ipv4=p2)
    assert p2.ID == 7 and struct.unpack_from(">H", one[0].Hdr, 4)[0] == 0
    assert O.c_checksum(bytes(one[0].Hdr[:20]), 0) == 0xFFFF
