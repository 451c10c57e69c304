"""CPU: the oracle (both restatements) against the pinned known answers and the
golden vectors, plus the invariants the reference's tests rely on."""
import numpy as np
import pytest

from make_golden import materialize


def test_reference_kats_vv(kat, oracle_mod):
    O = oracle_mod
    for c in kat["vv_with_offset"]:
        views = [bytes.fromhex(v) for v in c["views"]]
        # checksum_test.go:98 — through ChecksumVVWithOffset
        assert O.py_checksum_vv_with_offset(views, c["initial"], c["off"], c["size"]) == c["want"], c["name"]
        assert O.c_checksum_vv_with_offset(views, c["initial"], c["off"], c["size"]) == c["want"], c["name"]
        # checksum_test.go:101-105 — through Checksum on the flattened view
        flat = b"".join(views)[c["off"]:][: c["size"]]
        assert O.py_checksum(flat, c["initial"]) == c["want"], c["name"]
        assert O.c_checksum(flat, c["initial"]) == c["want"], c["name"]


def test_public_kats(kat, oracle_mod):
    for c in kat["checksum"]:
        buf = bytes.fromhex(c["buf"])
        assert oracle_mod.py_checksum(buf, c["initial"]) == c["want"], c["name"]
        assert oracle_mod.c_checksum(buf, c["initial"]) == c["want"], c["name"]


def test_c_matches_python_on_vectors(vectors, oracle_mod):
    O = oracle_mod
    for c in vectors["checksum"]:
        assert O.c_checksum(materialize(c["buf"]), c["initial"]) == c["want"], c["name"]
    for c in vectors["vv_with_offset"]:
        views = [materialize(v) for v in c["views"]]
        assert O.c_checksum_vv_with_offset(views, c["initial"], c["off"], c["size"]) == c["want"], c["name"]
    for c in vectors["views_restart"]:
        views = [materialize(v) for v in c["views"]]
        assert O.c_views_restart(views, c["initial"]) == c["want"], c["name"]
    for c in vectors["pseudo_header"]:
        got = O.c_pseudo_header(c["protocol"], bytes.fromhex(c["src"]), bytes.fromhex(c["dst"]), c["total_len"])
        assert got == c["want"], c["name"]
    for c in vectors["batch"]:
        arena = np.frombuffer(materialize(c["arena"]), dtype=np.uint8)
        d = np.array([tuple(x) for x in c["desc"]], dtype=O.DESC_DTYPE)
        got, bad = O.c_batch(arena, d, c["chained"])
        assert bad == 0
        assert got.tolist() == c["want"], c["name"]


def test_wrap_quirk(oracle_mod):
    # Go's un-folded uint32 wraps past 128 KiB.
    buf = b"\xff" * 200000
    assert oracle_mod.py_checksum(buf) == 0xFFFE
    assert oracle_mod.c_checksum(buf) == 0xFFFE
    # RFC 1071 (exact one's complement) would give 0xFFFF here.
    assert oracle_mod.c_checksum(b"\xff" * 131072, 0xFFFF) == 0xFFFF


def test_zero_representation(oracle_mod):
    O = oracle_mod
    assert O.c_checksum(bytes(1500), 0) == 0
    assert O.c_checksum(bytes(1500), 0xFFFF) == 0xFFFF
    assert O.c_checksum(bytes.fromhex("fffe0001"), 0) == 0xFFFF


def test_vv_equals_flattened_property(oracle_mod):
    """checksum_test.go:98-106 as a property: VV == Checksum(flattened) while no
    single view wraps."""
    O = oracle_mod
    rng = np.random.default_rng(3)
    for _ in range(200):
        views = [rng.integers(0, 256, int(rng.integers(0, 50)), dtype=np.uint8).tobytes()
                 for _ in range(int(rng.integers(1, 8)))]
        tot = sum(map(len, views))
        off = int(rng.integers(0, tot + 1))
        size = int(rng.integers(0, tot - off + 1))
        init = int(rng.integers(0, 65536))
        flat = b"".join(views)[off:off + size]
        assert O.c_checksum_vv_with_offset(views, init, off, size) == O.c_checksum(flat, init)


def test_tcp_segment_verify_and_corrupt(oracle_mod):
    """tcp_test.go:2214-2245 (data[i]=byte(i) segments verify) and
    tcp_test.go:3246-3254 (one corrupted payload byte must fail)."""
    O = oracle_mod
    src, dst = bytes([10, 0, 0, 1]), bytes([10, 0, 0, 2])
    payload = bytes(i & 0xFF for i in range(1000))
    hdr = bytearray(20)
    hdr[0:2], hdr[2:4], hdr[12] = (1234).to_bytes(2, "big"), (80).to_bytes(2, "big"), 5 << 4
    length = len(hdr) + len(payload)
    x = O.c_pseudo_header(6, src, dst, length)
    x = O.c_checksum(payload, x)
    x = O.c_checksum(bytes(hdr), x)
    hdr[16:18] = ((~x) & 0xFFFF).to_bytes(2, "big")  # tcp.SetChecksum(^...)
    # receiver (segment.go:174-180): pseudo + header + payload == 0xffff
    r = O.c_checksum(payload, O.c_checksum(bytes(hdr), O.c_pseudo_header(6, src, dst, length)))
    assert r == 0xFFFF
    bad = bytearray(payload)
    bad[0] = 0x4
    r = O.c_checksum(bytes(bad), O.c_checksum(bytes(hdr), O.c_pseudo_header(6, src, dst, length)))
    assert r != 0xFFFF


def test_negative_bounds_raise(oracle_mod):
    with pytest.raises(ValueError):
        oracle_mod.py_checksum_vv_with_offset([b"ab"], 0, 0, -1)
    with pytest.raises(ValueError):
        oracle_mod.c_checksum_vv_with_offset([b"ab"], 0, -1, 1)


def test_batch_mt_matches(oracle_mod):
    from netstack_amd import workloads as W

    b = W.config(4, n=4000)
    arena = b.arena_host()
    want, bad = oracle_mod.c_batch(arena, b.desc)
    assert bad == 0
    got = oracle_mod.c_batch_mt(arena, b.desc, 4)
    assert (got == want).all()


@pytest.mark.parametrize("fused", [True, False])
def test_rx_batch_generator_valid_packets(fused):
    """workloads.rx_batch writes valid IPv4 and TCP checksums (checked by the
    oracle composed as segment.parse and the IPv4 header check do) and breaks
    exactly the packets it says it corrupts; the fused table (2 independent
    descriptors per packet) gives exactly the chained table's results."""
    import torch  # noqa: F401  (generator runs on the CPU device here)

    import oracle as O
    from netstack_amd import workloads as W

    k = W.per_packet(fused)
    arena, d, bad = W.rx_batch(700, 3, "cpu", corrupt_every=11, fused=fused)
    out, nbad = O.c_batch(arena.numpy(), d, chained=not fused)
    assert nbad == 0
    assert (out[0::k] == 0xFFFF).all()
    assert np.array_equal(np.flatnonzero(out[k - 1::k] != 0xFFFF), bad)
    # the same TCP sums from the pure-Python chain of segment.parse (:176-180)
    a = arena.numpy()
    for i in (0, 1, 11, 699):
        b = 1504 * i
        xsum = O.py_pseudo_header(6, bytes(a[b + 12:b + 16]), bytes(a[b + 16:b + 20]), 1480)
        xsum = O.py_checksum(bytes(a[b + 20:b + 40]), xsum)
        xsum = O.py_checksum(bytes(a[b + 40:b + 1500]), xsum)
        assert xsum == out[k * i + k - 1]
    other, _ = O.c_batch(a, W._tcp_desc(700, not fused), chained=fused)
    kk = W.per_packet(not fused)
    assert np.array_equal(other[0::kk], out[0::k]) and np.array_equal(other[kk - 1::kk], out[k - 1::k])


@pytest.mark.parametrize("fused", [True, False])
def test_tx_stores_reproduce_rx_packets(fused):
    """oracle.apply_stores over tx_batch (zeroed checksum fields, the store
    flags of ns_csum_batch_dev_store) yields exactly rx_batch's packets, whose
    checksums torch integer ops wrote independently; the IPv4 store matches
    Go's ip.SetChecksum(^ip.CalculateChecksum()) (ipv4.go:236) restated in
    pure Python."""
    import oracle as O
    from netstack_amd import workloads as W

    tx, d = W.tx_batch(300, 9, "cpu", fused=fused)
    rx, _, _ = W.rx_batch(300, 9, "cpu")
    before = tx.numpy()
    res, nbad = O.c_batch(before, d, chained=not fused)
    assert nbad == 0
    after, dropped = O.apply_stores(before, d, res)
    assert dropped == 0 and np.array_equal(after, rx.numpy())
    for i in (0, 299):
        b = W.RX_STRIDE * i
        x = ~O.py_checksum(bytes(before[b:b + 20]), 0) & 0xFFFF
        assert after[b + 10] == x >> 8 and after[b + 11] == x & 0xFF


def test_apply_stores_raw_odd_and_dropped():
    """STORE_RAW writes r itself, offsets may be odd, and a store past the
    arena end is dropped and counted."""
    import oracle as O

    a = np.zeros(10, dtype=np.uint8)
    d = np.zeros(3, dtype=O.DESC_DTYPE)
    d["flags"] = [O.STORE | (3 << 4), O.STORE | O.STORE_RAW | (6 << 4), O.STORE | (9 << 4)]
    out, dropped = O.apply_stores(a, d, np.array([0x1234, 0xABCD, 1], dtype=np.uint16))
    assert dropped == 1
    assert list(out) == [0, 0, 0, 0xED, 0xCB, 0, 0xAB, 0xCD, 0, 0]


def _fold1(v: int) -> int:
    s = (v & 0xFFFF) + (v >> 16)
    return (s + (s >> 16)) & 0xFFFF


def test_run_fold_scan_algebra():
    """The algebra fold_scan relies on, checked in plain
    Python: with x <= 0xFFFF and a continuation partial p <= 0xFFFF0000,
    Go's chaining x' = fold1(x + p) (checksum.go:89 and :44-45) equals the
    state map (r, z) -> (r + p mod 65535, z and p == 0) read back as
    z ? 0 : (r or 0xFFFF); and that map composes associatively, so a
    segmented scan in any grouping gives Go's sequential results.  Edge
    values: 0, 0xFFFF, multiples of 65535, partials near the wrap bound."""
    rng = np.random.default_rng(17)
    edge = [0, 1, 0xFFFE, 0xFFFF, 0x10000, 65535 * 3, 65535 * 65537, 0xFFFF0000, 0xFFFEFFFF]

    def elem(p, head):
        if head:
            return ((0 if p == 0xFFFF else p), p == 0, True)
        return (p % 65535, p == 0, False)

    def comb(a, b):
        if b[2]:
            return b
        return ((a[0] + b[0]) % 65535, a[1] and b[1], a[2])

    def value(st):
        return 0 if st[1] else (st[0] if st[0] else 0xFFFF)

    for trial in range(300):
        n = int(rng.integers(1, 60))
        heads = rng.random(n) < 0.2
        heads[0] = True
        parts = []
        for k in range(n):
            if heads[k]:
                parts.append(int(rng.choice([0, 0xFFFF, int(rng.integers(0, 0x10000))])))
            else:
                parts.append(int(rng.choice(edge)) if rng.random() < 0.5 else int(rng.integers(0, 0xFFFF0001)))
        # Go's sequential fold
        want, x = [], 0
        for k in range(n):
            x = parts[k] if heads[k] else _fold1(x + parts[k])
            want.append(x)
        # the scan, grouped at random split points (associativity)
        es = [elem(parts[k], heads[k]) for k in range(n)]
        cuts = sorted(set(rng.integers(0, n + 1, 3).tolist()) | {0, n})
        got, carry = [], (0, True, False)
        for a, b in zip(cuts[:-1], cuts[1:]):
            agg = (0, True, False)
            for e in es[a:b]:
                agg = comb(agg, e)
            st = carry
            for e in es[a:b]:
                st = comb(st, e)
                got.append(value(st))
            carry = comb(carry, agg)
        assert got == want, (trial, parts, heads.tolist())


def test_packet_oracle_fill_then_verify(oracle_mod):
    """oracle/packets.py: what the transmit restatement fills, the receive
    restatement accepts (TCP over IPv4/IPv6, ICMPv4 echo), for payloads cut
    into views; one flipped byte is rejected; the IPv4 header then sums to
    0xffff (checker.go:51-53)."""
    import struct

    import packets as P

    rng = np.random.default_rng(8)
    for v6 in (False, True):
        for plen in (0, 1, 2, 1460, 3001):
            payload = bytes(rng.integers(0, 256, plen, dtype=np.uint8))
            tcp = bytearray(20)
            struct.pack_into(">HHIIBBH", tcp, 0, 1, 2, 3, 4, 0x50, 0x18, 5)
            if v6:
                ip = bytearray(40)
                ip[0] = 0x60
                struct.pack_into(">HBB", ip, 4, 20 + plen, 6, 64)
                ip[8:40] = bytes(rng.integers(0, 256, 32, dtype=np.uint8))
            else:
                ip = bytearray(20)
                struct.pack_into(">BBHHHBBH", ip, 0, 0x45, 0, 40 + plen, 7, 0, 64, 6, 0)
                ip[12:20] = bytes(rng.integers(0, 256, 8, dtype=np.uint8))
            cut = plen // 3
            hdr, net, tr = P.fill(bytes(ip + tcp), [payload[:cut], payload[cut:]], plen)
            wire = hdr + payload
            v, n2, t2 = P.verify(b"", [wire[:100], wire[100:]], len(wire))
            assert v == P.VALID and t2 == 0xFFFF
            if not v6:
                assert n2 == 0xFFFF
            if plen:
                bad = bytearray(wire)
                bad[-1] ^= 0x10
                assert P.verify(b"", [bytes(bad)], len(bad))[0] == P.INVALID
    icmp = bytearray(8)
    icmp[0] = 8
    ip = bytearray(20)
    struct.pack_into(">BBHHHBBH", ip, 0, 0x45, 0, 20 + 8 + 5, 7, 0, 64, 1, 0)
    hdr, _, _ = P.fill(bytes(ip + icmp), [b"hello"], 5)
    assert P.verify(b"", [hdr + b"hello"], len(hdr) + 5)[0] == P.VALID


def test_paired_oracle_is_go_chaining_on_runs_of_two(oracle_mod):
    """oracle.c_batch_paired (NS_BATCH_PAIRED): each odd-indexed CONT
    descriptor takes the previous descriptor's result as its initial —
    checked against the pure-Python restatement of checksum.go run descriptor
    by descriptor — and an even-indexed CONT bit changes nothing."""
    import oracle as O

    rng = np.random.default_rng(4242)
    n = 301
    arena = rng.integers(0, 256, 20000, dtype=np.uint8)
    d = np.zeros(n, dtype=O.DESC_DTYPE)
    d["off"] = rng.integers(0, 19000, n)
    d["len"] = rng.integers(0, 900, n)
    d["initial"] = rng.integers(0, 65536, n)
    d["flags"] = rng.integers(0, 4, n)  # ODD and CONT anywhere
    got, bad = O.c_batch_paired(arena, d)
    assert bad == 0
    want, prev = [], 0
    for i in range(n):
        o, ln, f = int(d["off"][i]), int(d["len"][i]), int(d["flags"][i])
        init = prev if (i % 2 == 1 and f & O.CONT) else int(d["initial"][i])
        s, _ = O.py_calculate_checksum(bytes(arena[o:o + ln]), bool(f & O.ODD), init)
        want.append(s)
        prev = s
    assert got.tolist() == want


def test_tx_split_layout_is_the_wire_segments_checksummed(oracle_mod):
    """workloads.tx_split_*: the sendTCPBatch layout (54-B header slots, a
    payload view).  The oracle's chained and paired fills equal the
    independently computed arena, and the filled segments verify."""
    import oracle as O
    from netstack_amd import workloads as W

    n = 1000
    arena, _ = W.tx_split_batch(n, 5, "cpu")
    exp = W.tx_split_expected(n, 5, "cpu", chunk=300).numpy()
    a = arena.numpy()
    for paired in (False, True):
        d = W.tx_split_desc(n, True, paired)
        want, bad = O.c_batch_paired(a, d) if paired else O.c_batch(a, d, chained=True)
        st, dropped = O.apply_stores(a, d, want)
        assert bad == 0 and dropped == 0 and np.array_equal(st, exp)
        vd = W.tx_split_desc(n, False, paired)
        res, _ = O.c_batch_paired(exp, vd) if paired else O.c_batch(exp, vd, chained=True)
        ip, tcp = W.tx_split_order(n, paired)
        assert (res[ip] == 0xFFFF).all() and (res[tcp] == 0xFFFF).all()
    with pytest.raises(ValueError):
        W.tx_split_desc(3, True, paired=True)


def test_send_tcp_batch_oracle_matches_the_table_fill(oracle_mod):
    """oracle.c_send_tcp_batch (sendTCPBatch's checksum steps restated in C,
    the checker of ns_csum_tcp_tx) over the bench's sendTCPBatch-layout arena
    equals the independently computed fill (workloads.tx_split_expected) and
    the descriptor-table fill; its sums are the un-complemented fields."""
    import oracle as O
    from netstack_amd import workloads as W

    n = 700
    arena, _ = W.tx_split_batch(n, 9, "cpu")
    a = arena.numpy()
    g = W.tx_struct_geometry(n)
    got, sums = O.c_send_tcp_batch(a, g["hdr_off"], g["pay_off"], g["size"], g["mss"], g["slot"], g["ip_at"],
                                   g["ip_len"], g["tcp_at"], g["tcp_len"], g["src"], g["dst"])
    assert np.array_equal(got, W.tx_split_expected(n, 9, "cpu", chunk=256).numpy())
    d = W.tx_split_desc(n, True, paired=True)
    res, _ = O.c_batch_paired(a, d)
    ip, tcp = W.tx_split_order(n, True)
    assert np.array_equal(sums[0::2], res[ip]) and np.array_equal(sums[1::2], res[tcp])


def test_send_tcp_batch_oracle_against_python_restatement(oracle_mod):
    """The C restatement against the pure-Python functions of checksum.go,
    segment by segment as connect.go:679-692 cuts them: odd MSS, odd slot
    size and offsets, a short last segment, the three TCP modes."""
    import oracle as O

    rng = np.random.default_rng(77)
    size, mss, slot, hdr_off, pay_off = 97 * 13 + 5, 97, 61, 3, 3 + 14 * 61 + 9
    n = -(-size // mss)
    a = rng.integers(0, 256, pay_off + size + 11, dtype=np.uint8)
    src, dst = bytes(rng.integers(0, 256, 16, dtype=np.uint8)), bytes(rng.integers(0, 256, 16, dtype=np.uint8))
    for mode in ("full", "partial", "none"):
        got, sums = O.c_send_tcp_batch(a, hdr_off, pay_off, size, mss, slot, 7, 24, 31, 28, src, dst, 6, mode)
        want = a.copy()
        left, off = size, 0
        for i in range(n):
            ps = min(mss, left)
            left -= ps
            s = hdr_off + i * slot
            tcp = bytearray(want[s + 31:s + 59])
            tcp[16:18] = b"\0\0"
            if mode != "none":
                x = O.py_pseudo_header(6, src, dst, (28 + ps) & 0xFFFF)
                if mode == "partial":
                    tcp[16:18] = x.to_bytes(2, "big")
                else:
                    x = O.py_checksum_vv_with_offset([bytes(a[pay_off:pay_off + size])], x, off, ps)
                    x = O.py_checksum(bytes(tcp), x)
                    tcp[16:18] = (~x & 0xFFFF).to_bytes(2, "big")
                want[s + 31:s + 59] = np.frombuffer(bytes(tcp), np.uint8)
                assert sums[2 * i + 1] == x
            ip = bytearray(want[s + 7:s + 31])
            ip[10:12] = b"\0\0"
            v = O.py_checksum(bytes(ip), 0)
            ip[10:12] = (~v & 0xFFFF).to_bytes(2, "big")
            want[s + 7:s + 31] = np.frombuffer(bytes(ip), np.uint8)
            assert sums[2 * i] == v
            off += ps
        assert np.array_equal(got, want), mode


def test_route_addr_sum_host_helper(oracle_mod):
    """engine.addr_sum (what ns_tcp_tx.addr_sum takes) is Checksum(dst,
    Checksum(src, 0)) for IPv4 and IPv6 addresses."""
    import oracle as O
    from netstack_amd.engine import addr_sum

    rng = np.random.default_rng(3)
    for ln in (4, 16):
        for _ in range(50):
            s, d = bytes(rng.integers(0, 256, ln, dtype=np.uint8)), bytes(rng.integers(0, 256, ln, dtype=np.uint8))
            assert addr_sum(s, d) == O.c_checksum(d, O.c_checksum(s, 0))
    assert addr_sum(b"\xff\xff\xff\xff", b"\xff\xff\xff\xff") == O.c_checksum(b"\xff" * 4, O.c_checksum(b"\xff" * 4))
