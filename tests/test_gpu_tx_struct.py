"""GPU: ns_csum_tcp_tx — sendTCPBatch's transmit checksums from the batch's
geometry (transport/tcp/connect.go:668-702, buildTCPHdr :634-666, addIPHeader
network/ipv4/ipv4.go:217-238) — against the oracle's C restatement of those
functions (oracle.c_send_tcp_batch), bit-exact: the whole arena after the
call (both fields of every segment written, every other byte unchanged) and
the un-complemented sums.

Geometries: netstack's own (54-B slots: Ethernet 14 + IPv4 20 + TCP 20,
MSS 1460), slots at odd addresses, odd MSS and slot sizes, TCP options, an
IPv6 route (no IPv4 header, 16-B addresses), MSS 1 and 16 (several segment
ends per 16-B chunk and per window), jumbo and 64 KiB GSO segments, a last
segment of 1 byte, CHECKSUM_PARTIAL, TX offload, 2-byte field stores, and
forced tiles (segments per wave) from 1 to 64."""

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

V4S, V4D = bytes([192, 168, 1, 7]), bytes([10, 200, 3, 99])
V6S = bytes(range(0x20, 0x30))
V6D = bytes(range(0xF0, 0x100))


def _geo(size, mss, slot=54, ip_at=14, ip_len=20, tcp_at=34, tcp_len=20, hdr_off=0, gap=64, pay_first=False,
         src=V4S, dst=V4D):
    n = -(-size // mss)
    if pay_first:
        pay_off = hdr_off
        hdr_off = pay_off + size + gap
        total = hdr_off + n * slot + 37
    else:
        pay_off = hdr_off + n * slot + gap
        total = pay_off + size + 37
    return dict(hdr_off=hdr_off, pay_off=pay_off, size=size, mss=mss, slot=slot, ip_at=ip_at, ip_len=ip_len,
                tcp_at=tcp_at, tcp_len=tcp_len, src=src, dst=dst, protocol=6), total


CASES = {
    "netstack_default": _geo(1460 * 40, 1460),
    "short_last_odd": _geo(1460 * 39 + 7, 1460),
    "last_is_one_byte": _geo(1460 * 5 + 1, 1460),
    "odd_slots_odd_mss": _geo(1461 * 50 + 3, 1461, slot=55, hdr_off=3, gap=5),
    "options_32b_tcp": _geo(1448 * 70 + 100, 1448, slot=66, tcp_len=32),
    "ipv6_route": _geo(1440 * 33 + 11, 1440, slot=74, ip_len=0, tcp_at=54, src=V6S, dst=V6D),
    "payload_before_slots": _geo(1460 * 20 + 9, 1460, pay_first=True, hdr_off=13),
    "mss_16": _geo(16 * 700 + 5, 16),
    "mss_7": _geo(7 * 900 + 3, 7, hdr_off=1),
    "mss_1": _geo(3000, 1),
    "size_below_mss": _geo(999, 1460),
    "jumbo_9000": _geo(9000 * 9 + 17, 9000, hdr_off=8),
    "gso_64k": _geo(65535 * 3 + 1, 65535, gap=1),
    "ip_header_with_options": _geo(1460 * 12, 1460, slot=78, ip_len=44, tcp_at=58),
    # IPv6 with TCP options: 86-B and 114-B slots, whose 64-slot header tiles
    # take 6 and 8 chunks per lane
    "ipv6_tcp_options": _geo(1408 * 70 + 5, 1408, slot=86, ip_len=0, tcp_at=54, tcp_len=32, src=V6S, dst=V6D),
    "ipv6_max_tcp_options": _geo(1380 * 66 + 1, 1380, slot=114, ip_len=0, tcp_at=54, tcp_len=60, src=V6S,
                                 dst=V6D),
}


def _arena(total, geo, seed):
    rng = np.random.default_rng(seed)
    a = rng.integers(0, 256, total, dtype=np.uint8)
    n = -(-geo["size"] // geo["mss"])
    # the route's addresses in each IPv4 header (the fields stay random: the
    # call must sum them as zero)
    if geo["ip_len"]:
        for i in range(n):
            at = geo["hdr_off"] + i * geo["slot"] + geo["ip_at"]
            a[at + 12:at + 16] = np.frombuffer(geo["src"], np.uint8)
            a[at + 16:at + 20] = np.frombuffer(geo["dst"], np.uint8)
    return a


def _run(engine, a, geo, mode="full", fields_only=False, tile=None, offset=0, htile=None, passes=None, variant=0):
    import torch

    buf = torch.empty(offset + a.size, dtype=torch.uint8, device="cuda")
    buf[offset:].copy_(torch.from_numpy(a))
    arena = buf[offset:]
    n = -(-geo["size"] // geo["mss"])
    out = torch.full((2 * n,), -1, dtype=torch.int16, device="cuda")
    # the A/B knobs go through ns_csum_set_tx_tuning (never the environment)
    engine.set_tx_tuning(variant=variant, tile=tile or 0, htile=htile or 0, passes=passes or 0)
    try:
        engine.tcp_tx(arena, geo, out=out, mode=mode, fields_only=fields_only)
        torch.cuda.synchronize()
    finally:
        engine.set_tx_tuning()
    return arena.cpu().numpy(), out.cpu().numpy().view(np.uint16)


def _want(oracle_mod, a, geo, mode="full"):
    g = geo
    return oracle_mod.c_send_tcp_batch(a, g["hdr_off"], g["pay_off"], g["size"], g["mss"], g["slot"], g["ip_at"],
                                       g["ip_len"], g["tcp_at"], g["tcp_len"], g["src"], g["dst"], g["protocol"],
                                       mode)


def _check(got_arena, got_sums, want_arena, want_sums, what):
    bad = np.flatnonzero(got_arena != want_arena)
    assert bad.size == 0, f"{what}: {bad.size} arena bytes differ, first at {bad[:8]}"
    diff = np.flatnonzero(got_sums != want_sums)
    assert diff.size == 0, f"{what}: {diff.size} sums differ, first at {diff[:8]}"


@pytest.mark.parametrize("name", sorted(CASES))
def test_geometry_bit_exact(engine, oracle_mod, name):
    """Each geometry in every shape: one fused pass (what batches below
    kTxTwoPassMinBytes take), the payload + header passes (production: the
    payload pass in 8-lane groups, one segment each, header stores written
    through, one tile per wave), the group pass with default-policy stores
    (variant 5), round 5's windowed payload pass (variant 6) and the
    persistent header pass (variant 7)."""
    geo, total = CASES[name]
    a = _arena(total, geo, seed=len(name))
    wa, ws = _want(oracle_mod, a, geo)
    for passes, variant in ((1, 0), (2, 0), (2, 5), (2, 6), (2, 7)):
        for offset in (0, 5):
            ga, gs = _run(engine, a, geo, offset=offset, passes=passes, variant=variant)
            _check(ga, gs, wa, ws, f"{name} ({passes} passes, variant {variant}, arena at +{offset})")


@pytest.mark.parametrize("tile", [1, 2, 7, 31, 32, 33, 64])
def test_forced_tiles(engine, oracle_mod, tile):
    for name in ("short_last_odd", "odd_slots_odd_mss", "mss_7", "options_32b_tcp"):
        geo, total = CASES[name]
        a = _arena(total, geo, seed=tile)
        wa, ws = _want(oracle_mod, a, geo)
        # (the tile is the fused pass's and the windowed payload pass's: a
        # forced tile selects the windowed pass)
        for passes, variant in ((1, 0), (2, 0)):
            ga, gs = _run(engine, a, geo, tile=tile, passes=passes, variant=variant)
            _check(ga, gs, wa, ws, f"{name} tile {tile}, {passes} passes, variant {variant}")


@pytest.mark.parametrize("htile", [1, 3, 64, 100, 129, 222])
def test_header_pass_tiles(engine, oracle_mod, htile):
    """The header pass's tile (ns_csum_set_tx_tuning htile): up to 256 segments per wave,
    each lane looping over every 64th; with and without d_out (payload values
    parked in d_out or in per-stream scratch).  At 64 segments the IPv6
    geometries' tiles take 5, 6 and 8 chunks per lane."""
    for name in ("short_last_odd", "odd_slots_odd_mss", "ipv6_route", "ipv6_tcp_options", "ipv6_max_tcp_options"):
        geo, total = CASES[name]
        if htile * geo["slot"] > 12 << 10:
            continue
        a = _arena(total, geo, seed=htile)
        wa, ws = _want(oracle_mod, a, geo)
        ga, gs = _run(engine, a, geo, htile=htile, passes=2)
        _check(ga, gs, wa, ws, f"{name} header tile {htile}")
        for mode in ("partial",):
            wa2, ws2 = _want(oracle_mod, a, geo, mode)
            ga2, gs2 = _run(engine, a, geo, mode=mode, tile=htile)  # one header-only pass
            _check(ga2, gs2, wa2, ws2, f"{name} {mode} tile {htile}")


def test_without_out_uses_scratch(engine, oracle_mod):
    """d_out = NULL: two passes keep the payload values in the stream's
    scratch (forced here, and by size in the large batch below)."""
    import torch

    geo, total = CASES["odd_slots_odd_mss"]
    a = _arena(total, geo, seed=21)
    wa, _ = _want(oracle_mod, a, geo)
    buf = torch.from_numpy(a).cuda()
    engine.set_tx_tuning(passes=2)
    try:
        engine.tcp_tx(buf, geo)
        torch.cuda.synchronize()
    finally:
        engine.set_tx_tuning()
    assert np.array_equal(buf.cpu().numpy(), wa)


@pytest.mark.parametrize("mode", ["partial", "none"])
def test_partial_and_offload(engine, oracle_mod, mode):
    for name in ("netstack_default", "odd_slots_odd_mss", "ipv6_route"):
        geo, total = CASES[name]
        a = _arena(total, geo, seed=3)
        wa, ws = _want(oracle_mod, a, geo, mode)
        ga, gs = _run(engine, a, geo, mode=mode)
        _check(ga, gs, wa, ws, f"{name} {mode}")


def test_fields_only_stores(engine, oracle_mod):
    for name in ("netstack_default", "odd_slots_odd_mss", "mss_7", "ipv6_route"):
        geo, total = CASES[name]
        a = _arena(total, geo, seed=4)
        for mode, passes in (("full", 1), ("full", 2), ("partial", None)):
            wa, ws = _want(oracle_mod, a, geo, mode)
            ga, gs = _run(engine, a, geo, mode=mode, fields_only=True, tile=32, passes=passes)
            _check(ga, gs, wa, ws, f"{name} {mode} fields only, {passes} passes")


def test_many_segments_full_tiles(engine, oracle_mod):
    """Batches large enough for the launcher's own tiles, MSS 1460 (102 MB:
    two passes by size), the same over an IPv6 route (74-B slots: the header
    pass's 64-slot tile would pass 4 KiB, so the launcher picks another) and
    MSS 16 (one pass; up to two segment ends per window per lane row), with
    and without d_out."""
    import torch

    for size, mss, v6 in ((1460 * 70_000 - 3, 1460, False), (1440 * 72_000 - 5, 1440, True),
                          (16 * 70_000 + 9, 16, False)):
        geo, total = (_geo(size, mss, slot=74, ip_len=0, tcp_at=54, src=V6S, dst=V6D, hdr_off=7) if v6
                      else _geo(size, mss, hdr_off=7))
        a = _arena(total, geo, seed=mss)
        wa, ws = _want(oracle_mod, a, geo)
        ga, gs = _run(engine, a, geo)
        _check(ga, gs, wa, ws, f"{size} B at MSS {mss}")
        buf = torch.from_numpy(a).cuda()
        engine.tcp_tx(buf, geo)  # no d_out: per-stream scratch above kTxTwoPassMinBytes
        torch.cuda.synchronize()
        assert np.array_equal(buf.cpu().numpy(), wa)


def test_bench_layout_matches_table_path(engine):
    """workloads.tx_struct_geometry over the bench's sendTCPBatch-layout arena:
    the same fill as the NS_BATCH_PAIRED table (tx_split_desc) and as
    tx_split_expected, byte for byte."""
    import torch

    from netstack_amd import workloads as W

    n = 20_000
    arena, _ = W.tx_split_batch(n, 11, "cuda")
    engine.tcp_tx(arena, W.tx_struct_geometry(n))
    want = W.tx_split_expected(n, 11, "cuda")
    torch.cuda.synchronize()
    assert torch.equal(arena, want)
    arena2, _ = W.tx_split_batch(n, 11, "cuda")
    desc = torch.from_numpy(W.tx_split_desc(n, paired=True).view(np.uint8).copy()).cuda()
    engine.batch_tensors(arena2, desc, store=True, paired=True)
    torch.cuda.synchronize()
    assert torch.equal(arena2, want)


def test_errors(engine):
    import ctypes

    import torch

    from netstack_amd import _lib

    L = _lib.lib()
    h = engine._h
    geo, total = CASES["netstack_default"]
    buf = torch.zeros(total, dtype=torch.uint8, device="cuda")

    def call(**kw):
        t = _lib.NsTcpTx()
        g = dict(geo, **kw)
        for k in ("hdr_off", "pay_off", "size", "mss", "slot", "ip_at", "ip_len", "tcp_at", "tcp_len"):
            setattr(t, k, g[k])
        t.protocol, t.flags = g.get("protocol", 6), g.get("flags", 0)
        return L.ns_csum_tcp_tx(h, buf.data_ptr(), g.get("arena_bytes", total), ctypes.byref(t), None, None)

    assert call() == _lib.NS_OK
    assert L.ns_csum_tcp_tx(None, buf.data_ptr(), total, None, None, None) == _lib.NS_EINVAL
    assert L.ns_csum_tcp_tx(h, buf.data_ptr(), total, None, None, None) == _lib.NS_EINVAL
    for bad in (dict(mss=0), dict(mss=65536), dict(slot=0), dict(slot=5000), dict(ip_len=10),
                dict(ip_len=64), dict(ip_at=40), dict(tcp_len=16), dict(tcp_len=64), dict(tcp_at=40),
                dict(flags=_lib.NS_TX_TCP_PARTIAL | _lib.NS_TX_TCP_NONE), dict(flags=0x80),
                dict(pay_off=geo["hdr_off"] + 100),  # payload over the slots
                dict(protocol=256),  # PseudoHeaderChecksum takes uint8(protocol) (checksum.go:121)
                dict(tcp_at=30)):  # TCP header over the IPv4 header's last bytes
        assert call(**bad) == _lib.NS_EINVAL, bad
    assert call(arena_bytes=geo["pay_off"] + 10) == _lib.NS_ERANGE
    assert call(pay_off=total - 10) == _lib.NS_ERANGE
    assert call(size=0) == _lib.NS_OK  # no segments (connect.go:675)
    # TX offload and no IPv4 header: nothing to do, and the slots may be anything
    assert call(flags=_lib.NS_TX_TCP_NONE, ip_len=0, tcp_len=0) == _lib.NS_OK
    torch.cuda.synchronize()
    assert engine.sync() == 0


def test_two_streams_keep_their_own_scratch(engine, oracle_mod):
    """Two-pass calls without d_out on two streams at once: each stream's
    payload values live in that stream's scratch, so interleaved calls never
    see each other's (ns_csum_stream_release frees them afterwards)."""
    import torch

    geos = [CASES["odd_slots_odd_mss"], CASES["options_32b_tcp"]]
    streams = [torch.cuda.Stream(), torch.cuda.Stream()]
    bufs, wants = [], []
    for k, (geo, total) in enumerate(geos):
        a = _arena(total, geo, seed=100 + k)
        wants.append(_want(oracle_mod, a, geo)[0])
        bufs.append(torch.from_numpy(a).cuda())
    torch.cuda.synchronize()
    engine.set_tx_tuning(passes=2)
    try:
        for _ in range(3):  # refills of the same fields: idempotent
            for k in range(2):
                engine.tcp_tx(bufs[k], geos[k][0], stream=streams[k])
        torch.cuda.synchronize()
    finally:
        engine.set_tx_tuning()
    for k in range(2):
        assert np.array_equal(bufs[k].cpu().numpy(), wants[k]), k
        engine.stream_release(streams[k])
    assert engine.sync() == 0


def test_many_calls_in_one_launch(engine, oracle_mod):
    """ns_csum_tcp_tx_multi: calls of different geometries (slot sizes, MSS,
    IPv6, options, partial / offload modes, empty) laid out side by side in
    one arena, in one launch; each call's fill and sums equal the oracle's
    for that call alone, and every other byte is unchanged."""
    import torch

    rng = np.random.default_rng(77)
    specs = [("netstack_default", "full"), ("odd_slots_odd_mss", "full"), ("ipv6_route", "full"),
             ("options_32b_tcp", "partial"), ("mss_7", "full"), ("size_below_mss", "none"),
             ("ip_header_with_options", "full"), ("last_is_one_byte", "full")]
    geos, pos, parts = [], 3, []
    for name, mode in specs * 3:
        geo, total = CASES[name]
        g = dict(geo)
        g["hdr_off"] += pos
        g["pay_off"] += pos
        g["mode"] = mode
        geos.append(g)
        parts.append((pos, total, mode))
        pos += total + int(rng.integers(0, 40))
    geos.append(dict(CASES["netstack_default"][0], size=0, hdr_off=0, pay_off=0))  # no segments
    a = rng.integers(0, 256, pos + 64, dtype=np.uint8)
    want = a.copy()
    sums = []
    for g, (p, total, mode) in zip(geos, parts):
        n = -(-g["size"] // g["mss"])
        if g["ip_len"]:
            for i in range(n):
                at = g["hdr_off"] + i * g["slot"] + g["ip_at"]
                a[at + 12:at + 16] = np.frombuffer(g["src"], np.uint8)
                a[at + 16:at + 20] = np.frombuffer(g["dst"], np.uint8)
    want = a.copy()
    for g, (p, total, mode) in zip(geos, parts):
        wa, ws = oracle_mod.c_send_tcp_batch(want, g["hdr_off"], g["pay_off"], g["size"], g["mss"], g["slot"],
                                             g["ip_at"], g["ip_len"], g["tcp_at"], g["tcp_len"], g["src"], g["dst"],
                                             g["protocol"], mode, copy=False)
        sums.append(ws)
    ntot = sum(len(x) // 2 for x in sums)
    buf = torch.from_numpy(a).cuda()
    out = torch.full((2 * ntot,), -1, dtype=torch.int16, device="cuda")
    engine.tcp_tx_multi(buf, geos, out=out)
    torch.cuda.synchronize()
    got = buf.cpu().numpy()
    bad = np.flatnonzero(got != want)
    assert bad.size == 0, f"{bad.size} bytes differ, first at {bad[:8]}"
    assert np.array_equal(out.cpu().numpy().view(np.uint16), np.concatenate(sums))
    # again without d_out, and an overlap is refused
    buf2 = torch.from_numpy(a).cuda()
    engine.tcp_tx_multi(buf2, geos)
    torch.cuda.synchronize()
    assert np.array_equal(buf2.cpu().numpy(), want)
    clash = [geos[0], dict(geos[1], hdr_off=geos[0]["hdr_off"] + 10)]
    with pytest.raises(ValueError):  # NS_EINVAL
        engine.tcp_tx_multi(buf2, clash)
    assert engine.sync() == 0


@pytest.mark.latency
def test_multi_calls_do_not_wait_for_a_busy_stream(engine, oracle_mod):
    """ns_csum_tcp_tx_multi is asynchronous: back-to-back calls behind ~100 ms
    of queued work on their stream return without waiting for it (each call's
    pinned table copy comes from a ring of 8; a wait happens only when the
    device is 8 uploads behind).  Round 4's single copy made call k wait for
    call k-1's upload, i.e. for everything queued before it.  The fills are
    then checked against the oracle."""
    import time

    import torch

    geo, total = CASES["netstack_default"]
    a = _arena(total, geo, seed=31)
    wa, _ = _want(oracle_mod, a, geo)
    bufs = [torch.from_numpy(a).cuda() for _ in range(6)]
    stream = torch.cuda.Stream()
    torch.cuda.synchronize()
    with torch.cuda.stream(stream):
        torch.cuda._sleep(200_000_000)  # ~100 ms of GPU time queued first
        t0 = time.perf_counter()
        for b in bufs:
            engine.tcp_tx_multi(b, [geo], stream=stream)
        host = time.perf_counter() - t0
    torch.cuda.synchronize()
    assert host < 0.03, f"{len(bufs)} calls took {host * 1e3:.1f} ms on the host"
    for b in bufs:
        assert np.array_equal(b.cpu().numpy(), wa)
    engine.stream_release(stream)
