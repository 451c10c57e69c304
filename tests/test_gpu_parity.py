"""GPU: the HIP engine (through the C ABI) against the oracle and the golden
vectors — bit-exact, every result.  Run on an MI355X: pytest -m gpu."""
import numpy as np
import pytest

from make_golden import materialize

pytestmark = pytest.mark.gpu


def _torch():
    import torch

    assert torch.cuda.is_available(), "GPU tests need a HIP device"
    return torch


def dev_batch(engine, arena_np, desc_np, chained=False, arena_offset=0, stream=None):
    """Run a batch device-resident; arena placed `arena_offset` bytes into a
    device buffer (so its base need not be 16-byte aligned)."""
    torch = _torch()
    buf = torch.empty(arena_offset + max(arena_np.size, 1), dtype=torch.uint8, device="cuda")
    if arena_np.size:
        buf[arena_offset:arena_offset + arena_np.size].copy_(torch.from_numpy(arena_np))
    arena = buf[arena_offset:arena_offset + arena_np.size]
    desc = torch.from_numpy(np.ascontiguousarray(desc_np).view(np.uint8).copy()).cuda()
    out = engine.batch_tensors(arena, desc, chained=chained, stream=stream)
    torch.cuda.synchronize()
    return out.cpu().numpy().view(np.uint16)


# ---- reference KATs through the tcpip/header mirror ------------------------
def test_reference_kats(kat, engine):
    from netstack_amd import header
    from netstack_amd.buffer import NewVectorisedView, NewViewFromBytes

    for c in kat["vv_with_offset"]:
        vv = NewVectorisedView(0, [NewViewFromBytes(bytes.fromhex(v)) for v in c["views"]])
        # checksum_test.go:98
        assert header.ChecksumVVWithOffset(vv, c["initial"], c["off"], c["size"]) == c["want"], c["name"]
        # checksum_test.go:101-105
        v = vv.ToView()
        v.TrimFront(c["off"])
        v.CapLength(c["size"])
        assert header.Checksum(v, c["initial"]) == c["want"], c["name"]
    for c in kat["checksum"]:
        assert header.Checksum(bytes.fromhex(c["buf"]), c["initial"]) == c["want"], c["name"]


def test_golden_vectors(vectors, engine):
    from netstack_amd import header
    from netstack_amd.buffer import NewVectorisedView

    for c in vectors["checksum"]:
        assert header.Checksum(materialize(c["buf"]), c["initial"]) == c["want"], c["name"]
    for c in vectors["vv_with_offset"]:
        views = [materialize(v) for v in c["views"]]
        vv = NewVectorisedView(sum(map(len, views)), views)
        assert header.ChecksumVVWithOffset(vv, c["initial"], c["off"], c["size"]) == c["want"], c["name"]
    for c in vectors["views_restart"]:
        assert header.ChecksumViews([materialize(v) for v in c["views"]], c["initial"]) == c["want"], c["name"]
    for c in vectors["pseudo_header"]:
        got = header.PseudoHeaderChecksum(c["protocol"], bytes.fromhex(c["src"]), bytes.fromhex(c["dst"]),
                                          c["total_len"])
        assert got == c["want"], c["name"]


def test_golden_batches_dev_and_host(vectors, engine):
    import oracle as O

    for c in vectors["batch"]:
        arena = np.frombuffer(materialize(c["arena"]), dtype=np.uint8).copy()
        d = np.array([tuple(x) for x in c["desc"]], dtype=O.DESC_DTYPE)
        for off in (0, 1, 3, 8):
            assert dev_batch(engine, arena, d, c["chained"], arena_offset=off).tolist() == c["want"], c["name"]
        assert engine.batch_host(arena, d, c["chained"]).tolist() == c["want"], c["name"]


# ---- BASELINE.json layouts, subsets and full size -------------------------
@pytest.mark.parametrize("cfg,n", [(2, 65536), (3, 65536), (4, 65536), (1, None)])
def test_config_subsets(engine, cfg, n):
    import oracle as O
    from netstack_amd import workloads as W

    b = W.config(cfg, n)
    arena = b.arena_host()
    want, bad = O.c_batch(arena, b.desc)
    assert bad == 0
    got = dev_batch(engine, arena, b.desc)
    assert np.array_equal(got, want)


@pytest.mark.slow
@pytest.mark.parametrize("cfg", [2, 3, 4])
def test_config_full_size(engine, cfg):
    """Full BASELINE.json batch, generated in HBM; every result vs the C oracle
    on the same bytes (copied back), multi-threaded."""
    torch = _torch()
    import os

    import oracle as O
    from netstack_amd import workloads as W

    b = W.config(cfg)
    arena = b.arena_device("cuda")
    desc = torch.from_numpy(b.desc.view(np.uint8).copy()).cuda()
    out = engine.batch_tensors(arena, desc)
    torch.cuda.synchronize()
    assert engine.sync() == 0
    got = out.cpu().numpy().view(np.uint16)
    host = arena.cpu().numpy()
    want = O.c_batch_mt(host, b.desc, min(16, os.cpu_count() or 1))
    assert np.array_equal(got, want), f"{int((got != want).sum())} mismatches"

    # size-independent property: write ^sum (big-endian) into the 4 padding
    # bytes after each 1500-B packet and re-sum the 1502 bytes: every packet
    # must verify as 0xffff (segment.go:180).  Only cfg2 has padding (stride
    # 1504); the writes stay inside each packet's own slot.
    if cfg == 2:
        assert int(b.desc["off"][-1]) + int(b.desc["len"][-1]) + 2 <= b.arena_bytes
        L = int(b.desc["len"][0])
        offs = torch.from_numpy(b.desc["off"].astype(np.int64)).cuda()
        comp = (~out.to(torch.int32)) & 0xFFFF
        arena[offs + L] = (comp >> 8).to(torch.uint8)
        arena[offs + L + 1] = (comp & 0xFF).to(torch.uint8)
        d2 = b.desc.copy()
        d2["len"] = L + 2
        out2 = engine.batch_tensors(arena, torch.from_numpy(d2.view(np.uint8).copy()).cuda())
        torch.cuda.synchronize()
        assert bool((out2.cpu().numpy().view(np.uint16) == 0xFFFF).all())


# ---- layout edge cases -----------------------------------------------------
def test_unaligned_packed_with_odd_flags(engine):
    import oracle as O
    from netstack_amd import workloads as W

    rng = np.random.default_rng(1)
    n = 20000
    lengths = rng.integers(0, 3000, n).astype(np.uint32)
    lengths[::13] = rng.integers(0, 20, len(lengths[::13]))
    init = rng.integers(0, 65536, n).astype(np.uint16)
    flags = rng.integers(0, 2, n).astype(np.uint16)
    d, end = W.make_desc(lengths, init, align=1, base=5, flags=flags)
    arena = W.random_bytes(99, end + 7)
    want, _ = O.c_batch(arena, d)
    for off in (0, 1, 2, 7, 15):
        assert np.array_equal(dev_batch(engine, arena, d, arena_offset=off), want)


@pytest.mark.parametrize("maxlen", [17, 66, 81, 300])
def test_small_unaligned_packets(engine, maxlen):
    """Small-packet batches (mean < 256 B/descriptor): tiles where every packet
    spans <= 5 chunks take the direct path, others the scanned one."""
    import oracle as O
    from netstack_amd import workloads as W

    rng = np.random.default_rng(maxlen)
    n = 40000
    lengths = rng.integers(0, maxlen, n).astype(np.uint32)
    init = rng.integers(0, 65536, n).astype(np.uint16)
    flags = rng.integers(0, 2, n).astype(np.uint16)
    d, end = W.make_desc(lengths, init, align=1, base=3, flags=flags)
    arena = W.random_bytes(7 + maxlen, end + 5)
    want, _ = O.c_batch(arena, d)
    for off in (0, 9):
        assert np.array_equal(dev_batch(engine, arena, d, arena_offset=off), want)
    perm = rng.permutation(n)  # unsorted table, same packets
    assert np.array_equal(dev_batch(engine, arena, d[perm]), want[perm])


@pytest.mark.parametrize("chained,store", [(False, False), (True, False), (False, True), (True, True)])
def test_quad_lane_direct_path_per_wave(engine, chained, store):
    """The small-packet tiles' two direct shapes, chosen per wave: waves whose
    64 packets all span <= 4 chunks take the quad-lane path (nontemporal
    whole-line loads, quad sums), the others one lane per packet.  Packets of
    0-64 B at every start alignment, odd carry-ins, empties, one 5-chunk
    packet in some waves, chained runs and in-packet stores; all against the
    oracle."""
    import oracle as O
    from netstack_amd import workloads as W

    torch = _torch()
    rng = np.random.default_rng(1234 + 2 * chained + store)
    n = 256 * 24 + 77
    lengths = rng.integers(0, 65, n).astype(np.uint32)
    starts = rng.integers(0, 16, n)
    # a packet spanning 5 chunks in every third wave
    for wv in range(0, n // 64, 3):
        lengths[wv * 64 + int(rng.integers(0, 64))] = 70
    flags = rng.integers(0, 2, n).astype(np.uint16)
    if chained:
        flags |= (2 * (rng.random(n) < 0.4)).astype(np.uint16)
    # packets placed at random 16-B phases with gaps
    off = np.zeros(n, np.uint64)
    pos = 3
    for k in range(n):
        pos = (pos // 16) * 16 + int(starts[k])
        off[k] = pos
        pos += int(lengths[k]) + int(rng.integers(0, 40))
    d = np.zeros(n, dtype=O.DESC_DTYPE)
    d["off"], d["len"], d["flags"] = off, lengths, flags
    d["initial"] = rng.integers(0, 65536, n)
    arena = rng.integers(0, 256, pos + 64, dtype=np.uint8)
    arena[int(off[7]):int(off[7]) + int(lengths[7])] = 0
    if store:
        st = np.flatnonzero((rng.random(n) < 0.3) & (lengths >= 2))
        at = (rng.random(st.size) * (lengths[st] - 1)).astype(np.uint16)
        d["flags"][st] |= (0x4 | (at << 4)).astype(np.uint16)
    want, bad = O.c_batch(arena, d, chained=chained)
    assert bad == 0
    dt = torch.from_numpy(arena).cuda()
    desc = torch.from_numpy(d.view(np.uint8).copy()).cuda()
    out = engine.batch_tensors(dt, desc, chained=chained, store=store)
    torch.cuda.synchronize()
    assert engine.sync() == 0
    got = out.cpu().numpy().view(np.uint16)
    assert np.array_equal(got, want), np.flatnonzero(got != want)[:8]
    if store:
        expect, dropped = O.apply_stores(arena, d, want)
        assert dropped == 0 and np.array_equal(dt.cpu().numpy(), expect)


@pytest.mark.slow
def test_arena_over_4gib_windowed_and_scattered(engine):
    """A 4.5 GiB arena (288 GB HBM makes such batches natural): sorted tiles
    take a per-tile SRD window anywhere in the arena, tiles whose packets
    span >= 4 GiB take the 64-bit global-load path."""
    torch = _torch()
    import oracle as O

    size = (9 << 29) + 12345                       # ~4.5 GiB, odd size
    g = torch.Generator(device="cuda").manual_seed(45)
    arena = torch.randint(0, 256, (size,), dtype=torch.uint8, device="cuda", generator=g)
    host = arena.cpu().numpy()
    rng = np.random.default_rng(45)
    n = 60000
    d = np.zeros(n, dtype=O.DESC_DTYPE)
    # (a) sorted, sparse across the whole arena: every tile fits a window
    d["off"][: n // 2] = np.sort(rng.integers(0, size - 10000, n // 2))
    # (b) scattered over the whole arena: tiles span > 4 GiB
    d["off"][n // 2:] = rng.integers(0, size - 10000, n - n // 2)
    d["len"] = rng.integers(0, 9001, n)
    d["len"][rng.random(n) < 0.3] %= 70
    d["initial"] = rng.integers(0, 65536, n)
    d["flags"] = rng.integers(0, 2, n)
    want, bad = O.c_batch(host, d)
    assert bad == 0
    desc = torch.from_numpy(d.view(np.uint8).copy()).cuda()
    got = engine.batch_tensors(arena, desc)
    torch.cuda.synchronize()
    assert engine.sync() == 0
    assert np.array_equal(got.cpu().numpy().view(np.uint16), want)
    # the last packet ends exactly at the arena's end
    d2 = d[:300].copy()
    d2["off"][-1], d2["len"][-1] = size - 4099, 4099
    want2, _ = O.c_batch(host, d2)
    got2 = engine.batch_tensors(arena, torch.from_numpy(d2.view(np.uint8).copy()).cuda())
    torch.cuda.synchronize()
    assert np.array_equal(got2.cpu().numpy().view(np.uint16), want2)


@pytest.mark.parametrize("lo,hi,n", [(60000, 70000, 3000), (100000, 400000, 300), (2000, 9000, 20000)])
def test_large_packet_tiles(engine, lo, hi, n):
    """Large packets get fewer descriptors per workgroup (launch_hyb's tile
    sizing): every tile size bit-exact, unaligned starts, odd flags."""
    import oracle as O
    from netstack_amd import workloads as W

    rng = np.random.default_rng(lo)
    lengths = rng.integers(lo, hi, n).astype(np.uint32)
    init = rng.integers(0, 65536, n).astype(np.uint16)
    flags = rng.integers(0, 2, n).astype(np.uint16)
    d, end = W.make_desc(lengths, init, align=1, base=7, flags=flags)
    arena = W.random_bytes(lo + 1, end + 3)
    want, _ = O.c_batch(arena, d)
    assert np.array_equal(dev_batch(engine, arena, d, arena_offset=5), want)


def test_random_overlapping_descriptors(engine):
    import oracle as O

    rng = np.random.default_rng(2)
    arena = rng.integers(0, 256, 1 << 20, dtype=np.uint8)
    n = 50000
    d = np.zeros(n, dtype=O.DESC_DTYPE)
    d["off"] = rng.integers(0, arena.size, n)
    d["len"] = np.minimum(rng.integers(0, 70000, n), arena.size - d["off"])
    d["len"][rng.random(n) < 0.5] %= 97
    d["initial"] = rng.integers(0, 65536, n)
    d["flags"] = rng.integers(0, 2, n)
    want, _ = O.c_batch(arena, d)
    assert np.array_equal(dev_batch(engine, arena, d), want)


def test_chained_runs(engine):
    import oracle as O

    rng = np.random.default_rng(3)
    n = 30000
    lengths = rng.integers(0, 400, n)
    d = np.zeros(n, dtype=O.DESC_DTYPE)
    pos = np.concatenate([[0], np.cumsum(lengths[:-1])])
    d["off"], d["len"] = pos, lengths
    d["initial"] = rng.integers(0, 65536, n)
    cont = rng.random(n) < 0.8
    d["flags"] = (cont * 2) | (pos & 1)
    arena = rng.integers(0, 256, int(lengths.sum()) + 1, dtype=np.uint8)
    want, _ = O.c_batch(arena, d, chained=True)
    assert np.array_equal(dev_batch(engine, arena, d, chained=True), want)
    assert np.array_equal(engine.batch_host(arena, d, chained=True), want)


def test_large_single_descriptors_wrap(engine):
    import oracle as O

    for L, fill, init in [(200000, 0xFF, 0), (131074, 0xFF, 0), (1 << 22, 0xFF, 0xFFFF), (3_000_001, None, 7)]:
        arena = np.full(L, fill, dtype=np.uint8) if fill is not None else \
            np.random.default_rng(L).integers(0, 256, L, dtype=np.uint8)
        d = np.zeros(1, dtype=O.DESC_DTYPE)
        d[0] = (0, L, init, 0)
        want, _ = O.c_batch(arena, d)
        assert dev_batch(engine, arena, d).tolist() == want.tolist()


def test_out_of_range_descriptors_counted(engine):
    import oracle as O

    arena = np.arange(1000, dtype=np.uint8)
    d = np.zeros(4, dtype=O.DESC_DTYPE)
    d[0] = (0, 1000, 1, 0)
    d[1] = (999, 2, 2, 0)     # past the end
    d[2] = (5000, 1, 3, 0)    # past the end
    d[3] = (1000, 0, 4, 0)    # empty at the end: fine
    engine.sync()
    got = dev_batch(engine, arena, d)
    assert engine.sync() == 2
    want, bad = O.c_batch(arena, d)
    assert bad == 2 and got.tolist() == want.tolist()
    from netstack_amd._lib import ChecksumError

    with pytest.raises(ChecksumError):
        engine.batch_host(arena, d)


def test_empty_batch_and_empty_packets(engine):
    import oracle as O

    arena = np.zeros(16, dtype=np.uint8)
    d = np.zeros(0, dtype=O.DESC_DTYPE)
    assert engine.batch_host(arena, d).size == 0
    d = np.zeros(300, dtype=O.DESC_DTYPE)
    d["initial"] = np.arange(300)
    assert dev_batch(engine, arena, d).tolist() == list(range(300))


def test_vv_batch_matches_oracle(engine):
    """sendTCPBatch: n x ChecksumVVWithOffset over one GSO payload VV."""
    import oracle as O
    from netstack_amd import header
    from netstack_amd.buffer import NewVectorisedView

    rng = np.random.default_rng(4)
    for trial in range(10):
        views = [rng.integers(0, 256, int(rng.integers(0, 9000)), dtype=np.uint8).tobytes()
                 for _ in range(int(rng.integers(1, 12)))]
        total = sum(map(len, views))
        mss = int(rng.integers(1, 1461))
        segs, off = [], 0
        while off < total:
            sz = min(mss, total - off)
            segs.append((off, sz, int(rng.integers(0, 65536))))
            off += sz
        segs.append((total + 5, 10, 3))  # past the end -> initial
        vv = NewVectorisedView(total, views)
        got = header.ChecksumVVBatch(vv, segs)
        want = [O.c_checksum_vv_with_offset(views, i, o, s) for (o, s, i) in segs]
        assert got == want


def test_on_side_stream(engine):
    torch = _torch()
    import oracle as O
    from netstack_amd import workloads as W

    b = W.config(2, 4096)
    arena = b.arena_host()
    want, _ = O.c_batch(arena, b.desc)
    s = torch.cuda.Stream()
    with torch.cuda.stream(s):
        got = dev_batch(engine, arena, b.desc, stream=s)
    assert np.array_equal(got, want)


@pytest.mark.parametrize("chained", [False, True])
def test_pipelined_batches_over_two_streams(engine, chained):
    """INTEGRATION.md §4's stream of batches (bench.py `pipelined`): distinct
    batches launched back to back round-robin over two streams, each stream
    with its own results, the next batch's ramp overlapping the previous
    one's tail; every batch's results against the oracle.  Chained batches
    also run their fold pass on their stream's own scratch."""
    torch = _torch()
    import oracle as O
    from netstack_amd import workloads as W

    rng = np.random.default_rng(31)
    batches = []
    for k in range(6):
        ln = W.zipf_lengths(40 + k, 3000 + 500 * k)
        d, end = W.make_desc(ln, rng.integers(0, 65536, len(ln)).astype(np.uint16), 16 if k % 2 else 1)
        if chained:
            d["flags"] = rng.integers(0, 4, len(d)).astype(np.uint16)
        arena = W.random_bytes(900 + k, end + 32)
        batches.append((arena, d, O.c_batch(arena, d, chained)[0]))
    ss = [torch.cuda.current_stream(), torch.cuda.Stream()]
    dev = [(torch.from_numpy(a).cuda(), torch.from_numpy(d.view(np.uint8).copy()).cuda()) for a, d, _ in batches]
    outs = [torch.empty(len(d), dtype=torch.int16, device="cuda") for _, d, _ in batches]
    torch.cuda.synchronize()
    for rnd in range(3):
        for o in outs:
            o.fill_(0x5A5A)
        torch.cuda.synchronize()
        for k, (a, d) in enumerate(dev):
            engine.batch_tensors(a, d, outs[k], chained=chained, stream=ss[k % 2])
        torch.cuda.synchronize()
        for k, (_, _, want) in enumerate(batches):
            assert np.array_equal(outs[k].cpu().numpy().view(np.uint16), want), (rnd, k)
    engine.stream_release(ss[1])


def test_fuzz_small(engine):
    import oracle as O

    rng = np.random.default_rng(7)
    for trial in range(30):
        size = int(rng.integers(1, 5000))
        arena = rng.integers(0, 256, size, dtype=np.uint8)
        n = int(rng.integers(1, 700))
        d = np.zeros(n, dtype=O.DESC_DTYPE)
        d["off"] = rng.integers(0, size + 1, n)
        d["len"] = [int(rng.integers(0, size - o + 1)) for o in d["off"]]
        d["initial"] = rng.integers(0, 65536, n)
        d["flags"] = rng.integers(0, 4, n)
        chained = bool(trial % 2)
        want, _ = O.c_batch(arena, d, chained)
        assert np.array_equal(dev_batch(engine, arena, d, chained, arena_offset=trial % 16), want), trial


def test_sorted_dense_tiles_with_gaps_and_empties(engine):
    """Packed (sorted, non-overlapping) tables exercise the dense path: mixed
    gaps, zero-length descriptors (also leading ones), multiple packets per
    16-byte chunk, odd flags, and tiles that fall back to the general path
    because their gaps are too large."""
    import oracle as O

    rng = np.random.default_rng(8)
    for trial in range(12):
        n = int(rng.integers(1, 5000))
        lens = rng.integers(0, [8, 64, 1600, 9000][trial % 4], n)
        lens[rng.random(n) < 0.1] = 0
        if trial % 3 == 0:
            lens[: min(n, 300)] = 0  # a whole leading tile of empties
        gaps = rng.integers(0, [1, 4, 16, 5000][(trial // 4) % 4], n)
        d = np.zeros(n, dtype=O.DESC_DTYPE)
        pos = 0
        for i in range(n):
            pos += int(gaps[i])
            d[i] = (pos if lens[i] else int(rng.integers(0, 1 << 20)), int(lens[i]),
                    int(rng.integers(0, 65536)), int(rng.integers(0, 2)))
            pos += int(lens[i])
        arena = rng.integers(0, 256, pos + 64, dtype=np.uint8)
        d["off"] = np.minimum(d["off"], arena.size)  # empty ones anywhere inside
        want, bad = O.c_batch(arena, d)
        assert bad == 0
        for off in (0, 5):
            assert np.array_equal(dev_batch(engine, arena, d, arena_offset=off), want), (trial, off)


def test_batch_multi_shards_over_contexts(engine):
    """ns_csum_batch_multi: one host batch split over several contexts (here
    three contexts on the single test GPU, standing in for three devices)."""
    import oracle as O
    from netstack_amd import Engine, workloads as W
    from netstack_amd.engine import batch_multi

    b = W.config(4, n=20000)
    arena = b.arena_host()
    want, _ = O.c_batch(arena, b.desc)
    extra = [Engine(0), Engine(0)]
    try:
        got = batch_multi([engine] + extra, arena, b.desc)
    finally:
        for e in extra:
            e.close()
    assert np.array_equal(got, want)


def test_cpp_mirror_reference_tests(engine):
    """tests/cpp/checksum_test.cc: checksum_test.go's TestChecksumVVWithOffset
    and protocol invariants through the C++ tcpip/header mirror."""
    import os
    import subprocess

    from conftest import ROOT

    exe = os.path.join(ROOT, "netstack_amd", "lib", "checksum_test")
    r = subprocess.run([exe], capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stdout + r.stderr
    assert "0 failed" in r.stdout


@pytest.mark.parametrize("chained", [False, True])
def test_w_only_threshold_and_zero_sums(engine, chained):
    """csum_hyb accumulates only W for packets of <= 8190 chunks and the exact
    (T, W) pair in tiles holding a longer one.  Packets on
    both sides of the threshold at odd starts, all-0xFF bytes (largest sums),
    all-zero bytes (S == 0 must stay distinguishable from S == 65535), initial
    0 / 1 / 0xFFFF, odd flags, mixed into the same tiles as small packets —
    plain and chained (the W-only class value as a chained partial)."""
    import oracle as O
    from netstack_amd import workloads as W

    rng = np.random.default_rng(8190)
    big = [131008, 131024, 131039, 131040, 131041, 131055, 131056, 131057, 131072, 131073, 200000]
    lengths, fills = [], []
    for L in big:
        lengths += [L] + list(rng.integers(1, 200, 150))
        fills += ["ff"] + ["rnd"] * 150
    for k in range(3000):  # tiles of small packets only: W-only
        lengths.append(int(rng.integers(0, 300)))
        fills.append(["zero", "ff", "rnd"][k % 3])
    n = len(lengths)
    lengths = np.array(lengths, dtype=np.uint32)
    init = rng.choice(np.array([0, 1, 0xFFFF], dtype=np.uint16), n)
    flags = rng.integers(0, 2, n).astype(np.uint16)
    if chained:
        flags = flags | (2 * (rng.random(n) < 0.6)).astype(np.uint16)
    d, end = W.make_desc(lengths, init, align=1, base=3, flags=flags)
    arena = rng.integers(0, 256, end + 5, dtype=np.uint8)
    for i in range(n):
        o, L = int(d["off"][i]), int(d["len"][i])
        if fills[i] == "ff":
            arena[o:o + L] = 0xFF
        elif fills[i] == "zero":
            arena[o:o + L] = 0
    want, _ = O.c_batch(arena, d, chained=chained)
    got = dev_batch(engine, arena, d, chained=chained, arena_offset=1)
    assert np.array_equal(got, want), np.flatnonzero(got != want)[:10]
    if not chained:
        assert (want == 0).any() and (want == 0xFFFF).any()


def test_concurrent_small_calls_are_combined_bit_exact(engine):
    """Small synchronous calls from many threads on ONE context are
    flat-combined into shared zero-copy launches (csum_api.cpp submit_small).
    Mixed call shapes — VectorisedView batches, single buffers, chained and
    unchained host batches whose CONT flags must be ignored when unchained —
    each result against the oracle."""
    import threading

    import oracle as O
    from netstack_amd import workloads as W

    errors = []

    def worker(t):
        rng = np.random.default_rng(1000 + t)
        try:
            for it in range(30):
                kind = (t + it) % 4
                if kind == 0:
                    buf = rng.integers(0, 256, int(rng.integers(1, 70000)), dtype=np.uint8)
                    cuts = np.sort(rng.integers(0, buf.size, 3))
                    views = [buf[:cuts[0]], buf[cuts[0]:cuts[1]], buf[cuts[1]:]]
                    segs = [(int(o), int(rng.integers(0, 3000)), int(rng.integers(0, 65536)))
                            for o in rng.integers(0, buf.size, 20)]
                    got = engine.vv_batch(views, segs)
                    want = [O.py_checksum_vv_with_offset([bytes(v) for v in views], i, o, s) for o, s, i in segs]
                    if list(got) != want:
                        errors.append((t, it, "vv_batch"))
                elif kind == 1:
                    buf = rng.integers(0, 256, int(rng.integers(0, 9000)), dtype=np.uint8)
                    ini = int(rng.integers(0, 65536))
                    if engine.checksum(buf, ini) != O.py_checksum(bytes(buf), ini):
                        errors.append((t, it, "checksum"))
                else:
                    chained = kind == 3
                    n = int(rng.integers(1, 400))
                    lengths = rng.integers(0, 1600, n).astype(np.uint32)
                    flags = (rng.integers(0, 2, n) | (2 * (rng.random(n) < 0.5))).astype(np.uint16)
                    d, end = W.make_desc(lengths, rng.integers(0, 65536, n).astype(np.uint16), align=1,
                                         base=int(rng.integers(0, 9)), flags=flags)
                    arena = rng.integers(0, 256, end + 3, dtype=np.uint8)
                    want, _ = O.c_batch(arena, d, chained=chained)
                    if not np.array_equal(engine.batch_host(arena, d, chained=chained), want):
                        errors.append((t, it, "batch_host", chained))
        except Exception as e:  # surfaced below
            errors.append((t, repr(e)))

    th = [threading.Thread(target=worker, args=(t,)) for t in range(8)]
    for x in th:
        x.start()
    for x in th:
        x.join(timeout=120)
    assert not errors, errors[:5]


@pytest.mark.parametrize("fused", [True, False])
def test_rx_verification_batch_device_resident(engine, fused):
    """SURVEY §8(f) rank 2 on the device: received IPv4/TCP packets in HBM,
    two independent descriptors per packet (fused: the pseudo-header
    addresses and the TCP segment as one contiguous piece) or three chained
    ones (workloads.rx_batch), one batch_dev.  Every result bit-exact with
    the oracle, every IPv4 header and every intact TCP segment sums to
    0xffff, exactly the corrupted ones fail."""
    import oracle as O
    from netstack_amd import workloads as W

    torch = _torch()
    k = W.per_packet(fused)
    arena, d, bad_idx = W.rx_batch(20000, 77, "cuda", corrupt_every=97, fused=fused)
    desc = torch.from_numpy(d.view(np.uint8).copy()).cuda()
    out = engine.batch_tensors(arena, desc, chained=not fused)
    torch.cuda.synchronize()
    got = out.cpu().numpy().view(np.uint16)
    want, nbad = O.c_batch(arena.cpu().numpy(), d, chained=not fused)
    assert nbad == 0 and np.array_equal(got, want)
    assert (got[0::k] == 0xFFFF).all()
    assert np.array_equal(np.flatnonzero(got[k - 1::k] != 0xFFFF), bad_idx)


@pytest.mark.parametrize("seed", range(12))
def test_randomized_layouts(engine, seed):
    """Randomised batches mixing every packet class the kernel distinguishes —
    empty, tiny (direct path), small runs, line-split big packets, jumbo, and
    >128 KiB packets that switch a tile to the exact accumulator — at random
    alignments, sorted or shuffled tables, random odd/CONT flags, chained or
    not, device- and host-resident; every result against the oracle."""
    import oracle as O
    from netstack_amd import workloads as W

    rng = np.random.default_rng(4242 + seed)
    n = int(rng.integers(1, 6000))
    kind = rng.choice(6, n, p=[0.05, 0.3, 0.3, 0.25, 0.09, 0.01])
    lo = np.array([0, 1, 65, 1000, 9000, 131041])[kind]
    hi = np.array([1, 65, 1000, 9000, 66000, 300000])[kind]
    lengths = rng.integers(lo, hi).astype(np.uint32)
    init = rng.integers(0, 65536, n).astype(np.uint16)
    chained = bool(seed % 2)
    flags = rng.integers(0, 2, n) | (2 * (rng.random(n) < (0.5 if chained else 0.3)))
    d, end = W.make_desc(lengths, init, align=int(rng.choice([1, 2, 16])), base=int(rng.integers(0, 40)),
                         flags=flags.astype(np.uint16))
    if seed % 3 == 0:
        d = d[rng.permutation(n)]
    arena = rng.integers(0, 256, end + int(rng.integers(0, 64)), dtype=np.uint8)
    if seed % 4 == 1:  # runs of 0xFF: largest sums
        arena[rng.random(arena.size) < 0.3] = 0xFF
    want, bad = O.c_batch(arena, d, chained=chained)
    assert bad == 0
    got = dev_batch(engine, arena, d, chained=chained, arena_offset=int(rng.integers(0, 16)))
    assert np.array_equal(got, want), np.flatnonzero(got != want)[:8]
    if seed % 3 == 1:
        assert np.array_equal(engine.batch_host(arena, d, chained=chained), want)


@pytest.mark.parametrize("fused", [True, False])
def test_tx_store_device_resident(engine, fused):
    """The transmit side on the device (ns_csum_batch_dev_store): tx_batch's
    packets with zeroed IPv4/TCP checksum fields, one launch computes and
    stores both fields in place (ipv4.go:236, connect.go:662-663): from the
    main kernel (fused table) or from the run-folding pass (chained table).
    The arena afterwards equals rx_batch's (checksums made independently by
    torch integer ops), the results match the oracle over the pre-store
    bytes, and the RX table over the stored packets verifies."""
    import oracle as O
    from netstack_amd import workloads as W

    torch = _torch()
    n = 20000
    k = W.per_packet(fused)
    arena, d = W.tx_batch(n, 77, "cuda", fused=fused)
    before = arena.cpu().numpy()
    want, nbad = O.c_batch(before, d, chained=not fused)
    assert nbad == 0
    desc = torch.from_numpy(d.view(np.uint8).copy()).cuda()
    out = engine.batch_tensors(arena, desc, chained=not fused, store=True)
    torch.cuda.synchronize()
    assert engine.sync() == 0
    assert np.array_equal(out.cpu().numpy().view(np.uint16), want)
    after = arena.cpu().numpy()
    expect, dropped = O.apply_stores(before, d, want)
    assert dropped == 0 and np.array_equal(after, expect)
    rx, _, _ = W.rx_batch(n, 77, "cuda")
    assert torch.equal(arena, rx)
    rd = torch.from_numpy(W._tcp_desc(n, fused).view(np.uint8).copy()).cuda()
    chk = engine.batch_tensors(arena, rd, chained=not fused)
    torch.cuda.synchronize()
    assert (chk.cpu().numpy().view(np.uint16)[0::k] == 0xFFFF).all()
    assert (chk.cpu().numpy().view(np.uint16)[k - 1::k] == 0xFFFF).all()


def _store_batch(rng, n, chained, big):
    """Random packets, each followed by a 4-byte unread gap; about half the
    descriptors store (^r or raw r) at a random, often odd, offset inside
    their own bytes or into their gap."""
    from netstack_amd import workloads as W

    lengths = (rng.integers(1000, 70000, n) if big else rng.integers(0, 300, n)).astype(np.uint32)
    init = rng.integers(0, 65536, n).astype(np.uint16)
    flags = rng.integers(0, 2, n).astype(np.uint16)
    if chained:
        flags |= (2 * (rng.random(n) < 0.5)).astype(np.uint16)
    d, end = W.make_desc(lengths + 4, init, align=int(rng.choice([1, 2, 16])), base=int(rng.integers(0, 40)),
                         flags=flags)
    d["len"] = lengths
    st = np.flatnonzero(rng.random(n) < 0.5)
    own = (rng.random(st.size) < 0.5) & (lengths[st] >= 2)
    at = np.where(own, (rng.random(st.size) * np.maximum(lengths[st].astype(np.int64) - 1, 1)).astype(np.int64),
                  lengths[st].astype(np.int64) + rng.integers(0, 3, st.size))
    raw = (rng.random(st.size) < 0.25).astype(np.uint16)
    at = np.minimum(at, 4095)  # the 12-bit offset field
    keep = at + 2 <= np.where(own, lengths[st], lengths[st] + 4)
    st, at, raw = st[keep], at[keep], raw[keep]
    d["flags"][st] |= (0x4 | (raw << 3) | (at.astype(np.uint16) << 4)).astype(np.uint16)
    arena = rng.integers(0, 256, end + 8, dtype=np.uint8)
    return arena, d


@pytest.mark.parametrize("seed", range(6))
def test_store_randomized(engine, seed):
    """NS_DESC_STORE over random layouts: small (direct path) and big
    packets, chained or not, stores inside the descriptor's own bytes (read
    before the store) or into an unread gap, ^r and raw r, odd addresses.
    The arena afterwards equals oracle.apply_stores over the oracle's results;
    ns_csum_batch_dev (no store) leaves the same flags unapplied."""
    import oracle as O

    torch = _torch()
    rng = np.random.default_rng(900 + seed)
    chained, big = bool(seed % 2), seed >= 3
    arena, d = _store_batch(rng, int(rng.integers(1, 3000)), chained, big)
    want, bad = O.c_batch(arena, d, chained=chained)
    assert bad == 0
    expect, dropped = O.apply_stores(arena, d, want)
    assert dropped == 0
    # without store: results identical, arena untouched
    dt = torch.from_numpy(arena).cuda()
    desc = torch.from_numpy(d.view(np.uint8).copy()).cuda()
    out = engine.batch_tensors(dt, desc, chained=chained)
    torch.cuda.synchronize()
    assert np.array_equal(out.cpu().numpy().view(np.uint16), want)
    assert np.array_equal(dt.cpu().numpy(), arena)
    out = engine.batch_tensors(dt, desc, chained=chained, store=True)
    torch.cuda.synchronize()
    assert engine.sync() == 0
    assert np.array_equal(out.cpu().numpy().view(np.uint16), want)
    got = dt.cpu().numpy()
    assert np.array_equal(got, expect), np.flatnonzero(got != expect)[:8]


@pytest.mark.parametrize("chained", [False, True])
def test_store_past_arena_dropped_and_counted(engine, chained):
    """A store whose 2 bytes would leave the arena is dropped and counted in
    ns_csum_sync's bad-descriptor count; the result is still written."""
    import oracle as O

    torch = _torch()
    arena = np.arange(64, dtype=np.uint8)
    d = np.zeros(3, dtype=O.DESC_DTYPE)
    d["off"] = [0, 40, 10]
    d["len"] = [20, 24, 6]
    d["flags"] = [0x4 | (63 << 4), 0x4 | (23 << 4), 0x4 | (2 << 4)]  # at 63 (1 byte left), 63, 12
    want, _ = O.c_batch(arena, d, chained=chained)
    expect, dropped = O.apply_stores(arena, d, want)
    assert dropped == 2
    dt = torch.from_numpy(arena).cuda()
    desc = torch.from_numpy(d.view(np.uint8).copy()).cuda()
    engine.sync()
    out = engine.batch_tensors(dt, desc, chained=chained, store=True)
    torch.cuda.synchronize()
    assert engine.sync() == 2
    assert np.array_equal(out.cpu().numpy().view(np.uint16), want)
    assert np.array_equal(dt.cpu().numpy(), expect)


@pytest.mark.parametrize("chained,huge", [(False, False), (True, False), (False, True)])
def test_store_raw_bit_alone_stores_nothing(engine, chained, huge):
    """NS_DESC_STORE_RAW (bit 3) means something only with NS_DESC_STORE
    (bit 2): descriptors flagged RAW alone, with an offset in range or past
    the arena, leave the arena unchanged and count nothing, in the tile
    kernel, the chained fold pass and the huge-descriptor split kernel."""
    import oracle as O

    torch = _torch()
    rng = np.random.default_rng(41 + chained + 2 * huge)
    n = 4 if huge else 3000
    lengths = rng.integers(2 << 20, 3 << 20, n) if huge else rng.integers(2, 2000, n)
    d = np.zeros(n, dtype=O.DESC_DTYPE)
    d["len"] = lengths
    d["off"] = np.concatenate([[0], np.cumsum(lengths + 3)[:-1]])
    d["initial"] = rng.integers(0, 65536, n)
    at = np.minimum(rng.integers(0, 4096, n), 4095).astype(np.uint16)
    d["flags"] = (0x8 | (at << 4) | rng.integers(0, 2, n)).astype(np.uint16)
    if chained:
        d["flags"][1::2] |= 2
    end = int(d["off"][-1] + d["len"][-1])
    d["flags"][-1] = 0x8 | (4095 << 4)  # past the arena too
    arena = rng.integers(0, 256, end, dtype=np.uint8)
    want, bad = O.c_batch(arena, d, chained=chained)
    expect, dropped = O.apply_stores(arena, d, want)
    assert bad == 0 and dropped == 0 and np.array_equal(expect, arena)
    dt = torch.from_numpy(arena).cuda()
    desc = torch.from_numpy(d.view(np.uint8).copy()).cuda()
    engine.sync()
    out = engine.batch_tensors(dt, desc, chained=chained, store=True)
    torch.cuda.synchronize()
    assert engine.sync() == 0
    assert np.array_equal(out.cpu().numpy().view(np.uint16), want)
    assert np.array_equal(dt.cpu().numpy(), arena)


def test_concurrent_chained_batches_on_two_streams_of_one_context(engine):
    """Chained batches (fold scratch) and huge-descriptor batches (split
    scratch) issued on two streams of ONE context without waiting: the
    context keeps scratch per stream, so both streams' results are
    bit-exact.  Out-of-range descriptors on both streams are counted exactly
    once across a sync of one stream (taken while the other may still run)
    and a sync of the device: ns_csum_sync reads and resets the count in one
    device atomic."""
    import oracle as O
    from netstack_amd import workloads as W

    torch = _torch()
    batches = []
    for k, (n, nbad) in enumerate([(250_000, 3), (180_000, 5)]):
        rng = np.random.default_rng(600 + k)
        flags = (2 * (rng.random(n) < 0.8)).astype(np.uint16) | rng.integers(0, 2, n).astype(np.uint16)
        flags[0] = 0
        d, end = W.make_desc(rng.integers(0, 300, n).astype(np.uint32),
                             rng.integers(0, 65536, n).astype(np.uint16), align=2, flags=flags)
        arena = rng.integers(0, 256, end, dtype=np.uint8)
        badi = rng.choice(n, nbad, replace=False)
        d["off"][badi] = end + 10
        d["len"][badi] = 4
        want, bad = O.c_batch(arena, d, chained=True)
        assert bad == nbad
        batches.append((torch.from_numpy(arena).cuda(), torch.from_numpy(d.view(np.uint8).copy()).cuda(), want))
    # two huge-descriptor batches (csum_split) as well
    huge = []
    for k in range(2):
        rng = np.random.default_rng(700 + k)
        d = np.zeros(3, dtype=O.DESC_DTYPE)
        d["len"] = rng.integers(4 << 20, 6 << 20, 3)
        d["off"] = np.concatenate([[1], 1 + np.cumsum(d["len"][:-1].astype(np.uint64))])
        d["initial"] = rng.integers(0, 65536, 3)
        arena = rng.integers(0, 256, int(d["off"][-1] + d["len"][-1]) + 1, dtype=np.uint8)
        want, _ = O.c_batch(arena, d)
        huge.append((torch.from_numpy(arena).cuda(), torch.from_numpy(d.view(np.uint8).copy()).cuda(), want))
    streams = [torch.cuda.Stream(), torch.cuda.Stream()]
    torch.cuda.synchronize()
    engine.sync()
    for rep in range(3):
        outs = []
        for k in range(2):
            a, dd, _ = batches[k]
            outs.append(engine.batch_tensors(a, dd, chained=True, stream=streams[k]))
        houts = [engine.batch_tensors(huge[k][0], huge[k][1], stream=streams[k]) for k in range(2)]
        first = engine.sync(streams[0].cuda_stream)
        torch.cuda.synchronize()
        rest = engine.sync()
        assert first + rest == 8, (rep, first, rest)
        for k in range(2):
            got = outs[k].cpu().numpy().view(np.uint16)
            assert np.array_equal(got, batches[k][2]), (rep, k, np.flatnonzero(got != batches[k][2])[:8])
            assert np.array_equal(houts[k].cpu().numpy().view(np.uint16), huge[k][2]), (rep, k)


@pytest.mark.parametrize("layout", ["one_run", "mixed", "zeros"])
def test_long_chained_runs(engine, layout):
    """Run folding at any run length (the segmented scan of fold_reduce /
    fold_apply): one run over 300K descriptors, runs of random length up to
    50K crossing many 2048-descriptor blocks, and all-zero runs whose results
    hinge on 0 vs 0xFFFF; every result against the oracle."""
    import oracle as O
    from netstack_amd import workloads as W

    rng = np.random.default_rng({"one_run": 1, "mixed": 2, "zeros": 3}[layout])
    n = 300_000
    lengths = rng.integers(0, 40, n).astype(np.uint32)
    init = rng.integers(0, 65536, n).astype(np.uint16)
    if layout == "one_run":
        flags = np.full(n, 2, np.uint16)
    else:
        flags = np.full(n, 2, np.uint16)
        heads = np.cumsum(rng.integers(1, 50_000, 40))
        heads = heads[heads < n]
        flags[heads] = 0
        flags[rng.random(n) < 0.001] = 0
    flags[0] = 0
    flags |= rng.integers(0, 2, n).astype(np.uint16)  # odd carry-ins
    d, end = W.make_desc(lengths, init, align=int(rng.choice([1, 2])), flags=flags)
    arena = rng.integers(0, 256, end + 16, dtype=np.uint8)
    if layout == "zeros":
        arena[:] = 0
        d["initial"][rng.random(n) < 0.9] = 0
    want, bad = O.c_batch(arena, d, chained=True)
    assert bad == 0
    got = dev_batch(engine, arena, d, chained=True)
    assert np.array_equal(got, want), np.flatnonzero(got != want)[:8]


def test_chain_wrap_fallback(engine):
    """A continuation whose 32-bit sum is 0xFFFFFFFF (65,537 words of 0xFFFF,
    above the W-only limit, so summed exactly) makes x + s wrap 2^32 for any
    x >= 1: the launch falls back to Go's sequential fold and stays bit-exact,
    including runs elsewhere in the batch and long runs."""
    import oracle as O
    from netstack_amd import workloads as W

    rng = np.random.default_rng(77)
    n = 20_000
    lengths = rng.integers(0, 60, n).astype(np.uint32)
    lengths[[5, 9000, 15000]] = 131_074
    flags = (2 * (rng.random(n) < 0.7)).astype(np.uint16)
    flags[[5, 9000, 15000]] = 2
    flags[[4, 8999]] = 0
    flags[0] = 0
    init = rng.integers(0, 65536, n).astype(np.uint16)
    d, end = W.make_desc(lengths, init, align=2, flags=flags)
    arena = rng.integers(0, 256, end, dtype=np.uint8)
    for k in (5, 9000, 15000):
        o = int(d["off"][k])
        arena[o:o + 131_074] = 0xFF
    want, bad = O.c_batch(arena, d, chained=True)
    assert bad == 0
    got = dev_batch(engine, arena, d, chained=True)
    assert np.array_equal(got, want), np.flatnonzero(got != want)[:8]
    # and the same batch without the wrapping pieces takes the scan
    d2 = d.copy()
    d2["len"][[5, 9000, 15000]] = 7
    want2, _ = O.c_batch(arena, d2, chained=True)
    assert np.array_equal(dev_batch(engine, arena, d2, chained=True), want2)


def test_fold_carry_walk_path(engine):
    """fold_scan's no-wait path in the product library: a context made with
    NS_OPT_FOLD_WALK folds chained runs with no look-back, every block
    deriving its carry-in by walking its run, as a block does when a
    predecessor is not running (libnetstack_csum.so's own fold_scan
    instance, through ns_csum_batch_dev).  Long runs, short runs and wrapping
    pieces, against the oracle; the same table through the default context
    gives the same results."""
    import oracle as O
    from netstack_amd import Engine, _lib
    from netstack_amd import workloads as W

    torch = _torch()
    rng = np.random.default_rng(31)
    n = 60_000
    lengths = rng.integers(256, 400, n).astype(np.uint32)  # the big-packet kernel instance
    flags = (2 * (rng.random(n) < 0.999)).astype(np.uint16) | rng.integers(0, 2, n).astype(np.uint16)
    flags[0] &= 1
    lengths[[100, 30_000]] = 131_074
    flags[[100, 30_000]] = 2
    d, end = W.make_desc(lengths, rng.integers(0, 65536, n).astype(np.uint16), align=2, flags=flags)
    arena = rng.integers(0, 256, end, dtype=np.uint8)
    for k in (100, 30_000):
        o = int(d["off"][k])
        arena[o:o + 131_074] = 0xFF
    want, bad = O.c_batch(arena, d, chained=True)
    assert bad == 0
    a = torch.from_numpy(arena).cuda()
    dd = torch.from_numpy(d.view(np.uint8).copy()).cuda()
    with Engine(0, flags=_lib.NS_OPT_FOLD_WALK) as walk:
        for eng in (walk, engine):
            out = torch.empty(n, dtype=torch.int16, device="cuda")
            eng.batch_tensors(a, dd, out, chained=True)
            torch.cuda.synchronize()
            assert eng.sync() == 0
            got = out.cpu().numpy().view(np.uint16)
            assert np.array_equal(got, want), np.flatnonzero(got != want)[:8]
    # an unknown option is refused
    with pytest.raises(Exception):
        Engine(0, flags=0x80)


@pytest.mark.parametrize("chained", [False, True])
def test_huge_descriptors_split(engine, chained):
    """A batch of a few descriptors of many MiB (average >= 1 MiB selects
    csum_split: 512-KiB slices over many workgroups): odd offsets and lengths,
    odd carry-ins, an empty and an out-of-range descriptor, runs of 0xFF (the
    uint32 wrap), stores; results and stored bytes against the oracle."""
    import oracle as O

    torch = _torch()
    rng = np.random.default_rng(5 + chained)
    lengths = [40 << 20, 3 << 20, 0, 17 << 20, 1, (9 << 20) + 3, 64 << 20, 12345]
    n = len(lengths)
    d = np.zeros(n, dtype=O.DESC_DTYPE)
    pos = 7
    for k, L in enumerate(lengths):
        d["off"][k] = pos
        d["len"][k] = L
        pos += L + int(rng.integers(0, 40))
    arena = rng.integers(0, 256, pos + 64, dtype=np.uint8)
    arena[int(d["off"][6]):int(d["off"][6]) + (8 << 20)] = 0xFF
    d["initial"] = rng.integers(0, 65536, n)
    d["flags"] = rng.integers(0, 2, n)
    if chained:
        d["flags"][[1, 4, 5, 7]] |= 2
    d["flags"][3] |= 0x4 | (3 << 4)       # store ^r at off + 3 (odd address)
    d["flags"][0] |= 0x4 | 0x8 | (0 << 4)  # raw r at off
    d = np.concatenate([d, np.array([(pos + 100, 5, 0, 0)], dtype=O.DESC_DTYPE)])  # out of range
    want, bad = O.c_batch(arena, d, chained=chained)
    assert bad == 1
    expect, dropped = O.apply_stores(arena, d, want)
    assert dropped == 0
    dt = torch.from_numpy(arena).cuda()
    desc = torch.from_numpy(d.view(np.uint8).copy()).cuda()
    engine.sync()
    out = engine.batch_tensors(dt, desc, chained=chained, store=True)
    torch.cuda.synchronize()
    assert engine.sync() == 1
    got = out.cpu().numpy().view(np.uint16)
    assert np.array_equal(got, want), (got, want)
    assert np.array_equal(dt.cpu().numpy(), expect)


@pytest.mark.parametrize("stride", [16, 32, 48, 64])
@pytest.mark.parametrize("chained", [False, True])
def test_fixed_stride_tables_speculative_loads(engine, stride, chained):
    """Small-packet tables over an arena of exactly n slots of `stride` bytes
    (16-B-aligned): the launcher predicts packet k at byte k * stride and
    loads it beside its descriptor.  Waves where every prediction holds
    (packets at their slot's start, any length up to the slot) use those
    loads; waves with a packet elsewhere in its slot, spanning 5 chunks, or
    out of order fall back, and waves holding a packet over many slots (one
    past the W-only limit) take the scan path.  Every result against the
    oracle, bit for bit, including empties, odd carry-ins, an out-of-range
    descriptor, a permuted table (every prediction wrong) and an unaligned
    arena (no speculation)."""
    import oracle as O

    torch = _torch()
    rng = np.random.default_rng(stride * 7 + chained)
    n = 64 * 40 + 17
    arena = rng.integers(0, 256, n * stride, dtype=np.uint8)
    d = np.zeros(n, dtype=O.DESC_DTYPE)
    d["off"] = np.arange(n, dtype=np.uint64) * np.uint64(stride)
    d["len"] = rng.integers(0, stride + 1, n)
    d["len"][rng.random(n) < 0.05] = 0
    d["initial"] = rng.integers(0, 65536, n)
    d["flags"] = rng.integers(0, 2, n)
    if chained:
        d["flags"] |= (2 * (rng.random(n) < 0.3)).astype(np.uint16)
    # waves 3, 9, ...: one packet moved inside its slot (prediction misses);
    # waves 5, 11, ...: one packet spanning 5 chunks (past its slot)
    for wv in range(3, n // 64, 6):
        k = wv * 64 + int(rng.integers(0, 64))
        d["off"][k] += np.uint64(int(rng.integers(1, 16)))
        d["len"][k] = min(int(d["len"][k]), stride - int(d["off"][k]) % stride)
    for wv in range(5, n // 64 - 1, 6):
        k = wv * 64 + int(rng.integers(0, 63))
        d["off"][k] += np.uint64(8)
        d["len"][k] = 66
    d["off"][100] = n * stride + 16  # out of range: counted, summed as empty
    # wave 7: a packet over many slots; wave 12: one past the W-only limit
    # (> 8190 chunks, Go's uint32 wraps) — each lane then walks its packet
    d["len"][7 * 64 + 5] = 3000
    d["len"][12 * 64 + 9] = min(140_000, n * stride - int(d["off"][12 * 64 + 9]))

    def check(table, arena_offset=0):
        want, bad = O.c_batch(arena, table, chained=chained)
        engine.sync()
        got = dev_batch(engine, arena, table, chained=chained, arena_offset=arena_offset)
        assert engine.sync() == bad
        assert np.array_equal(got, want), np.flatnonzero(got != want)[:10]

    check(d)
    check(d, arena_offset=8)  # unaligned arena base: no speculation
    check(d[rng.permutation(n)] if not chained else d[::-1].copy())  # every prediction wrong


@pytest.mark.parametrize("tiles", [False, True])
@pytest.mark.parametrize("chained", [False, True])
def test_maximum_length_descriptors(engine, chained, tiles):
    """The largest descriptor the table can hold: len = 0xFFFFFFFF (the u32
    maximum, 2^28 + 1 chunks from an unaligned start) at an odd offset, and a
    second one of 2^32 - 7 bytes ending 4 bytes before the end of a 4 GiB +
    4 MiB arena.  Go's uint32 accumulator wraps many times over such a buffer
    (checksum.go:41-43); the oracle wraps the same way.  With a few
    descriptors the batch takes csum_split; with `tiles`, 300 descriptors
    (n >= kSplitMaxN) send them through the tile kernel, where a tile holding
    one spans more than an SRD can address (the 64-bit global-load path)."""
    import oracle as O

    torch = _torch()
    size = (1 << 32) + (1 << 22)
    g = torch.Generator(device="cuda").manual_seed(77 + 2 * chained + tiles)
    arena = torch.randint(0, 256, (size,), dtype=torch.uint8, device="cuda", generator=g)
    host = arena.cpu().numpy()
    rng = np.random.default_rng(77 + 2 * chained + tiles)
    big = [(1, 0xFFFFFFFF), ((1 << 22) + 3, (1 << 32) - 7)]
    small = [(size - 1, 1), (12345, 0)]
    if tiles:
        offs = rng.integers(0, size - 70000, 296)
        small += [(int(o), int(rng.integers(0, 65536))) for o in offs]
    rows = big[:1] + small[: len(small) // 2] + big[1:] + small[len(small) // 2:]
    d = np.zeros(len(rows), dtype=O.DESC_DTYPE)
    d["off"] = [o for o, _ in rows]
    d["len"] = [L for _, L in rows]
    d["initial"] = rng.integers(0, 65536, len(rows))
    d["flags"] = rng.integers(0, 2, len(rows))
    d["flags"][0] |= 1  # odd carry-in on the u32-max descriptor
    if chained:
        d["flags"][1::3] |= 2
    want, bad = O.c_batch(host, d, chained=chained)
    assert bad == 0
    desc = torch.from_numpy(d.view(np.uint8).copy()).cuda()
    engine.sync()
    out = engine.batch_tensors(arena, desc, chained=chained)
    torch.cuda.synchronize()
    assert engine.sync() == 0
    got = out.cpu().numpy().view(np.uint16)
    assert np.array_equal(got, want), np.nonzero(got != want)


@pytest.mark.parametrize("bad_at", [5, 300_000])
def test_host_batch_out_of_range_is_erange_and_pipeline_recovers(engine, bad_at):
    """ns_csum_batch_host over a multi-chunk DMA pipeline (an arena above one
    staging buffer, 128K-descriptor chunks): a descriptor past the arena, in
    the first or a later chunk, fails the call with NS_ERANGE after the
    chunks in flight drained; the next call on the same context is exact."""
    import oracle as O
    from netstack_amd import workloads as W
    from netstack_amd._lib import NS_ERANGE, ChecksumError

    rng = np.random.default_rng(bad_at)
    n = 400_000
    d, end = W.make_desc(rng.integers(0, 64, n).astype(np.uint32), rng.integers(0, 65536, n).astype(np.uint16))
    arena = rng.integers(0, 256, end, dtype=np.uint8)
    bad = d.copy()
    bad["off"][bad_at] = end + 1
    bad["len"][bad_at] = 1
    with pytest.raises(ChecksumError) as ei:
        engine.batch_host(arena, bad)
    assert ei.value.status == NS_ERANGE
    want, _ = O.c_batch(arena, d)
    assert np.array_equal(engine.batch_host(arena, d), want)


def test_host_batch_fixed_stride_chunks(engine):
    """ns_csum_batch_host over 300,000 packets in cfg3's layout (64-B slots):
    the pipeline's 128K-descriptor chunks, rebased to their own staging
    arenas, are fixed-stride arenas of their own, so their launches take the
    speculative payload loads; a corrupted slot start in the last chunk makes
    its waves fall back.  Every result against the oracle."""
    import oracle as O
    from netstack_amd import workloads as W

    b = W.config(3, 300_000)
    arena = b.arena_host()
    d = b.desc.copy()
    d["off"][299_000] += np.uint64(3)
    d["len"][299_000] = 61
    want, bad = O.c_batch(arena, d)
    assert bad == 0
    got = engine.batch_host(arena, d)
    assert np.array_equal(got, want)


@pytest.mark.parametrize("chained", [False, True])
def test_host_batch_pinned_table_read_in_place(engine, chained):
    """ns_csum_batch_host with a page-locked descriptor table (torch
    pin_memory): the DMA pipeline sends each chunk's table straight from the
    caller's memory instead of copying it into staging first.  A multi-chunk
    batch (128K-descriptor chunks) with unaligned starts, odd flags and, with
    `chained`, NS_DESC_CONT runs (never split across chunks), bit-exact
    with the oracle and with the same table passed pageable."""
    import oracle as O
    from netstack_amd import workloads as W

    torch = _torch()
    rng = np.random.default_rng(404 + chained)
    n = 300_001
    lens = rng.integers(0, 200, n).astype(np.uint32)
    d, end = W.make_desc(lens, rng.integers(0, 65536, n).astype(np.uint16), align=1)
    d["flags"] |= rng.integers(0, 2, n).astype(np.uint16)  # NS_DESC_ODD
    if chained:
        d["flags"][1:] |= (rng.random(n - 1) < 0.6).astype(np.uint16) << 1  # NS_DESC_CONT
    arena = rng.integers(0, 256, end, dtype=np.uint8)
    pa = torch.empty(end, dtype=torch.uint8).pin_memory()
    pa.numpy()[:] = arena
    pt = torch.empty(d.nbytes, dtype=torch.uint8).pin_memory()
    pt.numpy()[:] = d.view(np.uint8)
    pd = pt.numpy().view(d.dtype)
    want, nbad = O.c_batch(arena, d, chained=chained)
    assert nbad == 0
    got = engine.batch_host(pa.numpy(), pd, chained=chained)
    assert np.array_equal(got, want)
    assert np.array_equal(engine.batch_host(arena, d, chained=chained), want)
    assert np.array_equal(pd, d)  # the caller's table is not rebased in place


@pytest.mark.parametrize("chained", [False, True])
def test_zero_copy_pass_shapes(engine, chained):
    """Small host batches (<= 1 MiB of bytes) run as zero-copy passes, which
    launch in a PCIe-latency shape: packets below 32 KiB through per-lane
    runs only, 16 KiB tiles, larger ones through the 8-lane groups
    (csum_kernels.hip kZeroCopyBigChunks).  Lengths on both sides of that
    threshold and of the W-only limit (8190 chunks), 1-byte and empty
    packets, odd offsets and odd flags, every result against the oracle."""
    import oracle as O
    from netstack_amd import workloads as W

    rng = np.random.default_rng(2048 + chained)
    edge = [0, 1, 15, 16, 17, 1500, 32 * 1024 - 16, 32 * 1024 - 1, 32 * 1024, 32 * 1024 + 1,
            32 * 1024 + 17, 65536, 131_040, 131_041, 200_000]
    for trial in range(6):
        lens = np.array(edge + list(rng.integers(0, 30_000, 10)), dtype=np.uint32)
        rng.shuffle(lens)
        d, end = W.make_desc(lens, rng.integers(0, 65536, len(lens)).astype(np.uint16), align=1,
                             base=int(rng.integers(0, 7)))
        d["flags"] |= rng.integers(0, 2, len(d)).astype(np.uint16)
        if chained:
            d["flags"][1:] |= (rng.random(len(d) - 1) < 0.5).astype(np.uint16) << 1
        arena = rng.integers(0, 256, end + 8, dtype=np.uint8)
        if trial % 2:
            arena[: end // 2] = 0xFF  # long runs of 0xFF words: the wrap of large packets
        assert end + 8 <= 1 << 20  # one zero-copy pass
        want, nbad = O.c_batch(arena, d, chained=chained)
        assert nbad == 0
        assert np.array_equal(engine.batch_host(arena, d, chained=chained), want)


def _small_call_mix(eng, seed):
    import oracle as O
    from netstack_amd import workloads as W

    rng = np.random.default_rng(seed)
    for L in (0, 1, 1500, 65536, 200_000):
        buf = rng.integers(0, 256, L, dtype=np.uint8)
        ini = int(rng.integers(0, 65536))
        assert eng.checksum(buf, ini) == O.c_checksum(bytes(buf), ini)
    # 40 segments over ~1.2 MB of views: the gather outgrows its 1 MiB stage
    views = [rng.integers(0, 256, int(k), dtype=np.uint8) for k in rng.integers(1, 400_000, 6)]
    segs = [(int(o), int(s), int(i)) for o, s, i in zip(rng.integers(0, 900_000, 40),
                                                        rng.integers(0, 300_000, 40),
                                                        rng.integers(0, 65536, 40))]
    vb = [bytes(v) for v in views]
    assert eng.vv_batch(views, segs).tolist() == [O.c_checksum_vv_with_offset(vb, i, o, s) for o, s, i in segs]
    n = 3000
    d, end = W.make_desc(rng.integers(0, 300, n).astype(np.uint32), rng.integers(0, 65536, n).astype(np.uint16),
                         align=1, flags=(rng.integers(0, 2, n) | (2 * (rng.random(n) < 0.5))).astype(np.uint16))
    arena = rng.integers(0, 256, end, dtype=np.uint8)
    for chained in (False, True):
        want, _ = O.c_batch(arena, d, chained=chained)
        assert np.array_equal(eng.batch_host(arena, d, chained=chained), want)


def test_small_call_mix_default_staging(engine):
    """Small synchronous calls through the default staging (device memory
    written through the BAR on MI355X): single buffers up to 200 KB, a
    VectorisedView batch whose gather outgrows its 1 MiB stage (re-copied
    from its sources), chained and unchained host batches."""
    _small_call_mix(engine, 77)


def test_small_calls_with_host_memory_staging():
    """NS_CSUM_NO_BAR_TABLE=1 (read at ns_csum_init): a context whose
    zero-copy tables and gather stages stay in mapped host memory, as on parts
    without a large BAR, gives the same bit-exact results."""
    import os

    from netstack_amd import Engine

    os.environ["NS_CSUM_NO_BAR_TABLE"] = "1"
    try:
        eng = Engine(0)
    finally:
        del os.environ["NS_CSUM_NO_BAR_TABLE"]
    try:
        _small_call_mix(eng, 78)
    finally:
        eng.close()


@pytest.mark.parametrize("total", [900_000, 1_500_000, 3_300_000, 9_000_000, 15_000_000, 40_000_000])
def test_gathers_across_stage_sizes(engine, total):
    """A VectorisedView batch and a single-buffer Checksum whose gathers end
    in every staging regime: the 1 MiB stage, a larger zero-copy stage it
    grows into (re-copied from the sources each time, up to 16 MiB:
    csum_api.cpp grow_stage), and past 16 MiB the pinned arena and the DMA
    pipeline.  Every result against the oracle."""
    import oracle as O

    rng = np.random.default_rng(total)
    sizes = rng.integers(1, max(2, total // 6), 12)
    sizes = (sizes * (total / sizes.sum())).astype(np.int64) + 1
    views = [rng.integers(0, 256, int(k), dtype=np.uint8) for k in sizes]
    vb = [bytes(v) for v in views]
    tot = int(sum(len(v) for v in vb))
    cuts = np.unique(np.concatenate([[0, tot], rng.integers(0, tot, 40)]))
    # consecutive segments over the whole view (as sendTCPBatch cuts its
    # payload), so the gather holds ~total bytes; one reaches past the end
    segs = [(int(a), int(b - a), int(rng.integers(0, 65536))) for a, b in zip(cuts[:-1], cuts[1:])]
    segs[-1] = (segs[-1][0], segs[-1][1] + 100, segs[-1][2])
    assert engine.vv_batch(views, segs).tolist() == [O.c_checksum_vv_with_offset(vb, i, o, s) for o, s, i in segs]
    buf = np.concatenate(views)
    assert engine.checksum(buf, 0xBEEF) == O.c_checksum(buf.tobytes(), 0xBEEF)


@pytest.mark.parametrize("seed", range(6))
def test_paired_batches_match_the_oracle(engine, seed):
    """NS_BATCH_PAIRED (include/netstack_csum.h): an odd-indexed CONT
    descriptor continues the one before it, a CONT bit on an even-indexed one
    is ignored; the pair is folded inside the tile.  Random tables with CONT
    bits anywhere, ODD bits, small packets (64-wide one-wave tiles) and big
    ones (tiles of 2 to 256 descriptors, the 2-descriptor floor included),
    with and without stores, against oracle.c_batch_paired and
    oracle.apply_stores."""
    import oracle as O

    torch = _torch()
    rng = np.random.default_rng(1700 + seed)
    arena, d = _store_batch(rng, int(rng.integers(1, 4000)), True, seed >= 3)
    want, bad = O.c_batch_paired(arena, d)
    assert bad == 0
    expect, dropped = O.apply_stores(arena, d, want)
    assert dropped == 0
    dt = torch.from_numpy(arena).cuda()
    desc = torch.from_numpy(d.view(np.uint8).copy()).cuda()
    out = engine.batch_tensors(dt, desc, paired=True)
    torch.cuda.synchronize()
    assert np.array_equal(out.cpu().numpy().view(np.uint16), want)
    assert np.array_equal(dt.cpu().numpy(), arena)
    out = engine.batch_tensors(dt, desc, paired=True, store=True)
    torch.cuda.synchronize()
    assert engine.sync() == 0
    assert np.array_equal(out.cpu().numpy().view(np.uint16), want)
    got = dt.cpu().numpy()
    assert np.array_equal(got, expect), np.flatnonzero(got != expect)[:8]


def test_paired_continuation_wraps_as_go_does(engine):
    """A pair whose continuation's word sum reaches 2^32 - 1 (131,074 bytes of
    0xFF: Go's uint32 accumulator wraps once the initial is added) and pieces
    of up to 3 MB (exact accumulation, and 1 MiB+ averages that unpaired
    batches send to csum_split): the in-tile fold reproduces Go's wrap."""
    import oracle as O

    torch = _torch()
    rng = np.random.default_rng(1777)
    lens = [100, 131074, 7, 131074, 131073, 131074, 3_000_001, 200_000, 0, 131074, 65536, 2_500_000]
    init = rng.integers(0, 65536, len(lens)).astype(np.uint16)
    flags = np.array([0, 2, 2, 2, 1, 2, 0, 3, 0, 2, 2, 2], np.uint16)
    from netstack_amd import workloads as W

    d, end = W.make_desc(np.array(lens, np.uint32), init, align=2, flags=flags)
    arena = np.full(end + 16, 0xFF, np.uint8)
    arena[: end // 3] = rng.integers(0, 256, end // 3, dtype=np.uint8)
    want, _ = O.c_batch_paired(arena, d)
    out = engine.batch_tensors(torch.from_numpy(arena).cuda(), torch.from_numpy(d.view(np.uint8).copy()).cuda(),
                               paired=True)
    torch.cuda.synchronize()
    assert np.array_equal(out.cpu().numpy().view(np.uint16), want)


@pytest.mark.parametrize("paired", [False, True])
def test_tx_split_layout_fill(engine, paired):
    """The transmit side in the layout sendTCPBatch builds
    (stack.NewPacketDescriptors' one buffer of header slots, the payload in a
    separate view; workloads.tx_split_*): chained (fold pass) or paired
    (in-tile) tables fill every IPv4 and TCP checksum field.  Results match the
    oracle over the pre-store bytes, the arena equals the one whose checksums
    torch integer ops computed independently, and every filled segment
    verifies."""
    import oracle as O
    from netstack_amd import workloads as W

    torch = _torch()
    n = 20000
    arena, _ = W.tx_split_batch(n, 77, "cuda")
    d = W.tx_split_desc(n, True, paired)
    before = arena.cpu().numpy()
    want, nbad = O.c_batch_paired(before, d) if paired else O.c_batch(before, d, chained=True)
    assert nbad == 0
    desc = torch.from_numpy(d.view(np.uint8).copy()).cuda()
    out = engine.batch_tensors(arena, desc, chained=not paired, paired=paired, store=True)
    torch.cuda.synchronize()
    assert engine.sync() == 0
    assert np.array_equal(out.cpu().numpy().view(np.uint16), want)
    assert torch.equal(arena, W.tx_split_expected(n, 77, "cuda"))
    vd = torch.from_numpy(W.tx_split_desc(n, False, paired).view(np.uint8).copy()).cuda()
    chk = engine.batch_tensors(arena, vd, chained=not paired, paired=paired).cpu().numpy().view(np.uint16)
    ip, tcp = W.tx_split_order(n, paired)
    assert (chk[ip] == 0xFFFF).all() and (chk[tcp] == 0xFFFF).all()


def test_paired_flag_is_device_resident_only(engine):
    """NS_BATCH_PAIRED with NS_BATCH_CHAINED, or on the host-memory entry
    point, is NS_EINVAL."""
    import ctypes

    from netstack_amd import _lib

    torch = _torch()
    a = torch.zeros(64, dtype=torch.uint8, device="cuda")
    d = np.zeros(2, dtype=_lib_desc_dtype())
    d["len"] = 8
    desc = torch.from_numpy(d.view(np.uint8).copy()).cuda()
    with pytest.raises(ValueError):
        engine.batch_tensors(a, desc, chained=True, paired=True)
    ha = np.zeros(64, np.uint8)
    out = np.zeros(2, np.uint16)
    rc = _lib.lib().ns_csum_batch_host(engine._h, ha.ctypes.data, ha.size, d.ctypes.data, 2,
                                       out.ctypes.data_as(ctypes.POINTER(ctypes.c_uint16)), _lib.NS_BATCH_PAIRED)
    assert rc == _lib.NS_EINVAL


def _lib_desc_dtype():
    from netstack_amd.engine import DESC_DTYPE

    return DESC_DTYPE


def test_paired_ring_of_fixed_slots(engine):
    """NS_BATCH_PAIRED on a receive ring of fixed 64-B slots (the one-wave
    small-packet tiles with speculative payload loads, csum_kernels.hip
    spec_load): pairs of slots chained, odd and even CONT bits, against the
    oracle."""
    import oracle as O

    torch = _torch()
    rng = np.random.default_rng(1811)
    n = 50_001
    arena = rng.integers(0, 256, n * 64, dtype=np.uint8)
    from netstack_amd.engine import DESC_DTYPE

    d = np.zeros(n, dtype=DESC_DTYPE)
    d["off"] = np.arange(n, dtype=np.uint64) * np.uint64(64)
    d["len"] = rng.integers(0, 65, n)
    d["initial"] = rng.integers(0, 65536, n)
    d["flags"] = rng.integers(0, 4, n)
    want, _ = O.c_batch_paired(arena, d)
    out = engine.batch_tensors(torch.from_numpy(arena).cuda(), torch.from_numpy(d.view(np.uint8).copy()).cuda(),
                               paired=True)
    torch.cuda.synchronize()
    assert np.array_equal(out.cpu().numpy().view(np.uint16), want)
