"""GPU: the error behaviour of every C-ABI entry point (include/netstack_csum.h,
INTEGRATION.md §1 "Error behaviour"), called through ctypes on a live
context.  Where Go panics (a negative slice bound, checksum.go:69-98's
callers) the ABI returns NS_EINVAL; a descriptor past the arena is
NS_ERANGE on the host path and summed as empty and counted (ns_csum_sync) on
the device path; empty inputs are not errors and give the reference's
results (Checksum(empty, x) == x, checksum.go:97).  No call may crash, hang
or leave the context unusable: a good call after the bad ones must still be
bit-exact."""
import ctypes

import numpy as np
import pytest

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def api():
    import torch  # noqa: F401  (one HIP runtime shared with torch)

    from netstack_amd import Engine, _lib

    eng = Engine(0)
    yield _lib.lib(), _lib, eng
    eng.close()


def _u16():
    return ctypes.c_uint16(0xBEEF)


def test_single_buffer_and_views(api):
    L, C, eng = api
    h = eng._h
    buf = np.arange(100, dtype=np.uint8)
    r = _u16()
    assert L.ns_csum_checksum(None, buf.ctypes.data, 100, 0, ctypes.byref(r)) == C.NS_EINVAL
    assert L.ns_csum_checksum(h, buf.ctypes.data, 100, 0, None) == C.NS_EINVAL
    assert L.ns_csum_checksum(h, None, 100, 0, ctypes.byref(r)) == C.NS_EINVAL
    assert L.ns_csum_checksum(h, buf.ctypes.data, 1 << 32, 0, ctypes.byref(r)) == C.NS_EINVAL
    assert L.ns_csum_checksum(h, None, 0, 0x1234, ctypes.byref(r)) == C.NS_OK and r.value == 0x1234

    views = (C.NsView * 2)(C.NsView(buf.ctypes.data, 60), C.NsView(buf.ctypes.data + 60, 40))
    for off, size in ((-1, 10), (0, -1), (-5, -5)):  # Go: a negative slice bound panics
        assert L.ns_csum_vv_with_offset(h, views, 2, 7, off, size, ctypes.byref(r)) == C.NS_EINVAL
    assert L.ns_csum_vv_with_offset(h, None, 2, 7, 0, 10, ctypes.byref(r)) == C.NS_EINVAL
    # off past the end, and an empty range: the initial (checksum.go:97)
    assert L.ns_csum_vv_with_offset(h, views, 2, 7, 500, 10, ctypes.byref(r)) == C.NS_OK and r.value == 7
    assert L.ns_csum_vv_with_offset(h, views, 2, 9, 10, 0, ctypes.byref(r)) == C.NS_OK and r.value == 9
    bad = (C.NsView * 1)(C.NsView(None, 5))
    assert L.ns_csum_views_restart(h, bad, 1, 0, ctypes.byref(r)) == C.NS_EINVAL
    assert L.ns_csum_views_restart(h, None, 0, 3, ctypes.byref(r)) == C.NS_OK and r.value == 3
    assert L.ns_csum_pseudo_header(h, 6, None, 4, buf.ctypes.data, 4, 20, ctypes.byref(r)) == C.NS_EINVAL


def test_batches_of_segments_and_chains(api):
    L, C, eng = api
    h = eng._h
    buf = np.arange(3000, dtype=np.uint8)
    views = (C.NsView * 1)(C.NsView(buf.ctypes.data, buf.size))
    out = np.zeros(4, np.uint16)
    po = out.ctypes.data_as(ctypes.POINTER(ctypes.c_uint16))
    segs = (C.NsSeg * 2)(C.NsSeg(0, 100, 1, 0, 0), C.NsSeg(-1, 100, 1, 0, 0))
    assert L.ns_csum_vv_batch(h, views, 1, segs, 2, po) == C.NS_EINVAL
    assert L.ns_csum_vv_batch(h, views, 1, None, 2, po) == C.NS_EINVAL
    assert L.ns_csum_vv_batch(h, views, 1, segs, 0, None) == C.NS_OK

    P = C.NsPiece
    end, rs = C.NS_PIECE_END, C.NS_PIECE_RESTART
    unterminated = (P * 2)(P(buf.ctypes.data, 10, 0, rs, 0), P(buf.ctypes.data + 10, 10, 0, 0, 0))
    assert L.ns_csum_chains(h, unterminated, 2, po, 4) == C.NS_EINVAL
    three = (P * 3)(P(buf.ctypes.data, 10, 0, end, 0), P(buf.ctypes.data, 10, 0, end, 0),
                    P(buf.ctypes.data, 10, 0, end, 0))
    assert L.ns_csum_chains(h, three, 3, po, 2) == C.NS_EINVAL  # more chains than outputs
    nulldata = (P * 1)(P(None, 10, 0, end, 0))
    assert L.ns_csum_chains(h, nulldata, 1, po, 4) == C.NS_EINVAL
    assert L.ns_csum_chains(h, None, 0, None, 0) == C.NS_OK


def test_descriptor_tables(api):
    import torch

    L, C, eng = api
    h = eng._h
    from netstack_amd.engine import DESC_DTYPE

    arena = np.arange(1000, dtype=np.uint8)
    d = np.zeros(3, DESC_DTYPE)
    d["off"] = [0, 500, 990]
    d["len"] = [100, 100, 20]  # the last reaches past the arena
    out = np.zeros(3, np.uint16)
    po = out.ctypes.data_as(ctypes.POINTER(ctypes.c_uint16))
    assert L.ns_csum_batch_host(h, arena.ctypes.data, arena.size, d.ctypes.data, 3, po, 0) == C.NS_ERANGE
    assert L.ns_csum_batch_host(h, arena.ctypes.data, arena.size, d.ctypes.data, 3, None, 0) == C.NS_EINVAL
    assert L.ns_csum_batch_host(h, arena.ctypes.data, arena.size, d.ctypes.data, 0, None, 0) == C.NS_OK
    assert L.ns_csum_batch_host(h, arena.ctypes.data, arena.size, d.ctypes.data, 3, po,
                                C.NS_BATCH_PAIRED) == C.NS_EINVAL

    # device path: the out-of-range descriptor is summed as empty (its
    # initial) and counted by ns_csum_sync; flags are validated
    da = torch.from_numpy(arena).cuda()
    dd = torch.from_numpy(d.view(np.uint8).copy()).cuda()
    do = torch.zeros(3, dtype=torch.int16, device="cuda")
    assert eng.sync() == 0
    assert L.ns_csum_batch_dev(h, da.data_ptr(), arena.size, dd.data_ptr(), 3, None, 0, None) == C.NS_EINVAL
    assert L.ns_csum_batch_dev(h, da.data_ptr(), arena.size, dd.data_ptr(), 3, do.data_ptr(),
                               C.NS_BATCH_CHAINED | C.NS_BATCH_PAIRED, None) == C.NS_EINVAL
    assert L.ns_csum_batch_dev(h, da.data_ptr(), arena.size, dd.data_ptr(), 3, do.data_ptr(), 0, None) == C.NS_OK
    torch.cuda.synchronize()
    assert eng.sync() == 1
    import oracle as O

    want, bad = O.c_batch(arena, d)
    assert bad == 1 and np.array_equal(do.cpu().numpy().view(np.uint16), want)
    assert want[2] == d["initial"][2]


def test_packet_buffers_stages_and_misc(api):
    L, C, eng = api
    h = eng._h
    pk = (C.NsPktBuf * 1)(C.NsPktBuf(None, 0, None, 0, 0, 0))
    v = np.zeros(1, np.uint8)
    assert L.ns_csum_packet_buffers(h, pk, 1, 7, None, v.ctypes.data_as(ctypes.POINTER(ctypes.c_uint8))) == \
        C.NS_EINVAL  # no such op
    assert L.ns_csum_packet_buffers(h, None, 1, C.NS_PKB_VERIFY, None, None) == C.NS_EINVAL
    hdr = np.zeros(8, np.uint8)
    huge = (C.NsPktBuf * 1)(C.NsPktBuf(hdr.ctypes.data, 1 << 32, None, 0, 0, 0))
    assert L.ns_csum_packet_buffers(h, huge, 1, C.NS_PKB_FILL, None, None) == C.NS_EINVAL
    # an empty Data: MALFORMED, not an error
    assert L.ns_csum_packet_buffers(h, pk, 1, C.NS_PKB_VERIFY, None,
                                    v.ctypes.data_as(ctypes.POINTER(ctypes.c_uint8))) == C.NS_OK
    assert v[0] == C.NS_PKB_MALFORMED

    stray = np.zeros(16, np.uint8)
    assert L.ns_csum_stage_release(h, stray.ctypes.data) == C.NS_EINVAL  # not an acquired stage
    base = ctypes.c_void_p()
    assert L.ns_csum_stage_acquire(h, 100, None) == C.NS_EINVAL
    assert L.ns_csum_stage_acquire(h, 100, ctypes.byref(base)) == C.NS_OK
    assert L.ns_csum_stage_release(h, base) == C.NS_OK
    assert L.ns_csum_stage_release(h, base) == C.NS_EINVAL  # released twice
    assert L.ns_csum_get_stats(h, None, 0) == C.NS_EINVAL
    assert L.ns_csum_get_stats(None, ctypes.byref(C.NsStats()), 0) == C.NS_EINVAL
    assert L.ns_csum_sync(None, None, None) == C.NS_EINVAL
    assert L.ns_csum_scratch_count(h, None) == C.NS_EINVAL
    assert L.ns_csum_stream_release(None, None) == C.NS_EINVAL


def test_context_still_bit_exact_after_the_errors(api):
    """After every bad call above, the same context's next calls are exact."""
    import oracle as O

    L, C, eng = api
    rng = np.random.default_rng(5)
    for n in (0, 1, 1500, 70_000):
        b = rng.integers(0, 256, n, dtype=np.uint8)
        assert eng.checksum(b, 0x55AA) == O.c_checksum(b.tobytes(), 0x55AA)
    assert eng.sync() == 0
