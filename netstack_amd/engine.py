"""Engine: a Python handle on one ``ns_csum_ctx`` (one GPU).

Thin wrappers over the C ABI (include/netstack_csum.h).  All checksum
arithmetic happens in the gfx950 kernels; this module only marshals pointers.
"""
from __future__ import annotations

import ctypes
import functools
import threading

import numpy as np

from . import _lib
from ._lib import NsOpts, NsPiece, NsSeg, NsView, check, lib

DESC_DTYPE = np.dtype(
    [("off", "<u8"), ("len", "<u4"), ("initial", "<u2"), ("flags", "<u2")], align=False)
assert DESC_DTYPE.itemsize == 16

ODD = _lib.NS_DESC_ODD
CONT = _lib.NS_DESC_CONT


def device_count() -> int:
    n = ctypes.c_int(0)
    rc = lib().ns_csum_device_count(ctypes.byref(n))
    if rc == _lib.NS_ENODEV:
        return 0
    check(rc, "ns_csum_device_count")
    return int(n.value)


def _u8(buf) -> np.ndarray:
    if isinstance(buf, np.ndarray):
        return np.ascontiguousarray(buf.reshape(-1).view(np.uint8))
    return np.frombuffer(memoryview(buf).cast("B"), dtype=np.uint8)


def _ptr(a: np.ndarray):
    return a.ctypes.data if a.size else None


def _views(views):
    """Marshal a sequence of byte buffers into an ns_view array (keep-alive
    list returned alongside)."""
    arrs = [_u8(v) for v in views]
    arr_t = NsView * max(len(arrs), 1)
    cv = arr_t(*[NsView(_ptr(a), a.size) for a in arrs])
    return cv, arrs


class Engine:
    """One ns_csum_ctx bound to a HIP device."""

    def __init__(self, device: int = 0, staging_bytes: int = 0, flags: int = 0):
        self.device = device
        opts = NsOpts(device, flags, staging_bytes)
        h = ctypes.c_void_p()
        check(lib().ns_csum_init(ctypes.byref(opts), ctypes.byref(h)), "ns_csum_init")
        self._h = h

    # -- lifetime -----------------------------------------------------------
    def close(self) -> None:
        if getattr(self, "_h", None):
            lib().ns_csum_destroy(self._h)
            self._h = None

    def __del__(self):  # pragma: no cover - interpreter shutdown order
        try:
            self.close()
        except Exception:
            pass

    def __enter__(self):
        return self

    def __exit__(self, *a):
        self.close()

    # -- device-resident batch (the hot path) ------------------------------
    def batch_dev(self, arena_ptr: int, arena_bytes: int, desc_ptr: int, n: int,
                  out_ptr: int, chained: bool = False, stream: int | None = None,
                  store: bool = False, paired: bool = False) -> None:
        """Enqueue (asynchronously) the batch on `stream` (hipStream_t as int).
        With store=True (ns_csum_batch_dev_store) descriptors flagged
        NS_DESC_STORE also write their result into the arena; paired=True is
        NS_BATCH_PAIRED (runs of two: an odd-indexed NS_DESC_CONT descriptor
        continues the one before it)."""
        fn, name = (lib().ns_csum_batch_dev_store, "ns_csum_batch_dev_store") if store else \
            (lib().ns_csum_batch_dev, "ns_csum_batch_dev")
        flags = (_lib.NS_BATCH_CHAINED if chained else 0) | (_lib.NS_BATCH_PAIRED if paired else 0)
        check(fn(self._h, arena_ptr, arena_bytes, desc_ptr, n, out_ptr, flags, stream), name)

    def batch_tensors(self, arena, desc, out=None, chained: bool = False, stream=None, store: bool = False,
                      paired: bool = False):
        """torch front end: `arena` uint8 CUDA tensor, `desc` CUDA tensor whose
        bytes are the 16-byte ns_pkt_desc table, `out` int16/uint16 CUDA tensor
        of n elements (allocated if None).  Launches on `stream` (a
        torch.cuda.Stream, default: torch's current stream) and returns `out`
        without synchronising."""
        import torch

        if not (arena.is_cuda and desc.is_cuda):
            raise ValueError("arena and desc must be device tensors")
        if desc.numel() * desc.element_size() % 16:
            raise ValueError("descriptor table must be a whole number of 16-byte entries")
        n = desc.numel() * desc.element_size() // 16
        if out is None:
            out = torch.empty(n, dtype=torch.int16, device=arena.device)
        if out.numel() < n or out.element_size() != 2:
            raise ValueError("out must hold n 16-bit results")
        if stream is None:
            stream = torch.cuda.current_stream(arena.device)
        self.batch_dev(arena.data_ptr(), arena.numel() * arena.element_size(), desc.data_ptr(), n,
                       out.data_ptr(), chained, stream.cuda_stream, store, paired)
        return out

    def tcp_tx(self, arena, geo: dict, out=None, stream=None, mode: str = "full",
               fields_only: bool = False):
        """sendTCPBatch's transmit checksums from its geometry
        (ns_csum_tcp_tx): `arena` a uint8 CUDA tensor holding the header slots
        and the payload; `geo` the keys of ns_tcp_tx (hdr_off, pay_off, size,
        mss, slot, ip_at, ip_len, tcp_at, tcp_len, protocol) plus the route's
        `src` and `dst` addresses (or `addr_sum`).  mode: "full", "partial"
        (CHECKSUM_PARTIAL) or "none" (TX checksum offload).  `out` (optional)
        receives the 2n un-complemented sums.  Launches on `stream` (default:
        torch's current stream) without synchronising; returns `out`."""
        import torch

        if not arena.is_cuda:
            raise ValueError("arena must be a device tensor")
        t = _lib.NsTcpTx(geo["hdr_off"], geo["pay_off"], geo["size"], geo["mss"], geo["slot"], geo["ip_at"],
                         geo["ip_len"], geo["tcp_at"], geo["tcp_len"],
                         geo["addr_sum"] if "addr_sum" in geo else addr_sum(bytes(geo["src"]), bytes(geo["dst"])),
                         geo.get("protocol", 6),
                         _TX_MODES[mode] | (_lib.NS_TX_FIELDS_ONLY if fields_only else 0))
        if out is not None:
            n = -(-int(geo["size"]) // max(int(geo["mss"]), 1))
            if not out.is_cuda or out.numel() < 2 * n or out.element_size() != 2:
                raise ValueError("out must be a device tensor of 2n 16-bit sums")
        if stream is None:
            stream = torch.cuda.current_stream(arena.device)
        check(lib().ns_csum_tcp_tx(self._h, arena.data_ptr(), arena.numel() * arena.element_size(),
                                   ctypes.byref(t), out.data_ptr() if out is not None else None,
                                   getattr(stream, "cuda_stream", stream)), "ns_csum_tcp_tx")
        return out

    def tcp_tx_multi(self, arena, geos, out=None, stream=None, mode: str = "full"):
        """Many sendTCPBatch calls over one arena in one launch
        (ns_csum_tcp_tx_multi): `geos` a list of tcp_tx geometries; `out`
        (optional) receives call k's 2n_k sums after those of calls < k."""
        import torch

        if not arena.is_cuda:
            raise ValueError("arena must be a device tensor")
        arr = geos if isinstance(geos, ctypes.Array) else tx_table(geos, mode)
        if out is not None:
            # every call's 2 n_k sums, n_k = ceil(size / mss) (connect.go:675)
            total = sum(-(-int(t.size) // max(int(t.mss), 1)) for t in (arr[k] for k in range(len(geos))))
            if not out.is_cuda or out.numel() < 2 * total or out.element_size() != 2:
                raise ValueError("out must be a device tensor of 2 * sum(n_k) 16-bit sums")
        if stream is None:
            stream = torch.cuda.current_stream(arena.device)
        check(lib().ns_csum_tcp_tx_multi(self._h, arena.data_ptr(), arena.numel() * arena.element_size(), arr,
                                         len(arr) if len(geos) else 0, out.data_ptr() if out is not None else None,
                                         getattr(stream, "cuda_stream", stream)), "ns_csum_tcp_tx_multi")
        return out

    def tcp_tx_host(self, arena: np.ndarray, geos, mode: str = "full") -> np.ndarray:
        """sendTCPBatch calls over host memory (ns_csum_tcp_tx_host): `arena`
        a writable, contiguous uint8 numpy array (pageable, or a stage from
        stage_acquire) holding the calls' header slots and payloads; `geos`
        as for tcp_tx_multi.  Synchronous: the fields are written into
        `arena` in place; returns the 2 * sum(n_k) un-complemented sums."""
        arr, count, total = _tx_host_args(arena, geos, mode)
        out = np.zeros(max(2 * total, 1), dtype=np.uint16)
        check(lib().ns_csum_tcp_tx_host(self._h, _ptr(arena), arena.size, arr, count, _ptr(out)),
              "ns_csum_tcp_tx_host")
        return out[:2 * total]

    def set_tx_tuning(self, variant: int = 0, tile: int = 0, htile: int = 0, passes: int = 0) -> None:
        """ns_csum_tcp_tx's A/B and test knobs on this context
        (ns_csum_set_tx_tuning; all zero = production)."""
        check(lib().ns_csum_set_tx_tuning(self._h, variant, tile, htile, passes), "ns_csum_set_tx_tuning")

    def rx_ring(self, arena, ring: dict, lens, sums=None, verdict=None, stream=None):
        """Verify a receive ring resident in HBM (ns_csum_rx_ring): `arena` a
        uint8 CUDA tensor holding n slots of `stride` bytes from `ring_off`;
        `ring` the keys of ns_rx_ring (ring_off, stride, n, frame_at,
        link_hdr, first_view); `lens` an int32/uint32 CUDA tensor of the n
        received lengths.  `verdict` (uint8, n) and `sums` (16-bit, 2n) are
        allocated when None.  Launches on `stream` (default: torch's current
        stream) without synchronising; returns (verdict, sums)."""
        import torch

        n = int(ring["n"])
        if not (arena.is_cuda and lens.is_cuda):
            raise ValueError("arena and lens must be device tensors")
        if lens.element_size() != 4 or lens.numel() < n or not lens.is_contiguous():
            raise ValueError("lens must be a contiguous tensor of n 32-bit lengths")
        if verdict is None:
            verdict = torch.empty(max(n, 1), dtype=torch.uint8, device=arena.device)
        if sums is None:
            sums = torch.empty(max(2 * n, 1), dtype=torch.int16, device=arena.device)
        if not verdict.is_cuda or verdict.element_size() != 1 or verdict.numel() < n:
            raise ValueError("verdict must be a device tensor of n bytes")
        if not sums.is_cuda or sums.element_size() != 2 or sums.numel() < 2 * n:
            raise ValueError("sums must be a device tensor of 2n 16-bit sums")
        r = _lib.NsRxRing(int(ring.get("ring_off", 0)), int(ring["stride"]), n, int(ring.get("frame_at", 0)),
                          int(ring.get("link_hdr", 0)), int(ring.get("first_view", 0)), int(ring.get("flags", 0)))
        if stream is None:
            stream = torch.cuda.current_stream(arena.device)
        check(lib().ns_csum_rx_ring(self._h, arena.data_ptr(), arena.numel() * arena.element_size(),
                                    ctypes.byref(r), lens.data_ptr(), sums.data_ptr(), verdict.data_ptr(),
                                    getattr(stream, "cuda_stream", stream)), "ns_csum_rx_ring")
        return verdict, sums

    def rx_bufs(self, arena, ring: dict, offs, lens, sums=None, verdict=None, stream=None):
        """Verify received frames in buffers at per-packet offsets of a device
        arena (ns_csum_rx_bufs): `ring` as for rx_ring with `stride` the
        buffers' capacity; `offs` and `lens` uint32/int32 CUDA tensors of n
        offsets (from ring_off, 16-B aligned) and received lengths.  Launches
        on `stream` without synchronising; returns (verdict, sums)."""
        import torch

        n = int(ring["n"])
        if not (arena.is_cuda and lens.is_cuda and offs.is_cuda):
            raise ValueError("arena, offs and lens must be device tensors")
        for t, what in ((lens, "lens"), (offs, "offs")):
            if t.element_size() != 4 or t.numel() < n or not t.is_contiguous():
                raise ValueError(f"{what} must be a contiguous tensor of n 32-bit values")
        if verdict is None:
            verdict = torch.empty(max(n, 1), dtype=torch.uint8, device=arena.device)
        if sums is None:
            sums = torch.empty(max(2 * n, 1), dtype=torch.int16, device=arena.device)
        if not verdict.is_cuda or verdict.element_size() != 1 or verdict.numel() < n:
            raise ValueError("verdict must be a device tensor of n bytes")
        if not sums.is_cuda or sums.element_size() != 2 or sums.numel() < 2 * n:
            raise ValueError("sums must be a device tensor of 2n 16-bit sums")
        r = _lib.NsRxRing(int(ring.get("ring_off", 0)), int(ring["stride"]), n, int(ring.get("frame_at", 0)),
                          int(ring.get("link_hdr", 0)), int(ring.get("first_view", 0)), int(ring.get("flags", 0)))
        if stream is None:
            stream = torch.cuda.current_stream(arena.device)
        check(lib().ns_csum_rx_bufs(self._h, arena.data_ptr(), arena.numel() * arena.element_size(),
                                    ctypes.byref(r), offs.data_ptr(), lens.data_ptr(), sums.data_ptr(),
                                    verdict.data_ptr(), getattr(stream, "cuda_stream", stream)), "ns_csum_rx_bufs")
        return verdict, sums

    def rx_ring_host(self, arena, ring: dict, lens):
        """Verify a receive ring in HOST memory (ns_csum_rx_ring_host):
        `arena` a contiguous uint8 numpy array, `ring` as for rx_ring, `lens`
        the n received lengths (uint32).  Synchronous; returns (verdict,
        sums) as numpy arrays of n bytes and 2n u16."""
        a = _u8(arena)
        n = int(ring["n"])
        ln = np.ascontiguousarray(lens, dtype=np.uint32)
        if ln.size < n:
            raise ValueError("lens must hold n received lengths")
        verdict = np.zeros(max(n, 1), dtype=np.uint8)
        sums = np.zeros(max(2 * n, 1), dtype=np.uint16)
        r = _lib.NsRxRing(int(ring.get("ring_off", 0)), int(ring["stride"]), n, int(ring.get("frame_at", 0)),
                          int(ring.get("link_hdr", 0)), int(ring.get("first_view", 0)), int(ring.get("flags", 0)))
        check(lib().ns_csum_rx_ring_host(self._h, _ptr(a), a.size, ctypes.byref(r), _ptr(ln), _ptr(sums),
                                         _ptr(verdict)), "ns_csum_rx_ring_host")
        return verdict[:n], sums[:2 * n]

    def stream_release(self, stream) -> None:
        """Free the scratch this context keeps for `stream` (a torch.cuda.Stream
        or a raw hipStream_t) after its last launch (ns_csum_stream_release);
        call before destroying a stream that ran chained batches."""
        h = getattr(stream, "cuda_stream", stream)
        check(lib().ns_csum_stream_release(self._h, h), "ns_csum_stream_release")

    def scratch_count(self) -> int:
        """Streams currently holding device-resident scratch on this context."""
        c = ctypes.c_uint32(0)
        check(lib().ns_csum_scratch_count(self._h, ctypes.byref(c)), "ns_csum_scratch_count")
        return int(c.value)

    def stats(self, reset: bool = False) -> dict:
        """The context's diagnostic counters (ns_csum_get_stats) as a dict;
        reset=True zeroes them after reading."""
        st = _lib.NsStats()
        check(lib().ns_csum_get_stats(self._h, ctypes.byref(st), 1 if reset else 0), "ns_csum_get_stats")
        return {name: int(getattr(st, name)) for name, _ in st._fields_}

    def sync(self, stream: int | None = None) -> int:
        """Wait for `stream`; return the number of out-of-range descriptors."""
        bad = ctypes.c_uint64(0)
        check(lib().ns_csum_sync(self._h, stream, ctypes.byref(bad)), "ns_csum_sync")
        return int(bad.value)

    # -- host-memory batch ---------------------------------------------------
    def batch_host(self, arena, desc: np.ndarray, chained: bool = False) -> np.ndarray:
        a = _u8(arena)
        d = np.ascontiguousarray(desc, dtype=DESC_DTYPE)
        out = np.zeros(len(d), dtype=np.uint16)
        check(lib().ns_csum_batch_host(self._h, _ptr(a), a.size, _ptr(d), len(d), _ptr(out),
                                       _lib.NS_BATCH_CHAINED if chained else 0),
              "ns_csum_batch_host")
        return out

    # -- reference-shaped entry points --------------------------------------
    def checksum(self, buf, initial: int = 0) -> int:
        a = _u8(buf)
        r = ctypes.c_uint16(0)
        check(lib().ns_csum_checksum(self._h, _ptr(a), a.size, initial & 0xFFFF, ctypes.byref(r)),
              "ns_csum_checksum")
        return int(r.value)

    def vv_with_offset(self, views, initial: int, off: int, size: int) -> int:
        cv, keep = _views(views)
        r = ctypes.c_uint16(0)
        check(lib().ns_csum_vv_with_offset(self._h, cv, len(keep), initial & 0xFFFF, off, size,
                                           ctypes.byref(r)), "ns_csum_vv_with_offset")
        return int(r.value)

    def vv_batch(self, views, segs) -> np.ndarray:
        """segs: iterable of (off, size, initial)."""
        cv, keep = _views(views)
        segs = list(segs)
        st = (NsSeg * max(len(segs), 1))(*[NsSeg(o, s, i & 0xFFFF, 0, 0) for (o, s, i) in segs])
        out = np.zeros(len(segs), dtype=np.uint16)
        check(lib().ns_csum_vv_batch(self._h, cv, len(keep), st, len(segs),
                                     out.ctypes.data_as(ctypes.POINTER(ctypes.c_uint16))),
              "ns_csum_vv_batch")
        return out

    def views_restart(self, views, initial: int) -> int:
        cv, keep = _views(views)
        r = ctypes.c_uint16(0)
        check(lib().ns_csum_views_restart(self._h, cv, len(keep), initial & 0xFFFF, ctypes.byref(r)),
              "ns_csum_views_restart")
        return int(r.value)

    def chains(self, chains) -> np.ndarray:
        """ns_csum_chains: `chains` is a list of chains; a chain is a list of
        (bytes_like, restart: bool) pieces, optionally with the chain's initial
        as ("init", value) first.  Returns one u16 per chain (one device pass)."""
        keep, flat = [], []
        for ch in chains:
            init = 0
            items = list(ch)
            if items and isinstance(items[0], tuple) and items[0][0] == "init":
                init = items[0][1] & 0xFFFF
                items = items[1:]
            if not items:
                items = [(b"", True)]
            for k, (buf, restart) in enumerate(items):
                a = _u8(buf)
                keep.append(a)
                fl = (_lib.NS_PIECE_RESTART if restart else 0) | (_lib.NS_PIECE_END if k == len(items) - 1 else 0)
                flat.append(NsPiece(_ptr(a), a.size, init if k == 0 else 0, fl, 0))
        out = np.zeros(len(chains), dtype=np.uint16)
        arr = (NsPiece * max(len(flat), 1))(*flat)
        check(lib().ns_csum_chains(self._h, arr, len(flat),
                                   out.ctypes.data_as(ctypes.POINTER(ctypes.c_uint16)), len(chains)),
              "ns_csum_chains")
        return out

    # -- caller-filled staging (ns_csum_stage_acquire) -----------------------
    def stage_acquire(self, nbytes: int) -> np.ndarray:
        """A leased, pinned, device-mapped host buffer of >= nbytes as a
        writable numpy array.  Pointers into it passed to the gather entry
        points are read in place.  Return it with stage_release."""
        base = ctypes.c_void_p()
        check(lib().ns_csum_stage_acquire(self._h, nbytes, ctypes.byref(base)), "ns_csum_stage_acquire")
        buf = (ctypes.c_uint8 * max(nbytes, 1)).from_address(base.value)
        return np.frombuffer(buf, dtype=np.uint8)[:nbytes]

    def stage_release(self, arr: np.ndarray) -> None:
        check(lib().ns_csum_stage_release(self._h, arr.ctypes.data), "ns_csum_stage_release")

    def pseudo_header(self, protocol: int, src: bytes, dst: bytes, total_len: int) -> int:
        s, d = _u8(bytes(src)), _u8(bytes(dst))
        r = ctypes.c_uint16(0)
        check(lib().ns_csum_pseudo_header(self._h, protocol, _ptr(s), s.size, _ptr(d), d.size,
                                          total_len & 0xFFFF, ctypes.byref(r)),
              "ns_csum_pseudo_header")
        return int(r.value)


_TX_MODES = {"full": 0, "partial": _lib.NS_TX_TCP_PARTIAL, "none": _lib.NS_TX_TCP_NONE}


def tx_table(geos, mode: str = "full"):
    """The ns_tcp_tx array of a list of tcp_tx geometries (each may carry its
    own "mode"), built once and reusable across Engine.tcp_tx_multi calls."""
    arr = (_lib.NsTcpTx * max(len(geos), 1))()
    for k, geo in enumerate(geos):
        arr[k] = _lib.NsTcpTx(geo["hdr_off"], geo["pay_off"], geo["size"], geo["mss"], geo["slot"],
                              geo["ip_at"], geo["ip_len"], geo["tcp_at"], geo["tcp_len"],
                              geo["addr_sum"] if "addr_sum" in geo else addr_sum(bytes(geo["src"]), bytes(geo["dst"])),
                              geo.get("protocol", 6), _TX_MODES[geo.get("mode", mode)])
    return arr


def _tx_host_args(arena, geos, mode):
    """Checks a host arena for the host TX entry points and returns the
    ns_tcp_tx table, the call count and the calls' total segments
    (n_k = ceil(size / mss), connect.go:675; the C side refuses mss 0)."""
    if not (isinstance(arena, np.ndarray) and arena.dtype == np.uint8 and arena.flags.c_contiguous
            and arena.flags.writeable):
        raise ValueError("arena must be a writable, contiguous uint8 numpy array")
    arr = geos if isinstance(geos, ctypes.Array) else tx_table(geos, mode)
    count = len(arr) if len(geos) else 0
    t = np.ctypeslib.as_array(arr)[:count]
    total = int((-(-t["size"].astype(np.int64) // np.maximum(t["mss"], 1))).sum()) if count else 0
    return arr, count, total


@functools.lru_cache(maxsize=1024)
def addr_sum(src: bytes, dst: bytes) -> int:
    """Checksum(dst, Checksum(src, 0)) (checksum.go:113-114): the address part
    of a route's pseudo-header sum, as ns_tcp_tx.addr_sum takes it."""
    x = 0
    for a in (bytes(src), bytes(dst)):
        v = x + sum((a[i] << 8) + (a[i + 1] if i + 1 < len(a) else 0) for i in range(0, len(a), 2))
        v = (v & 0xFFFF) + (v >> 16)
        x = (v + (v >> 16)) & 0xFFFF
    return x


def combine(a: int, b: int) -> int:
    """header.ChecksumCombine (checksum.go:104-107), via the C ABI."""
    return int(lib().ns_csum_combine(a & 0xFFFF, b & 0xFFFF))


def shard_plan(desc: np.ndarray, parts: int) -> np.ndarray:
    """Byte-balanced contiguous split of a descriptor table into `parts`
    ranges (ns_csum_shard_plan); returns `parts+1` boundaries."""
    d = np.ascontiguousarray(desc, dtype=DESC_DTYPE)
    first = np.zeros(parts + 1, dtype=np.uint32)
    check(lib().ns_csum_shard_plan(_ptr(d), len(d), parts,
                                   first.ctypes.data_as(ctypes.POINTER(ctypes.c_uint32))),
          "ns_csum_shard_plan")
    return first


def batch_multi(engines, arena, desc: np.ndarray, chained: bool = False) -> np.ndarray:
    """One host batch sharded over several engines (devices) by
    ns_csum_batch_multi: byte-balanced contiguous shards, one host thread and
    one device per shard, no collective."""
    a = _u8(arena)
    d = np.ascontiguousarray(desc, dtype=DESC_DTYPE)
    out = np.zeros(len(d), dtype=np.uint16)
    hs = (ctypes.c_void_p * len(engines))(*[e._h for e in engines])
    check(lib().ns_csum_batch_multi(hs, len(engines), _ptr(a), a.size, _ptr(d), len(d), _ptr(out),
                                    _lib.NS_BATCH_CHAINED if chained else 0), "ns_csum_batch_multi")
    return out


def tcp_tx_host_multi(engines, arena: np.ndarray, geos, mode: str = "full") -> np.ndarray:
    """sendTCPBatch calls over host memory sharded over several engines
    (devices) by ns_csum_tcp_tx_host_multi: byte-balanced consecutive parts,
    one host thread and one device per part, no collective.  Fields written
    into `arena` in place; returns the 2 * sum(n_k) sums in call order."""
    arr, count, total = _tx_host_args(arena, geos, mode)
    out = np.zeros(max(2 * total, 1), dtype=np.uint16)
    hs = (ctypes.c_void_p * len(engines))(*[e._h for e in engines])
    check(lib().ns_csum_tcp_tx_host_multi(hs, len(engines), _ptr(arena), arena.size, arr, count, _ptr(out)),
          "ns_csum_tcp_tx_host_multi")
    return out[:2 * total]


_engines: dict[int, Engine] = {}
_elock = threading.Lock()


def default_engine(device: int | None = None) -> Engine:
    """Process-wide engine per device (created once), as the Go shim would
    keep one context per device behind package `header`."""
    if device is None:
        try:
            import torch

            device = torch.cuda.current_device() if torch.cuda.is_available() else 0
        except Exception:
            device = 0
    e = _engines.get(device)
    if e is None:
        with _elock:
            e = _engines.get(device)
            if e is None:
                e = Engine(device)
                _engines[device] = e
    return e
