"""ORACLE — TEST INFRASTRUCTURE ONLY.  Not part of the product.

Two restatements of google/netstack's RFC 1071 checksum
(``tcpip/header/checksum.go``), used as the parity checker:

* ``py_*`` — pure-Python loops that follow checksum.go line by line (small
  inputs only; used to generate and to cross-check ``tests/golden``).
* ``C`` — ctypes binding of ``oracle/csum_oracle.c`` (built by
  ``oracle/Makefile`` into ``oracle/liboracle_csum.so``), fast enough for the
  full BASELINE.json sizes and timed as bench.py's ``cpu_baseline``.

Only ``tests/``, ``__graft_entry__.smoke()`` and bench.py's cpu_baseline leg
may import this module.  The product (``netstack_amd``) never does.

Parity pin: the reference cannot run here (Go, no toolchain), so both
restatements are pinned by the six known-answer tests of
``tcpip/header/checksum_test.go:34-94`` and public RFC 1071 vectors
(``tests/golden/kat.json``); see DESIGN.md §Oracle.
"""
from __future__ import annotations

import ctypes
import os
import subprocess

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(_HERE, "liboracle_csum.so")

DESC_DTYPE = np.dtype(
    [("off", "<u8"), ("len", "<u4"), ("initial", "<u2"), ("flags", "<u2")], align=False
)
assert DESC_DTYPE.itemsize == 16

ODD = 0x1
CONT = 0x2


# --------------------------------------------------------------------------
# pure-Python restatement (checksum.go line by line)
# --------------------------------------------------------------------------
def py_combine(a: int, b: int) -> int:
    """checksum.go:104-107."""
    v = (a & 0xFFFF) + (b & 0xFFFF)
    return (v + (v >> 16)) & 0xFFFF


def py_calculate_checksum(buf: bytes, odd: bool, initial: int) -> tuple[int, bool]:
    """checksum.go:26-46 — uint32 accumulator, wraps mod 2^32, no inner fold."""
    v = initial & 0xFFFFFFFF
    if odd:  # :29-32
        v = (v + buf[0]) & 0xFFFFFFFF
        buf = buf[1:]
    l = len(buf)
    odd = (l & 1) != 0  # :34-39
    if odd:
        l -= 1
        v = (v + (buf[l] << 8)) & 0xFFFFFFFF
    for i in range(0, l, 2):  # :41-43
        v = (v + (buf[i] << 8) + buf[i + 1]) & 0xFFFFFFFF
    return py_combine(v & 0xFFFF, v >> 16), odd  # :45


def py_checksum(buf: bytes, initial: int = 0) -> int:
    """checksum.go:52-55."""
    return py_calculate_checksum(bytes(buf), False, initial)[0]


def py_checksum_vv_with_offset(views, initial: int, off: int, size: int) -> int:
    """checksum.go:69-98 over a list of byte strings (the VV's views)."""
    if off < 0 or size < 0:
        raise ValueError("negative slice bound (Go panics)")
    odd = False
    s = initial
    for v in views:
        v = bytes(v)
        if len(v) == 0:
            continue
        if off >= len(v):
            off -= len(v)
            continue
        v = v[off:]
        l = min(len(v), size)
        v = v[:l]
        s, odd = py_calculate_checksum(v, odd, s)
        size -= len(v)
        if size == 0:
            break
        off = 0
    return s


def py_checksum_vv(views, initial: int) -> int:
    """checksum.go:61-63 (size = Σ view lengths when no CapLength was applied)."""
    return py_checksum_vv_with_offset(views, initial, 0, sum(len(v) for v in views))


def py_views_restart(views, initial: int) -> int:
    """udp/endpoint.go:811-813: xsum = Checksum(v, xsum) for each view."""
    x = initial
    for v in views:
        x = py_checksum(v, x)
    return x


def py_pseudo_header(protocol: int, src: bytes, dst: bytes, total_len: int) -> int:
    """checksum.go:112-122."""
    x = py_checksum(src, 0)
    x = py_checksum(dst, x)
    x = py_checksum(bytes([(total_len >> 8) & 0xFF, total_len & 0xFF]), x)
    return py_checksum(bytes([0, protocol & 0xFF]), x)


def py_batch(arena: bytes, desc: np.ndarray, chained: bool = False) -> np.ndarray:
    """The ns_pkt_desc batch contract (include/netstack_csum.h) over
    calculateChecksum; small inputs only."""
    out = np.zeros(len(desc), dtype=np.uint16)
    prev = 0
    for i, d in enumerate(desc):
        init = prev if (chained and (int(d["flags"]) & CONT)) else int(d["initial"])
        o, l = int(d["off"]), int(d["len"])
        if o > len(arena) or l > len(arena) - o:
            l = 0
        piece = arena[o : o + l]
        prev = py_calculate_checksum(piece, bool(int(d["flags"]) & ODD) and l > 0, init)[0]
        out[i] = prev
    return out


STORE = 0x4
STORE_RAW = 0x8
STORE_SHIFT = 4


def apply_stores(arena: np.ndarray, desc: np.ndarray, results: np.ndarray) -> tuple[np.ndarray, int]:
    """The NS_DESC_STORE contract of ns_csum_batch_dev_store: every sum is
    taken over the arena as it was before the call (`results` = py_batch /
    c_batch of it), then each flagged descriptor writes its result r
    big-endian at off + (flags >> 4): ^r, as header SetChecksum(^xsum)
    (ipv4.go:223 via ipv4.go:236; tcp.go:252 via connect.go:663), or r itself
    with STORE_RAW (the CHECKSUM_PARTIAL pseudo-header sum, connect.go:660).
    A store whose 2 bytes leave the arena is dropped and counted.
    Returns (new arena copy, dropped stores)."""
    a = np.array(arena, dtype=np.uint8, copy=True)
    dropped = 0
    for i in np.flatnonzero(desc["flags"] & STORE):
        f = int(desc["flags"][i])
        at = int(desc["off"][i]) + (f >> STORE_SHIFT)
        if at + 2 > len(a):
            dropped += 1
            continue
        r = int(results[i])
        v = r if f & STORE_RAW else (~r & 0xFFFF)
        a[at] = v >> 8
        a[at + 1] = v & 0xFF
    return a, dropped


# --------------------------------------------------------------------------
# C restatement (oracle/csum_oracle.c)
# --------------------------------------------------------------------------
def build(force: bool = False) -> str:
    """Compile oracle/csum_oracle.c (make) if the .so is missing."""
    if force or not os.path.exists(LIB_PATH):
        subprocess.run(["make", "-s", "-C", _HERE], check=True)
    return LIB_PATH


class _C:
    _lib = None

    @classmethod
    def lib(cls):
        if cls._lib is None:
            if not os.path.exists(LIB_PATH):
                build()
            lib = ctypes.CDLL(LIB_PATH)
            u8p = ctypes.c_void_p
            lib.oracle_combine.restype = ctypes.c_uint16
            lib.oracle_combine.argtypes = [ctypes.c_uint16, ctypes.c_uint16]
            lib.oracle_checksum.restype = ctypes.c_uint16
            lib.oracle_checksum.argtypes = [u8p, ctypes.c_uint64, ctypes.c_uint16]
            lib.oracle_calculate_checksum.restype = ctypes.c_uint16
            lib.oracle_calculate_checksum.argtypes = [
                u8p, ctypes.c_uint64, ctypes.c_int, ctypes.c_uint32, ctypes.POINTER(ctypes.c_int)]
            lib.oracle_vv_with_offset.restype = ctypes.c_int
            lib.oracle_vv_with_offset.argtypes = [
                ctypes.POINTER(ctypes.c_void_p), ctypes.POINTER(ctypes.c_uint64), ctypes.c_uint32,
                ctypes.c_uint16, ctypes.c_int64, ctypes.c_int64, ctypes.POINTER(ctypes.c_uint16)]
            lib.oracle_views_restart.restype = ctypes.c_uint16
            lib.oracle_views_restart.argtypes = [
                ctypes.POINTER(ctypes.c_void_p), ctypes.POINTER(ctypes.c_uint64), ctypes.c_uint32,
                ctypes.c_uint16]
            lib.oracle_pseudo_header.restype = ctypes.c_uint16
            lib.oracle_pseudo_header.argtypes = [
                ctypes.c_uint32, u8p, ctypes.c_uint32, u8p, ctypes.c_uint32, ctypes.c_uint16]
            lib.oracle_batch.restype = ctypes.c_int
            lib.oracle_batch.argtypes = [u8p, ctypes.c_uint64, u8p, ctypes.c_uint32, u8p, ctypes.c_int]
            lib.oracle_batch_mt.restype = ctypes.c_int
            lib.oracle_batch_mt.argtypes = [u8p, u8p, ctypes.c_uint32, u8p, ctypes.c_int]
            u64, u32 = ctypes.c_uint64, ctypes.c_uint32
            lib.oracle_send_tcp_batch.restype = u64
            lib.oracle_send_tcp_batch.argtypes = [u8p, u64, u64, u64, u32, u32, u32, u32, u32, u32, u32,
                                                  u8p, u32, u8p, u32, ctypes.c_int, u8p]
            lib.oracle_rx_ring.restype = ctypes.c_int
            lib.oracle_rx_ring.argtypes = [u8p, u64, u32, u8p, u32, u32, u32, u8p, u8p, ctypes.c_int]
            cls._lib = lib
        return cls._lib


def _ptr(a: np.ndarray) -> int:
    return a.ctypes.data


def c_checksum(buf, initial: int = 0) -> int:
    a = np.frombuffer(bytes(buf), dtype=np.uint8) if not isinstance(buf, np.ndarray) else buf
    a = np.ascontiguousarray(a, dtype=np.uint8)
    return int(_C.lib().oracle_checksum(_ptr(a) if a.size else None, a.size, initial))


def c_calculate_checksum(buf, odd: bool, initial: int) -> tuple[int, bool]:
    a = np.ascontiguousarray(np.frombuffer(bytes(buf), dtype=np.uint8))
    o = ctypes.c_int(0)
    r = _C.lib().oracle_calculate_checksum(_ptr(a) if a.size else None, a.size, int(odd), initial, ctypes.byref(o))
    return int(r), bool(o.value)


def c_combine(a: int, b: int) -> int:
    return int(_C.lib().oracle_combine(a, b))


def _views_args(views):
    arrs = [np.ascontiguousarray(np.frombuffer(bytes(v), dtype=np.uint8)) for v in views]
    n = len(arrs)
    ptrs = (ctypes.c_void_p * max(n, 1))(*[(_ptr(a) if a.size else None) for a in arrs])
    lens = (ctypes.c_uint64 * max(n, 1))(*[a.size for a in arrs])
    return arrs, ptrs, lens, n


def c_checksum_vv_with_offset(views, initial: int, off: int, size: int) -> int:
    arrs, ptrs, lens, n = _views_args(views)
    out = ctypes.c_uint16(0)
    rc = _C.lib().oracle_vv_with_offset(ptrs, lens, n, initial, off, size, ctypes.byref(out))
    if rc != 0:
        raise ValueError("negative slice bound (Go panics)")
    del arrs
    return int(out.value)


def c_views_restart(views, initial: int) -> int:
    arrs, ptrs, lens, n = _views_args(views)
    r = int(_C.lib().oracle_views_restart(ptrs, lens, n, initial))
    del arrs
    return r


def c_pseudo_header(protocol: int, src: bytes, dst: bytes, total_len: int) -> int:
    s = np.frombuffer(bytes(src) or b"\0", dtype=np.uint8)
    d = np.frombuffer(bytes(dst) or b"\0", dtype=np.uint8)
    return int(_C.lib().oracle_pseudo_header(protocol, _ptr(s), len(src), _ptr(d), len(dst), total_len))


def c_batch(arena: np.ndarray, desc: np.ndarray, chained: bool = False) -> tuple[np.ndarray, int]:
    """Returns (results, number of out-of-range descriptors)."""
    arena = np.ascontiguousarray(arena, dtype=np.uint8)
    desc = np.ascontiguousarray(desc, dtype=DESC_DTYPE)
    out = np.zeros(len(desc), dtype=np.uint16)
    bad = _C.lib().oracle_batch(_ptr(arena) if arena.size else None, arena.size,
                                _ptr(desc) if desc.size else None, len(desc),
                                _ptr(out) if out.size else None, int(chained))
    return out, int(bad)


def c_batch_paired(arena: np.ndarray, desc: np.ndarray) -> tuple[np.ndarray, int]:
    """NS_BATCH_PAIRED (include/netstack_csum.h): runs of at most two.  An
    odd-indexed NS_DESC_CONT descriptor continues the one before it (Go's
    `xsum = Checksum(v, xsum)` chaining, checksum.go:89); a CONT flag on an
    even-indexed one is ignored.  That is the chained semantics on the table
    with its even-indexed CONT bits cleared."""
    d = np.array(desc, dtype=DESC_DTYPE, copy=True)
    d["flags"][0::2] &= ~np.uint16(CONT)
    return c_batch(arena, d, chained=True)


def c_send_tcp_batch(arena: np.ndarray, hdr_off: int, pay_off: int, size: int, mss: int, slot: int,
                     ip_at: int, ip_len: int, tcp_at: int, tcp_len: int, src: bytes, dst: bytes,
                     protocol: int = 6, mode: str = "full", copy: bool = True) -> tuple[np.ndarray, np.ndarray]:
    """sendTCPBatch's checksum steps (transport/tcp/connect.go:668-702 with
    buildTCPHdr :634-666, then addIPHeader network/ipv4/ipv4.go:217-238 per
    segment) over its header slots and payload view in `arena`, restated in C
    (oracle_send_tcp_batch).  mode: "full", "partial" (CHECKSUM_PARTIAL) or
    "none" (TX checksum offload).  Returns (the arena with the fields
    written, the 2n un-complemented sums [IPv4, TCP] per segment).  copy=False
    writes into `arena` itself (a contiguous uint8 array)."""
    if copy:
        a = np.array(arena, dtype=np.uint8, copy=True)
    else:
        assert arena.dtype == np.uint8 and arena.flags["C_CONTIGUOUS"]
        a = arena
    n = (size + mss - 1) // mss
    out = np.zeros(2 * max(n, 1), dtype=np.uint16)
    s = np.frombuffer(bytes(src) or b"\0", dtype=np.uint8)
    d = np.frombuffer(bytes(dst) or b"\0", dtype=np.uint8)
    L = _C.lib()
    L.oracle_send_tcp_batch(_ptr(a), hdr_off, pay_off, size, mss, slot, ip_at, ip_len, tcp_at, tcp_len,
                            protocol, _ptr(s), len(src), _ptr(d), len(dst),
                            {"full": 0, "partial": 1, "none": 2}[mode], _ptr(out))
    return a, out[:2 * n]


def c_rx_ring(arena: np.ndarray, lens: np.ndarray, stride: int, n: int, ring_off: int = 0, frame_at: int = 0,
              link_hdr: int = 0, first_view: int = 0, nthreads: int = 1) -> tuple[np.ndarray, np.ndarray]:
    """The receive path of n recvmmsg slots (oracle_rx_ring, the C
    restatement of oracle/packets.py verify_frame): (verdicts, 2n sums)."""
    assert arena.dtype == np.uint8 and arena.flags["C_CONTIGUOUS"]
    assert ring_off + n * stride <= arena.size
    ln = np.ascontiguousarray(lens[:n], dtype=np.uint32)
    verdict = np.zeros(max(n, 1), dtype=np.uint8)
    sums = np.zeros(2 * max(n, 1), dtype=np.uint16)
    _C.lib().oracle_rx_ring(_ptr(arena) + ring_off, stride, n, _ptr(ln), frame_at, link_hdr, first_view,
                            _ptr(verdict), _ptr(sums), int(nthreads))
    return verdict[:n], sums[:2 * n]


def c_batch_mt(arena: np.ndarray, desc: np.ndarray, nthreads: int, out: np.ndarray | None = None) -> np.ndarray:
    """Packet-parallel scalar port over `nthreads` pthreads (independent
    descriptors only).  This is the timed CPU baseline."""
    desc = np.ascontiguousarray(desc, dtype=DESC_DTYPE)
    if out is None:
        out = np.zeros(len(desc), dtype=np.uint16)
    _C.lib().oracle_batch_mt(_ptr(arena), _ptr(desc), len(desc), _ptr(out), int(nthreads))
    return out
