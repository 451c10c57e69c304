"""ctypes binding of the C ABI in include/netstack_csum.h.

The library is netstack_amd/lib/libnetstack_csum.so, built in-tree by
``netstack_amd/csrc/Makefile`` (``__graft_entry__.build()``).  There is no
fallback: if the library is missing or cannot be loaded, every entry point
raises ``NativeLibraryError``.
"""
from __future__ import annotations

import ctypes
import os
import threading

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(_HERE, "lib", "libnetstack_csum.so")
CSRC = os.path.join(_HERE, "csrc")

# The NS_CSUM_ABI_VERSION this binding is written against; lib() refuses a
# library that reports another (a stale build).
ABI_VERSION = 9

NS_OK = 0
NS_EINVAL = -1
NS_ERANGE = -2
NS_ENODEV = -3
NS_ENOMEM = -4
NS_EHIP = -5

NS_DESC_ODD = 0x1
NS_DESC_CONT = 0x2
NS_DESC_STORE = 0x4
NS_DESC_STORE_RAW = 0x8
NS_DESC_STORE_SHIFT = 4
NS_BATCH_CHAINED = 0x1
NS_BATCH_PAIRED = 0x2
NS_OPT_FOLD_WALK = 0x1

# Every symbol include/netstack_csum.h declares (checked by the CPU tests).
EXPORTED = (
    "ns_csum_abi_version", "ns_csum_last_hip_error", "ns_csum_strerror", "ns_csum_device_count",
    "ns_csum_init", "ns_csum_destroy", "ns_csum_sync", "ns_csum_batch_dev", "ns_csum_batch_dev_store",
    "ns_csum_batch_host", "ns_csum_checksum", "ns_csum_vv_with_offset",
    "ns_csum_vv_batch", "ns_csum_views_restart", "ns_csum_pseudo_header",
    "ns_csum_combine", "ns_csum_shard_plan", "ns_csum_batch_multi", "ns_csum_chains",
    "ns_csum_stage_acquire", "ns_csum_stage_release", "ns_csum_packet_buffers",
    "ns_csum_stream_release", "ns_csum_scratch_count", "ns_csum_get_stats", "ns_csum_tcp_tx",
    "ns_csum_tcp_tx_multi", "ns_csum_rx_ring", "ns_csum_set_tx_tuning", "ns_csum_tcp_tx_host",
    "ns_csum_tcp_tx_host_multi", "ns_csum_rx_ring_host", "ns_csum_rx_bufs",
)
NS_PIECE_RESTART = 0x1
NS_PIECE_END = 0x2
NS_PKB_VERIFY = 1
NS_PKB_FILL = 2
NS_PKB_INVALID = 0
NS_PKB_VALID = 1
NS_PKB_UNCHECKED = 2
NS_PKB_MALFORMED = 3


class NativeLibraryError(RuntimeError):
    """The HIP engine library is missing or failed to load."""


class ChecksumError(RuntimeError):
    """A C-ABI call returned a negative status."""

    def __init__(self, status: int, what: str):
        self.status = status
        try:
            self.hip_error = int(lib().ns_csum_last_hip_error())
        except Exception:
            self.hip_error = None
        super().__init__(f"{what}: {strerror(status)} ({status}, hipError {self.hip_error})")


class NsPktDesc(ctypes.Structure):
    _fields_ = [("off", ctypes.c_uint64), ("len", ctypes.c_uint32),
                ("initial", ctypes.c_uint16), ("flags", ctypes.c_uint16)]


class NsView(ctypes.Structure):
    _fields_ = [("data", ctypes.c_void_p), ("len", ctypes.c_uint64)]


class NsSeg(ctypes.Structure):
    _fields_ = [("off", ctypes.c_int64), ("size", ctypes.c_int64),
                ("initial", ctypes.c_uint16), ("pad0", ctypes.c_uint16),
                ("pad1", ctypes.c_uint32)]


class NsPiece(ctypes.Structure):
    _fields_ = [("data", ctypes.c_void_p), ("len", ctypes.c_uint64), ("initial", ctypes.c_uint16),
                ("flags", ctypes.c_uint16), ("pad", ctypes.c_uint32)]


class NsPktBuf(ctypes.Structure):
    _fields_ = [("hdr", ctypes.c_void_p), ("hdr_len", ctypes.c_uint64), ("data", ctypes.c_void_p),
                ("ndata", ctypes.c_uint32), ("flags", ctypes.c_uint32), ("data_size", ctypes.c_uint64)]


class NsStats(ctypes.Structure):
    """ns_csum_stats: where a context's host time went (diagnostics)."""
    _fields_ = [(f, ctypes.c_uint64) for f in (
        "calls", "call_ns_max", "lock_ns_max", "zc_passes", "zc_late", "zc_pass_ns_max",
        "growths", "growth_ns_total", "growth_ns_max", "retires", "retire_ns_max",
        "stage_allocs", "stage_alloc_ns_max")]


class NsTcpTx(ctypes.Structure):
    """ns_tcp_tx: one sendTCPBatch batch's geometry (ns_csum_tcp_tx)."""
    _fields_ = [("hdr_off", ctypes.c_uint64), ("pay_off", ctypes.c_uint64), ("size", ctypes.c_uint64),
                ("mss", ctypes.c_uint32), ("slot", ctypes.c_uint32),
                ("ip_at", ctypes.c_uint16), ("ip_len", ctypes.c_uint16),
                ("tcp_at", ctypes.c_uint16), ("tcp_len", ctypes.c_uint16),
                ("addr_sum", ctypes.c_uint16), ("protocol", ctypes.c_uint16), ("flags", ctypes.c_uint32)]


class NsRxRing(ctypes.Structure):
    """ns_rx_ring: a receive ring of fixed-stride slots (ns_csum_rx_ring)."""
    _fields_ = [("ring_off", ctypes.c_uint64), ("stride", ctypes.c_uint64), ("n", ctypes.c_uint32),
                ("frame_at", ctypes.c_uint16), ("link_hdr", ctypes.c_uint16),
                ("first_view", ctypes.c_uint32), ("flags", ctypes.c_uint32)]


NS_TX_TCP_PARTIAL = 0x1
NS_TX_TCP_NONE = 0x2
NS_TX_FIELDS_ONLY = 0x4


class NsOpts(ctypes.Structure):
    _fields_ = [("device", ctypes.c_int32), ("flags", ctypes.c_uint32),
                ("staging_bytes", ctypes.c_uint64)]


assert ctypes.sizeof(NsPktDesc) == 16 and ctypes.sizeof(NsSeg) == 24 and ctypes.sizeof(NsPiece) == 24
assert ctypes.sizeof(NsPktBuf) == 40 and ctypes.sizeof(NsStats) == 13 * 8 and ctypes.sizeof(NsTcpTx) == 48
assert ctypes.sizeof(NsRxRing) == 32

_lock = threading.Lock()
_lib = None


def _declare(lib):
    c = ctypes
    vp, u8p = c.c_void_p, c.c_void_p
    u16p = c.POINTER(c.c_uint16)
    sig = {
        "ns_csum_abi_version": (c.c_int, []),
        "ns_csum_last_hip_error": (c.c_int, []),
        "ns_csum_strerror": (c.c_char_p, [c.c_int]),
        "ns_csum_device_count": (c.c_int, [c.POINTER(c.c_int)]),
        "ns_csum_init": (c.c_int, [c.POINTER(NsOpts), c.POINTER(vp)]),
        "ns_csum_destroy": (None, [vp]),
        "ns_csum_sync": (c.c_int, [vp, vp, c.POINTER(c.c_uint64)]),
        "ns_csum_batch_dev": (c.c_int, [vp, u8p, c.c_uint64, vp, c.c_uint32, vp, c.c_uint32, vp]),
        "ns_csum_batch_dev_store": (c.c_int, [vp, u8p, c.c_uint64, vp, c.c_uint32, vp, c.c_uint32, vp]),
        "ns_csum_batch_host": (c.c_int, [vp, u8p, c.c_uint64, vp, c.c_uint32, vp, c.c_uint32]),
        "ns_csum_checksum": (c.c_int, [vp, u8p, c.c_uint64, c.c_uint16, u16p]),
        "ns_csum_vv_with_offset": (c.c_int, [vp, c.POINTER(NsView), c.c_uint32, c.c_uint16,
                                             c.c_int64, c.c_int64, u16p]),
        "ns_csum_vv_batch": (c.c_int, [vp, c.POINTER(NsView), c.c_uint32, c.POINTER(NsSeg),
                                       c.c_uint32, u16p]),
        "ns_csum_views_restart": (c.c_int, [vp, c.POINTER(NsView), c.c_uint32, c.c_uint16, u16p]),
        "ns_csum_pseudo_header": (c.c_int, [vp, c.c_uint32, u8p, c.c_uint32, u8p, c.c_uint32,
                                            c.c_uint16, u16p]),
        "ns_csum_combine": (c.c_uint16, [c.c_uint16, c.c_uint16]),
        "ns_csum_shard_plan": (c.c_int, [vp, c.c_uint32, c.c_uint32, c.POINTER(c.c_uint32)]),
        "ns_csum_chains": (c.c_int, [vp, c.POINTER(NsPiece), c.c_uint32, u16p, c.c_uint32]),
        "ns_csum_batch_multi": (c.c_int, [c.POINTER(vp), c.c_uint32, u8p, c.c_uint64, vp, c.c_uint32,
                                          vp, c.c_uint32]),
        "ns_csum_stage_acquire": (c.c_int, [vp, c.c_uint64, c.POINTER(vp)]),
        "ns_csum_stage_release": (c.c_int, [vp, vp]),
        "ns_csum_packet_buffers": (c.c_int, [vp, c.POINTER(NsPktBuf), c.c_uint32, c.c_uint32, u16p,
                                             c.POINTER(c.c_uint8)]),
        "ns_csum_stream_release": (c.c_int, [vp, vp]),
        "ns_csum_scratch_count": (c.c_int, [vp, c.POINTER(c.c_uint32)]),
        "ns_csum_get_stats": (c.c_int, [vp, c.POINTER(NsStats), c.c_int]),
        "ns_csum_tcp_tx": (c.c_int, [vp, u8p, c.c_uint64, c.POINTER(NsTcpTx), vp, vp]),
        "ns_csum_tcp_tx_multi": (c.c_int, [vp, u8p, c.c_uint64, c.POINTER(NsTcpTx), c.c_uint32, vp, vp]),
        "ns_csum_rx_ring": (c.c_int, [vp, u8p, c.c_uint64, c.POINTER(NsRxRing), vp, vp, vp, vp]),
        "ns_csum_rx_ring_host": (c.c_int, [vp, u8p, c.c_uint64, c.POINTER(NsRxRing), vp, vp, vp]),
        "ns_csum_rx_bufs": (c.c_int, [vp, u8p, c.c_uint64, c.POINTER(NsRxRing), vp, vp, vp, vp, vp]),
        "ns_csum_set_tx_tuning": (c.c_int, [vp, c.c_uint32, c.c_uint32, c.c_uint32, c.c_uint32]),
        "ns_csum_tcp_tx_host": (c.c_int, [vp, u8p, c.c_uint64, c.POINTER(NsTcpTx), c.c_uint32, vp]),
        "ns_csum_tcp_tx_host_multi": (c.c_int, [c.POINTER(vp), c.c_uint32, u8p, c.c_uint64, c.POINTER(NsTcpTx),
                                                c.c_uint32, vp]),
    }
    for name, (res, args) in sig.items():
        fn = getattr(lib, name)
        fn.restype = res
        fn.argtypes = args


def lib():
    """Load (once) and return the HIP engine library; raise if unavailable."""
    global _lib
    if _lib is not None:
        return _lib
    with _lock:
        if _lib is None:
            if not os.path.exists(LIB_PATH):
                raise NativeLibraryError(
                    f"{LIB_PATH} is missing: build it with `make -C {CSRC}` "
                    "(or __graft_entry__.build()); there is no CPU fallback")
            # Share one HIP runtime with torch when torch is present: importing
            # torch first makes the loader reuse its libamdhip64.so.7.
            try:
                import torch  # noqa: F401
            except Exception:  # pragma: no cover - torch is optional here
                pass
            try:
                l = ctypes.CDLL(LIB_PATH, mode=ctypes.RTLD_GLOBAL)
            except OSError as e:
                raise NativeLibraryError(f"cannot load {LIB_PATH}: {e}") from e
            try:
                ver_fn = l.ns_csum_abi_version
            except AttributeError as e:
                raise NativeLibraryError(f"{LIB_PATH} exports no ns_csum_abi_version") from e
            ver_fn.restype = ctypes.c_int
            ver_fn.argtypes = []
            ver = int(ver_fn())
            if ver != ABI_VERSION:
                raise NativeLibraryError(
                    f"{LIB_PATH} has C ABI version {ver}, this binding needs {ABI_VERSION}: "
                    f"rebuild it with `make -C {CSRC}`")
            _declare(l)
            _lib = l
    return _lib


def strerror(status: int) -> str:
    try:
        return lib().ns_csum_strerror(status).decode()
    except NativeLibraryError:
        return f"status {status}"


def check(status: int, what: str) -> None:
    if status != NS_OK:
        if status == NS_EINVAL:
            raise ValueError(f"{what}: {strerror(status)}")
        raise ChecksumError(status, what)
