"""netstack_amd — MI355X-native (gfx950) Internet-checksum engine for
google/netstack's tcpip/header checksum hot path.

Layers:
  include/netstack_csum.h            C ABI (the drop-in boundary a cgo shim binds)
  netstack_amd/csrc/*.hip, *.cpp     HIP kernels + C-ABI implementation
  netstack_amd/engine.py             ctypes handle on one device context
  netstack_amd/buffer.py             mirror of tcpip/buffer (View, VectorisedView)
  netstack_amd/header.py             mirror of tcpip/header checksum functions
  netstack_amd/workloads.py          synthetic packet batches of BASELINE.json
"""
from ._lib import ChecksumError, NativeLibraryError  # noqa: F401
from .engine import DESC_DTYPE, Engine, default_engine, device_count, shard_plan  # noqa: F401

__all__ = ["Engine", "default_engine", "device_count", "shard_plan", "DESC_DTYPE",
           "ChecksumError", "NativeLibraryError"]
