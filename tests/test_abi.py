"""CPU: the C-ABI library loads and exports every symbol include/*.h declares;
host-only entry points (combine, strerror, shard plan) behave; no compute is
issued (there is no GPU here)."""
import ctypes
import os
import re
import subprocess

import numpy as np
import pytest

from conftest import ROOT
from netstack_amd import _lib, engine
from netstack_amd import workloads as W


def declared_symbols():
    syms = set()
    inc = os.path.join(ROOT, "include")
    for fn in os.listdir(inc):
        if fn.endswith(".h"):
            txt = open(os.path.join(inc, fn)).read()
            syms |= set(re.findall(r"\b(ns_csum_\w+)\s*\(", txt))
    return syms


def test_header_declares_the_boundary():
    syms = declared_symbols()
    for s in ("ns_csum_checksum", "ns_csum_vv_with_offset", "ns_csum_batch_dev",
              "ns_csum_batch_host", "ns_csum_pseudo_header", "ns_csum_combine"):
        assert s in syms


def test_library_exports_every_declared_symbol():
    L = _lib.lib()
    for s in declared_symbols():
        assert hasattr(L, s), s
    assert set(_lib.EXPORTED) == declared_symbols()
    out = subprocess.run(["nm", "-D", "--defined-only", _lib.LIB_PATH], capture_output=True, text=True).stdout
    for s in declared_symbols():
        assert re.search(rf"\bT {s}\b", out), f"{s} not exported with C linkage"


def test_abi_version_and_strerror():
    L = _lib.lib()
    assert L.ns_csum_abi_version() == 2
    for code in (0, -1, -2, -3, -4, -5):
        assert L.ns_csum_strerror(code)


def test_struct_layouts_match_header():
    assert ctypes.sizeof(_lib.NsPktDesc) == 16
    assert ctypes.sizeof(_lib.NsSeg) == 24
    assert engine.DESC_DTYPE.itemsize == 16
    assert W.DESC_DTYPE == engine.DESC_DTYPE


def test_combine_matches_checksum_go(oracle_mod):
    rng = np.random.default_rng(0)
    for a, b in [(0, 0), (0xFFFF, 1), (0xFFFF, 0xFFFF), (0x8000, 0x8000)] + \
            [tuple(map(int, rng.integers(0, 65536, 2))) for _ in range(500)]:
        assert engine.combine(a, b) == oracle_mod.py_combine(a, b)


def test_shard_plan_byte_balanced():
    b = W.config(4, n=10000)
    for parts in (1, 2, 3, 4, 8):
        first = engine.shard_plan(b.desc, parts)
        assert first[0] == 0 and first[-1] == b.n
        assert (np.diff(first.astype(np.int64)) >= 0).all()
        sizes = [int(b.desc["len"][first[p]:first[p + 1]].sum()) for p in range(parts)]
        assert max(sizes) - min(sizes) <= 2 * 9000


def test_shard_plan_keeps_chains_whole():
    d = np.zeros(100, dtype=engine.DESC_DTYPE)
    d["len"] = 100
    d["flags"][1::2] = engine.CONT  # pairs (head, cont)
    first = engine.shard_plan(d, 4)
    for p in first[1:-1]:
        assert not (d["flags"][p] & engine.CONT)


def test_no_device_is_reported_not_faked():
    if engine.device_count() > 0:
        pytest.skip("a GPU is present")
    with pytest.raises(_lib.ChecksumError) as ei:
        engine.Engine(0)
    assert ei.value.status == _lib.NS_ENODEV


def test_header_mirror_is_device_only():
    """The product path never imports the oracle or computes on the host."""
    pkg = os.path.join(ROOT, "netstack_amd")
    for dirpath, _, files in os.walk(pkg):
        for fn in files:
            if fn.endswith((".py", ".cpp", ".hip", ".h")):
                txt = open(os.path.join(dirpath, fn)).read()
                assert "import oracle" not in txt and "oracle_" not in txt, fn


def test_cpp_mirror_buffer_tables():
    """The C++ mirror's view_test.go tables (no GPU needed)."""
    exe = os.path.join(ROOT, "netstack_amd", "lib", "checksum_test")
    if not os.path.exists(exe):
        subprocess.run(["make", "-s", "-C", os.path.join(ROOT, "netstack_amd", "csrc")], check=True)
    r = subprocess.run([exe, "--cpu-only"], capture_output=True, text=True, timeout=60)
    assert r.returncode == 0, r.stdout + r.stderr


def test_product_kernels_never_spill_and_keep_occupancy():
    """The build keeps hipcc's kernel resource report (netstack_amd/csrc/
    Makefile).  No checksum kernel may use scratch memory: an if-chain over a
    register array once compiled to a scratch lookup and cost 45% of the
    bandwidth.  The group kernels must keep >= 6 waves per SIMD and the
    small-packet kernels 8, the windowed (arena >= 4 GiB) ones 4."""
    rep = os.path.join(ROOT, "netstack_amd", "lib", "csum_kernels.resources.txt")
    txt = open(rep).read()
    kernels = {}
    cur = None
    for line in txt.splitlines():
        m = re.search(r"Function Name: (\S+)", line)
        if m:
            cur = m.group(1)
            kernels[cur] = {}
            continue
        m = re.search(r"(ScratchSize \[bytes/lane\]|Occupancy \[waves/SIMD\]|VGPRs): (\d+)", line)
        if m and cur:
            kernels[cur][m.group(1).split()[0]] = int(m.group(2))
    hyb = {k: v for k, v in kernels.items() if "csum_hyb" in k}
    assert len(hyb) >= 18, sorted(kernels)
    for k, v in kernels.items():
        assert v["ScratchSize"] == 0, (k, v)
    for k, v in hyb.items():
        small = "ILi256ELi256ELi16ELi8ELi4ELi2ELi5E" in k
        windowed = "Li5ELb1E" in k or "Li0ELb1E" in k  # WIN = true: carries the 64-bit-address fallback too
        chained = "Lb1EEEv" in k  # CH = true (the last template argument)
        assert v["Occupancy"] >= (8 if small else 4 if (windowed or chained) else 6), (k, v)
    assert any("Lb1EEEv" in k for k in hyb) and any("Lb0EEEv" in k for k in hyb), sorted(hyb)
    for k, v in kernels.items():  # the huge-descriptor kernel runs the same scan
        if "csum_split" in k:
            assert v["Occupancy"] >= 6, (k, v)


def test_go_shim_keeps_reference_signatures_and_binds_declared_symbols():
    """No Go toolchain here, so the cgo shim (go/header/checksum_hip.go) is
    checked statically: it declares netstack's exported checksum functions
    with the reference's exact signatures (tcpip/header/checksum.go:52, 61,
    69, 104, 112) and calls only functions include/netstack_csum.h declares."""
    src = open(os.path.join(ROOT, "go", "header", "checksum_hip.go")).read()
    for sig in (
        "func Checksum(buf []byte, initial uint16) uint16",
        "func ChecksumVV(vv buffer.VectorisedView, initial uint16) uint16",
        "func ChecksumVVWithOffset(vv buffer.VectorisedView, initial uint16, off int, size int) uint16",
        "func ChecksumCombine(a, b uint16) uint16",
        "func PseudoHeaderChecksum(protocol tcpip.TransportProtocolNumber, srcAddr tcpip.Address, "
        "dstAddr tcpip.Address, totalLen uint16) uint16",
    ):
        assert sig in src, sig
    assert "// +build hipcsum" in src and "package header" in src
    called = set(re.findall(r"C\.(ns_csum_\w+)\(", src))
    assert called and called <= declared_symbols(), called - declared_symbols()
