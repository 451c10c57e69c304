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
    assert L.ns_csum_abi_version() == _lib.ABI_VERSION == 9
    for code in (0, -1, -2, -3, -4, -5):
        assert L.ns_csum_strerror(code)


def test_struct_layouts_match_header():
    assert ctypes.sizeof(_lib.NsPktDesc) == 16
    assert ctypes.sizeof(_lib.NsSeg) == 24
    assert ctypes.sizeof(_lib.NsPktBuf) == 40 and _lib.NsPktBuf.data_size.offset == 32
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
        small = "ILi64ELi64ELi16ELi8ELi4ELi2ELi5E" in k
        windowed = "Li5ELb1E" in k or "Li0ELb1E" in k  # WIN = true: carries the 64-bit-address fallback too
        chained = "Lb1EEEv" in k  # CH = true (the last template argument)
        assert v["Occupancy"] >= (8 if small else 4 if (windowed or chained) else 6), (k, v)
    assert any("Lb1EEEv" in k for k in hyb) and any("Lb0EEEv" in k for k in hyb), sorted(hyb)
    for k, v in kernels.items():  # the huge-descriptor kernel runs the same scan
        if "csum_split" in k:
            assert v["Occupancy"] >= 6, (k, v)
    # the structured TX kernels (tcp_tx.hip): no scratch; the payload-reading
    # passes keep 6 waves per SIMD, the header pass 8
    tx = {}
    cur = None
    for line in open(os.path.join(ROOT, "netstack_amd", "lib", "tcp_tx.resources.txt")).read().splitlines():
        m = re.search(r"Function Name: (\S+)", line)
        if m:
            cur = m.group(1)
            tx[cur] = {}
            continue
        m = re.search(r"(ScratchSize \[bytes/lane\]|Occupancy \[waves/SIMD\]|VGPRs): (\d+)", line)
        if m and cur:
            tx[cur][m.group(1).split()[0]] = int(m.group(2))
    assert len(tx) >= 5 and all("tcp_tx" in k for k in tx), sorted(tx)
    for k, v in tx.items():
        assert v["ScratchSize"] == 0, (k, v)
        assert v["Occupancy"] >= (8 if k.endswith("Li2EEEvNS_5TxGeoE") else 6), (k, v)


    # the receive-ring kernels (rx_ring.hip): no scratch; the product's
    # MTU instance (13 lines per batch, ring and buffer list) keeps 5 waves
    rx = {}
    cur = None
    for line in open(os.path.join(ROOT, "netstack_amd", "lib", "rx_ring.resources.txt")).read().splitlines():
        m = re.search(r"Function Name: (\S+)", line)
        if m:
            cur = m.group(1)
            rx[cur] = {}
            continue
        m = re.search(r"(ScratchSize \[bytes/lane\]|Occupancy \[waves/SIMD\]|VGPRs): (\d+)", line)
        if m and cur:
            rx[cur][m.group(1).split()[0]] = int(m.group(2))
    assert len(rx) >= 10 and all("rx_ring" in k for k in rx), sorted(rx)
    for k, v in rx.items():
        assert v["ScratchSize"] == 0, (k, v)
        if "rx_ringILi13E" in k:
            assert v["Occupancy"] >= 5, (k, v)


def test_host_and_list_entry_points_check_arguments_before_the_device():
    """The round-5 entry points refuse bad arguments with NS_EINVAL before
    touching a device (so this runs on a CPU-only host)."""
    import ctypes

    L = _lib.lib()
    t = (_lib.NsTcpTx * 1)()
    r = _lib.NsRxRing(0, 1504, 1, 0, 0, 0, 0)
    buf = (ctypes.c_uint8 * 4096)()
    u32 = (ctypes.c_uint32 * 4)()
    u16 = (ctypes.c_uint16 * 8)()
    assert L.ns_csum_tcp_tx_host(None, buf, 4096, t, 1, None) == _lib.NS_EINVAL
    assert L.ns_csum_tcp_tx_host_multi(None, 1, buf, 4096, t, 1, None) == _lib.NS_EINVAL
    hs = (ctypes.c_void_p * 1)(None)
    assert L.ns_csum_tcp_tx_host_multi(hs, 0, buf, 4096, t, 1, None) == _lib.NS_EINVAL
    assert L.ns_csum_tcp_tx_host_multi(hs, 1, buf, 4096, t, 1, None) == _lib.NS_EINVAL  # a NULL context
    assert L.ns_csum_rx_ring_host(None, buf, 4096, ctypes.byref(r), u32, u16, None) == _lib.NS_EINVAL
    assert L.ns_csum_rx_bufs(None, buf, 4096, ctypes.byref(r), u32, u32, u16, None, None) == _lib.NS_EINVAL


GO_SHIM = os.path.join(ROOT, "go", "header", "checksum_batch_hip.go")
# Identifiers tcpip/header/checksum.go declares (checksum.go:26-122): the shim
# is added NEXT to that file, so it must declare none of them.
CHECKSUM_GO_NAMES = {"calculateChecksum", "Checksum", "ChecksumVV", "ChecksumVVWithOffset", "ChecksumCombine",
                     "PseudoHeaderChecksum"}
# APIs newer than the reference's Go (<= 1.14: tcpip/time_unsafe.go:15-16).
POST_GO114 = (r"runtime\.Pinner", r"unsafe\.Slice", r"unsafe\.Add", r"unsafe\.String", r"\bany\b",
              r"\[\s*\w+\s+(any|comparable)\b", r"\bcomparable\b", r"strings\.Cut\b", r"atomic\.(Int|Uint|Bool|Pointer)\w*\b",
              r"errors\.Join", r"\bmin\(", r"\bmax\(", r"\bclear\(", r"//go:build", r"\bio\.ReadAll\b",
              r"os\.ReadFile", r"os\.WriteFile")


def _go_code(src):
    """The Go source without comments and string literals (a cgo preamble
    comment stays out of the scan too)."""
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    src = re.sub(r"//[^\n]*", "", src)
    return re.sub(r'"(?:[^"\\\n]|\\.)*"|`[^`]*`', '""', src)


def test_go_shim_builds_with_the_reference_go_version_and_adds_only_new_names():
    """No Go toolchain exists here, so the cgo shim is checked statically:
    it uses no API newer than Go 1.14 (the reference's newest supported Go),
    carries the hipcsum build tag in the pre-1.17 form, declares none of
    checksum.go's names (it is added next to that file, which stays
    untouched), passes C only functions include/netstack_csum.h declares,
    and checks the library's ABI version before use."""
    raw = open(GO_SHIM).read()
    code = _go_code(raw)
    for pat in POST_GO114:
        assert not re.search(pat, code), pat
    # build tag: a +build line before the package clause, then a blank line
    assert "\n\n// +build hipcsum\n\npackage header\n" in raw
    declared = set(re.findall(r"^func (?:\([^)]*\)\s*)?(\w+)\(", code, flags=re.M))
    declared |= set(re.findall(r"^type (\w+)\b", code, flags=re.M))
    declared |= set(re.findall(r"^\s*(\w+)\s*=", code[code.index("const ("):] if "const (" in code else "",
                               flags=re.M))
    assert declared and not (declared & CHECKSUM_GO_NAMES), declared & CHECKSUM_GO_NAMES
    for name in ("ChecksumVVBatch", "ChecksumChains", "ChecksumBatch", "VerifyPacketBuffers", "FillPacketBuffers",
                 "FillTCPBatches", "VerifyRingDevice"):
        assert name in declared, name
    called = set(re.findall(r"C\.(ns_csum_\w+)\(", code))
    assert called and called <= declared_symbols(), called - declared_symbols()
    assert "C.ns_csum_abi_version()" in code and "C.NS_CSUM_ABI_VERSION" in code
    # #cgo paths come from CGO_CFLAGS / CGO_LDFLAGS, not ${SRCDIR}-relative guesses
    assert "${SRCDIR}" not in raw


def test_go_shim_names_do_not_collide_with_the_reference_package():
    """Where the reference tree is present (this container), every top-level
    identifier of its package header, in any file, differs from the shim's."""
    hdr = "/root/reference/tcpip/header"
    if not os.path.isdir(hdr):
        pytest.skip("reference tree absent")
    ref = set()
    for fn in os.listdir(hdr):
        if fn.endswith(".go") and not fn.endswith("_test.go"):
            code = _go_code(open(os.path.join(hdr, fn)).read())
            ref |= set(re.findall(r"^func (?:\([^)]*\)\s*)?(\w+)\(", code, flags=re.M))
            ref |= set(re.findall(r"^type (\w+)\b", code, flags=re.M))
            ref |= set(re.findall(r"^(?:var|const)\s+(\w+)", code, flags=re.M))
            for blk in re.findall(r"^(?:const|var) \((.*?)^\)", code, flags=re.M | re.S):
                ref |= set(re.findall(r"^\s*(\w+)", blk, flags=re.M))
    assert CHECKSUM_GO_NAMES <= ref
    code = _go_code(open(GO_SHIM).read())
    mine = set(re.findall(r"^func (\w+)\(", code, flags=re.M)) | set(re.findall(r"^type (\w+)\b", code, flags=re.M))
    mine |= set(re.findall(r"^var \((.*?)^\)", code, flags=re.M | re.S) and
                re.findall(r"^\s+(\w+)\s", re.findall(r"^var \((.*?)^\)", code, flags=re.M | re.S)[0], flags=re.M))
    for blk in re.findall(r"^const \((.*?)^\)", code, flags=re.M | re.S):
        mine |= set(re.findall(r"^\s*(\w+)\s*=", blk, flags=re.M))
    mine |= set(re.findall(r"^const (\w+)", code, flags=re.M))
    assert mine and not (mine & ref), mine & ref


GO_CALLERS = {  # file -> (package, build tag)
    "go/transport/tcp/csum_batch_hip.go": ("tcp", "hipcsum"),
    "go/transport/tcp/csum_batch_go.go": ("tcp", "!hipcsum"),
    "go/link/fdbased/csum_rx_hip.go": ("fdbased", "linux,hipcsum"),
    "go/link/fdbased/csum_rx_go.go": ("fdbased", "linux,!hipcsum"),
}
GO_SHARED = {  # untagged files both builds compile -> package
    "go/transport/tcp/csum_batch_ref.go": "tcp",
}
GO_PATCH = os.path.join(ROOT, "go", "netstack-hipcsum.patch")


def _top_level(code):
    names = set(re.findall(r"^func (\w+)\(", code, flags=re.M)) | set(re.findall(r"^type (\w+)\b", code, flags=re.M))
    names |= set(re.findall(r"^(?:var|const)\s+(\w+)", code, flags=re.M))
    for blk in re.findall(r"^(?:const|var) \((.*?)^\)", code, flags=re.M | re.S):
        names |= set(re.findall(r"^\s*(\w+)", blk, flags=re.M))
    return names


def _signatures(code):
    return dict(re.findall(r"^func (\w+)(\(.*?\)[^{]*)\{", code, flags=re.M))


def test_go_caller_files_pair_up_and_use_only_what_exists():
    """The build-tagged caller files: Go <= 1.14 forms,
    the tag before the package clause, each hipcsum file paired with a
    default-build file declaring the same functions with the same
    signatures; every header.X they call exists in the shim or the reference
    package, and every tcpip.RXChecksum* they use is declared by the patch."""
    shim = _top_level(_go_code(open(GO_SHIM).read()))
    patch = open(GO_PATCH).read()
    added = "\n".join(l[1:] for l in patch.splitlines() if l.startswith("+") and not l.startswith("+++"))
    by_pkg = {}
    for rel, (pkg, tag) in GO_CALLERS.items():
        raw = open(os.path.join(ROOT, rel)).read()
        code = _go_code(raw)
        for pat in POST_GO114:
            assert not re.search(pat, code), (rel, pat)
        assert f"\n\n// +build {tag}\n\npackage {pkg}\n" in raw, rel
        by_pkg.setdefault(pkg, []).append((tag, _signatures(code), code))
        for name in set(re.findall(r"\bheader\.(\w+)", code)):
            assert name in shim or name in REF_HEADER_NAMES or not os.path.isdir("/root/reference"), (rel, name)
        for name in set(re.findall(r"\btcpip\.(RXChecksum\w*)", code)):
            assert re.search(rf"\b{name}\b", added), (rel, name)
    for rel, pkg in GO_SHARED.items():
        raw = open(os.path.join(ROOT, rel)).read()
        code = _go_code(raw)
        for pat in POST_GO114:
            assert not re.search(pat, code), (rel, pat)
        assert "+build" not in raw and f"\npackage {pkg}\n" in raw, rel
        for name in set(re.findall(r"\bheader\.(\w+)", code)):
            assert name in REF_HEADER_NAMES or not os.path.isdir("/root/reference"), (rel, name)  # reference only
    for pkg, files in by_pkg.items():
        (t1, s1, c1), (t2, s2, c2) = files
        assert t1.replace("!", "") == t2.replace("!", "") and t1 != t2
        # what the patch calls in this package is declared by both variants, alike
        for name in ("deferTCPBatchChecksums", "finishTCPBatchChecksums") if pkg == "tcp" else ("verifyRXChecksums",):
            assert re.search(rf"\b{name}\b", added)
            assert s1.get(name) == s2.get(name), (pkg, name)
            assert re.search(rf"^(?:func|const) {name}\b", c1, flags=re.M) and \
                re.search(rf"^(?:func|const) {name}\b", c2, flags=re.M), (pkg, name)


def _ref_names(d):
    out = set()
    for fn in os.listdir(d):
        if fn.endswith(".go") and not fn.endswith("_test.go"):
            out |= _top_level(_go_code(open(os.path.join(d, fn)).read()))
    return out


REF_HEADER_NAMES = _ref_names("/root/reference/tcpip/header") if os.path.isdir("/root/reference/tcpip/header") \
    else set()


def test_go_patch_applies_to_the_reference_and_adds_no_colliding_names(tmp_path):
    """go/netstack-hipcsum.patch applies cleanly to the reference's files
    (patch --dry-run on a copy), and the caller files' top-level names are
    new in their packages."""
    if not os.path.isdir("/root/reference/tcpip"):
        pytest.skip("reference tree absent")
    import shutil

    files = re.findall(r"^\+\+\+ b/(\S+)", open(GO_PATCH).read(), flags=re.M)
    assert set(files) == {"tcpip/packet_buffer.go", "tcpip/transport/tcp/segment.go",
                          "tcpip/transport/tcp/connect.go", "tcpip/network/ipv4/ipv4.go",
                          "tcpip/link/fdbased/packet_dispatchers.go"}
    for f in files:
        os.makedirs(tmp_path / os.path.dirname(f), exist_ok=True)
        shutil.copy(os.path.join("/root/reference", f), tmp_path / f)
    r = subprocess.run(["patch", "-p1", "--dry-run", "-i", GO_PATCH], cwd=tmp_path, capture_output=True, text=True)
    assert r.returncode == 0 and "FAILED" not in r.stdout and "fuzz" not in r.stdout, r.stdout + r.stderr
    for rel, (pkg, _) in GO_CALLERS.items():
        d = {"tcp": "tcpip/transport/tcp", "fdbased": "tcpip/link/fdbased"}[pkg]
        mine = _top_level(_go_code(open(os.path.join(ROOT, rel)).read()))
        assert mine and not (mine & _ref_names(os.path.join("/root/reference", d))), (rel, mine)


def test_latency_bounds_are_collected_after_every_parity_test():
    """A wall-clock bound (@pytest.mark.latency) is collected after every
    other GPU test, so under -x a timing outlier cannot hide parity results."""
    import subprocess
    import sys

    r = subprocess.run([sys.executable, "-m", "pytest", "-q", "--collect-only", "-m", "gpu", "-p", "no:cacheprovider",
                        os.path.join(ROOT, "tests")], capture_output=True, text=True, cwd=ROOT, timeout=300)
    ids = [l for l in r.stdout.splitlines() if "::" in l]
    assert len(ids) > 100, r.stdout[-2000:]
    r2 = subprocess.run([sys.executable, "-m", "pytest", "-q", "--collect-only", "-m", "gpu and latency", "-p",
                         "no:cacheprovider", os.path.join(ROOT, "tests")], capture_output=True, text=True, cwd=ROOT,
                        timeout=300)
    marked = {l for l in r2.stdout.splitlines() if "::" in l}
    assert any("test_growing_scratch_does_not_hold_up_synchronous_calls" in l for l in marked)
    assert len(marked) >= 3, marked
    lat = [i for i, l in enumerate(ids) if l in marked]
    assert lat == list(range(len(ids) - len(marked), len(ids))), ids[-5:]
    par = [i for i, l in enumerate(ids) if "test_gpu_tcp.py" in l or "test_gpu_sync.py" in l]
    assert par and max(par) < lat[0]


def test_go_engine_errors_fall_back_to_the_reference_go():
    """SURVEY §8(b)'s error policy: no engine status ever panics.  Every
    C.ns_csum_* call's status goes to engineFailed (counted, exported as
    EngineFallbacks); the no-error batch functions then compute with the
    reference's own package-header functions, and the build-tagged callers
    use the ...Err variants and run their default-build path: TX the
    reference's per-segment loop (csum_batch_ref.go, shared with the default
    build), RX nothing (RXChecksumUnknown: segment.parse verifies).  The only
    panics left are argument misuse the reference's Go panics on too."""
    shim = _go_code(open(GO_SHIM).read())
    raw = open(GO_SHIM).read()
    assert "csumMust" not in shim and "strerror" not in "".join(re.findall(r"panic\((.*?)\)\n", raw))
    for m in re.finditer(r"panic\(\"([^\"]*)\"\)", raw):
        assert re.search(r"too short|slice bounds|views in one packet", m.group(1)), m.group(1)
    # every engine call's status is checked and routed to engineFailed
    calls = re.findall(r"C\.(ns_csum_\w+)\(", shim)
    checked = re.findall(r"(?:rc :=|rc =|csumErr =) C\.(ns_csum_\w+)\(", shim)
    passive = {"ns_csum_abi_version", "ns_csum_strerror", "ns_csum_stage_release"}
    assert set(calls) - passive <= set(checked), set(calls) - passive - set(checked)
    assert shim.count("engineFailed(") >= len(set(checked)) and "func EngineFallbacks() uint64" in shim
    for fn, ref in (("ChecksumVVBatch", "ChecksumVVWithOffset(vv"), ("ChecksumChains", "checksumChainsGo(chains"),
                    ("ChecksumBatch", "calculateChecksum(b"), ("VerifyPacketBuffers", "PacketChecksumUnchecked"),
                    ("FillPacketBuffers", "fillPacketGo("), ("FillTCPBatches", "fillTCPBatchGo(&batches[i])")):
        body = re.search(rf"^func {fn}\(.*?^}}", shim, flags=re.M | re.S).group(0)
        assert ref in body, fn
    tx = _go_code(open(os.path.join(ROOT, "go/transport/tcp/csum_batch_hip.go")).read())
    rx = _go_code(open(os.path.join(ROOT, "go/link/fdbased/csum_rx_hip.go")).read())
    assert "header.ChecksumChainsErr(" in tx and "tcpBatchChecksumsRef(hdrs, data, pseudo)" in tx
    assert "header.VerifyPacketBuffersErr(" in rx
    dflt = _go_code(open(os.path.join(ROOT, "go/transport/tcp/csum_batch_go.go")).read())
    assert "tcpBatchChecksumsRef(hdrs, data, pseudo)" in dflt
    for rel in list(GO_CALLERS) + list(GO_SHARED):
        assert "panic(" not in _go_code(open(os.path.join(ROOT, rel)).read()), rel


def test_go_offload_gates_sit_at_the_measured_crossover():
    """The build-tagged callers offload only calls at or above the sizes
    where one engine call beat one core (tools/crossover.cc on MI355X,
    profiles/r05/crossover.json: per-point medians of six runs,
    tools/crossover_merge.py); below them the reference's own Go code runs
    (INTEGRATION.md §2).  Each gate is a measured point no smaller than the
    measured crossover and no more than 2x it, and each caller tests it
    before calling the engine."""
    import json

    code = _go_code(open(GO_SHIM).read())
    env = {}
    for name in ("ChainsOffloadMinBytes", "VerifyOffloadMinBytes", "TxBatchOffloadMinBytes"):
        m = re.search(rf"^\s*{name}\s*=\s*([0-9<>* ]+)$", code, flags=re.M)
        assert m, name
        env[name] = int(eval(m.group(1), {}))  # a constant expression of integers
    with open(os.path.join(ROOT, "profiles", "r05", "crossover.json")) as f:
        xo = json.load(f)
    # (ChecksumVVBatch has no gated caller: the TX hook sends ChecksumChains)
    for gate, shape in (("ChainsOffloadMinBytes", "chains"), ("VerifyOffloadMinBytes", "verify"),
                        ("TxBatchOffloadMinBytes", "tx_host")):
        x = xo[shape]["crossover"]
        assert x is not None, shape
        assert x["bytes"] <= env[gate] <= 2 * x["bytes"], (gate, shape, x, env[gate])
        assert env[gate] in {p["bytes"] for p in xo[shape]["points"]}, (gate, shape)
    tx = _go_code(open(os.path.join(ROOT, "go/transport/tcp/csum_batch_hip.go")).read())
    assert re.search(r"return payload >= header\.ChainsOffloadMinBytes", tx)
    rx = _go_code(open(os.path.join(ROOT, "go/link/fdbased/csum_rx_hip.go")).read())
    assert re.search(r"if total < header\.VerifyOffloadMinBytes \{\s*return\s*\}", rx)
    assert rx.index("VerifyOffloadMinBytes") < rx.index("header.VerifyPacketBuffersErr(")
    body = re.search(r"^func FillTCPBatches\(.*?^}", code, flags=re.M | re.S).group(0)
    assert body.index("TxBatchOffloadMinBytes") < body.index("FillTCPBatchesErr(")
    patch = open(GO_PATCH).read()
    assert "+\tdeferCsum := deferTCPBatchChecksums(data.Size()) &&" in patch

GO_GATE_TESTS = {  # Go tests of the engine paths behind the gates -> (package, build tag, gate)
    "go/transport/tcp/csum_batch_hip_test.go": ("tcp", "hipcsum", "ChainsOffloadMinBytes"),
    "go/link/fdbased/csum_rx_hip_test.go": ("fdbased", "linux,hipcsum", "VerifyOffloadMinBytes"),
}


def test_go_gate_tests_open_the_gates_and_compare_with_the_reference():
    """with the measured gates the hooks never reach the engine
    at the reference's sizes, so Go tests open each gate (a package
    variable, restored after) and check the engine path against the
    reference's own decision: finishTCPBatchChecksums against
    tcpBatchChecksumsRef byte for byte, verifyRXChecksums' verdicts against
    segment.parse's rule, with no engine fallback counted.  Checked
    statically (no Go toolchain): Go <= 1.14 forms, the tag before the
    package clause, the gate set and restored, the functions they test
    exist in the paired hipcsum files."""
    shim = _go_code(open(GO_SHIM).read())
    assert re.search(r"^var \(.*?^\s*ChainsOffloadMinBytes\s*=.*?^\s*VerifyOffloadMinBytes\s*=.*?^\)", shim,
                     flags=re.M | re.S), "the gates must be variables a test can set"
    for rel, (pkg, tag, gate) in GO_GATE_TESTS.items():
        raw = open(os.path.join(ROOT, rel)).read()
        code = _go_code(raw)
        for pat in POST_GO114:
            assert not re.search(pat, code), (rel, pat)
        assert f"\n\n// +build {tag}\n\npackage {pkg}\n" in raw, rel
        assert re.search(rf"defer func\(v int\) {{ header\.{gate} = v }}\(header\.{gate}\)", code), rel
        assert re.search(rf"header\.{gate} = 0", code), rel
        assert "header.EngineFallbacks()" in code, rel
        tested = {"tcp": ("deferTCPBatchChecksums", "finishTCPBatchChecksums", "tcpBatchChecksumsRef"),
                  "fdbased": ("verifyRXChecksums",)}[pkg]
        for fn in tested:
            assert re.search(rf"\b{fn}\(", code), (rel, fn)
        for name in set(re.findall(r"\bheader\.(\w+)", code)):
            assert name in _top_level(shim) or name in REF_HEADER_NAMES or not os.path.isdir("/root/reference"), \
                (rel, name)


def test_go_tx_host_test_compares_with_the_reference_go():
    """FillTCPBatches (ns_csum_tcp_tx_host) has a Go test in package header
    that fills many batches through the engine and through fillTCPBatchGo
    (the reference's buildTCPHdr / addIPHeader arithmetic) and compares the
    slot bytes, with no fallback counted.  fillTCPBatchGo itself calls only
    the reference's package-header functions.  Checked statically."""
    raw = open(os.path.join(ROOT, "go/header/checksum_batch_hip_test.go")).read()
    code = _go_code(raw)
    for pat in POST_GO114:
        assert not re.search(pat, code), pat
    assert "\n\n// +build hipcsum\n\npackage header\n" in raw
    for call in ("FillTCPBatchesErr(got)", "FillTCPBatches(got)", "fillTCPBatchGo(&want[i])", "EngineFallbacks()",
                 "bytes.Equal(", "defer func(v int) { TxBatchOffloadMinBytes = v }(TxBatchOffloadMinBytes)"):
        assert call in code, call
    for mode in ("TxCsumFull", "TxCsumPartial", "TxCsumOffload"):
        assert mode in code, mode
    shim = _go_code(open(GO_SHIM).read())
    body = re.search(r"^func fillTCPBatchGo\(.*?^}", shim, flags=re.M | re.S).group(0)
    for ref in ("PseudoHeaderChecksum(", "ChecksumVVWithOffset(", "tcp.CalculateChecksum(", "ip.CalculateChecksum()"):
        assert ref in body, ref
        if os.path.isdir("/root/reference/tcpip/header"):
            assert ref.split("(")[0].split(".")[-1] in REF_HEADER_NAMES | {"CalculateChecksum"}, ref
    assert "C.ns_csum_tcp_tx_host(" in shim and "ns_csum_tcp_tx_host" in declared_symbols()
