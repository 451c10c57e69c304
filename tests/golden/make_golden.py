"""Generate tests/golden/*.json (run: python tests/golden/make_golden.py).

kat.json      — known answers that do NOT come from our restatement: the six
                cases of the reference's own test (tcpip/header/checksum_test.go:
                34-94, inputs and `want` copied as data), the RFC 1071 §3
                numerical example, and the classic IPv4 header whose checksum
                field is correct (sums to 0xffff).  These pin the oracle.
vectors.json  — edge cases and seeded random cases whose expected values are
                computed by the pure-Python restatement oracle/oracle.py
                (py_*), itself pinned by kat.json.  Inputs are literal hex
                (<= a few KiB each) or a compact generator spec:
                {"fill": byte, "len": n} or {"splitmix": seed, "len": n}.

The reference is Go and cannot run in this image (no Go toolchain), so no
output of the reference itself is included; see DESIGN.md §Oracle.
"""
from __future__ import annotations

import json
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, os.path.join(ROOT, "oracle"))
sys.path.insert(0, ROOT)

import numpy as np  # noqa: E402

import oracle as O  # noqa: E402
from netstack_amd.workloads import random_bytes, splitmix64  # noqa: E402


def materialize(spec) -> bytes:
    """Bytes of a fixture input (hex string or generator spec)."""
    if isinstance(spec, str):
        return bytes.fromhex(spec)
    if "fill" in spec:
        return bytes([spec["fill"]]) * spec["len"]
    if "splitmix" in spec:
        return random_bytes(spec["splitmix"], spec["len"]).tobytes()
    raise ValueError(spec)


def kat():
    # tcpip/header/checksum_test.go:34-94 — name, views, off, size, initial, want
    ref = [
        ("empty", [[1, 9, 0, 5, 4]], 0, 0, 0, 0),
        ("OneView", [[1, 9, 0, 5, 4]], 0, 5, 0, 1294),
        ("TwoViews", [[1, 9, 0, 5, 4], [4, 3, 7, 1, 2, 123]], 0, 11, 0, 33819),
        ("TwoViewsWithOffset", [[98, 1, 9, 0, 5, 4], [4, 3, 7, 1, 2, 123]], 1, 11, 0, 33819),
        ("ThreeViewsWithOffset",
         [[98, 1, 9, 0, 5, 4], [98, 1, 9, 0, 5, 4], [4, 3, 7, 1, 2, 123]], 7, 11, 0, 33819),
        ("ThreeViewsWithInitial",
         [[77, 11, 33, 0, 55, 44], [98, 1, 9, 0, 5, 4], [4, 3, 7, 1, 2, 123, 99]], 7, 11, 77, 33896),
    ]
    vv = [{"name": n, "views": [bytes(v).hex() for v in views], "off": off, "size": size,
           "initial": init, "want": want,
           "source": "tcpip/header/checksum_test.go:34-94"} for (n, views, off, size, init, want) in ref]
    single = [
        {"name": "rfc1071_sec3_example", "buf": "0001f203f4f5f6f7", "initial": 0, "want": 0xDDF2,
         "source": "RFC 1071 section 3 numerical example (sum ddf2)"},
        {"name": "ipv4_header_valid", "buf": "45000073000040004011b861c0a80001c0a800c7", "initial": 0,
         "want": 0xFFFF, "source": "IPv4 header with a correct checksum field sums to 0xffff "
                                   "(the invariant of ipv4_test.go:140-142 / checker.go:51-53)"},
        {"name": "ipv4_header_zeroed_csum", "buf": "450000730000400040110000c0a80001c0a800c7",
         "initial": 0, "want": 0x479E, "source": "same header, checksum field zeroed: ^0x479e == 0xb861"},
    ]
    return {"vv_with_offset": vv, "checksum": single}


def vectors():
    out_single, out_vv, out_restart, out_pseudo, out_batch = [], [], [], [], []

    def add_single(name, spec, initial):
        buf = materialize(spec)
        out_single.append({"name": name, "buf": spec, "initial": initial,
                           "want": O.py_checksum(buf, initial)})

    # lengths 0..3, odd lengths, all-zero and all-0xFF, initial in {0,1,0xFFFF}
    for L in (0, 1, 2, 3, 5, 7, 63, 64, 65, 1499, 1500, 1501):
        for init in (0, 1, 0xFFFF):
            add_single(f"zeros_{L}_{init}", {"fill": 0, "len": L}, init)
            add_single(f"ones_{L}_{init}", {"fill": 0xFF, "len": L}, init)
            add_single(f"rand_{L}_{init}", {"splitmix": 1000 + L, "len": L}, init)
    # zero representation: all-zero with initial 0 -> 0x0000; V == k*65535 -> 0xFFFF
    add_single("fffe_plus_1", "fffe0001", 0)
    # uint32 wrap quirk: > 128 KiB (200,000 x 0xFF -> 0xFFFE in Go)
    add_single("wrap_200000_ff", {"fill": 0xFF, "len": 200000}, 0)
    add_single("wrap_131074_ff", {"fill": 0xFF, "len": 131074}, 0)
    add_single("wrap_131076_ff_init", {"fill": 0xFF, "len": 131076}, 0xFFFF)
    add_single("nowrap_131072_ff", {"fill": 0xFF, "len": 131072}, 0xFFFF)
    add_single("big_random_300000", {"splitmix": 77, "len": 300000}, 0x1234)
    add_single("cfg1_64KiB", {"splitmix": 1, "len": 65536}, 0)

    # VectorisedView cases: odd views (1000 views of 7 bytes, ipv4_test.go:257-278),
    # BufConfig-shaped RX views (packet_dispatchers.go:30), offsets/sizes.
    def add_vv(name, views, initial, off, size):
        vb = [materialize(v) for v in views]
        out_vv.append({"name": name, "views": views, "initial": initial, "off": off, "size": size,
                       "want": O.py_checksum_vv_with_offset(vb, initial, off, size)})

    seven = [{"splitmix": 2000 + k, "len": 7} for k in range(1000)]
    add_vv("views_1000x7", seven, 0, 0, 7000)
    add_vv("views_1000x7_off3", seven, 0xBEEF, 3, 6990)
    bufcfg = [128, 256, 256, 512, 348]
    rx = [{"splitmix": 3000 + k, "len": L} for k, L in enumerate(bufcfg)]
    add_vv("rx_bufconfig_1500", rx, 0x1111, 40, 1460)  # TrimFront(40) then ChecksumVV
    add_vv("rx_bufconfig_odd_off", rx, 0x2222, 41, 1459)
    add_vv("size_past_end", rx, 7, 100, 100000)
    add_vv("off_past_end", rx, 7, 5000, 10)
    add_vv("empty_views_mixed", ["", "01", "", "0203", "", "040506"], 0, 0, 6)
    add_vv("zero_size", rx, 0x4321, 10, 0)
    big = [{"fill": 0xFF, "len": 140000}, {"fill": 0xFF, "len": 140001}, {"splitmix": 9, "len": 3}]
    add_vv("big_views_wrap", big, 0xFFFF, 0, 280004)
    add_vv("big_views_wrap_off", big, 0x10, 1, 280000)
    many_small = [{"fill": 0xFF, "len": 1001} for _ in range(200)]  # > 128 KiB total, each small
    add_vv("many_small_views_no_wrap", many_small, 0xFFFF, 0, 200200)
    rng = np.random.default_rng(11)
    for k in range(20):
        nv = int(rng.integers(1, 12))
        views = [{"splitmix": 5000 + 100 * k + j, "len": int(rng.integers(0, 300))} for j in range(nv)]
        tot = sum(v["len"] for v in views)
        off = int(rng.integers(0, tot + 2))
        size = int(rng.integers(0, tot + 5))
        add_vv(f"random_vv_{k}", views, int(rng.integers(0, 65536)), off, size)

    # per-view restart callers (sendUDP / ICMP)
    def add_restart(name, views, initial):
        vb = [materialize(v) for v in views]
        out_restart.append({"name": name, "views": views, "initial": initial,
                            "want": O.py_views_restart(vb, initial)})

    add_restart("udp_even_views", [{"splitmix": 6000, "len": 100}, {"splitmix": 6001, "len": 200}], 0x5555)
    add_restart("udp_odd_views", [{"splitmix": 6002, "len": 7}, {"splitmix": 6003, "len": 9},
                                  {"splitmix": 6004, "len": 1}], 0x0101)
    add_restart("restart_with_empty", ["", "ff", "", "0102"], 0)

    # pseudo headers
    for k, (proto, src, dst, tl) in enumerate([
            (6, "0a000001", "0a000002", 1480),
            (17, "c0a80001", "c0a800c7", 8),
            (6, "20010db8000000000000000000000001", "20010db8000000000000000000000002", 1440),
            (58, "fe800000000000000000000000000001", "ff020000000000000000000000000001", 32),
            (6, "0a0000", "0a000002", 5)]):  # odd-length address (restart semantics)
        out_pseudo.append({"name": f"pseudo_{k}", "protocol": proto, "src": src, "dst": dst,
                           "total_len": tl, "want": O.py_pseudo_header(proto, bytes.fromhex(src),
                                                                         bytes.fromhex(dst), tl)})

    # descriptor batches over one arena (include/netstack_csum.h contract)
    def add_batch(name, arena_spec, descs, chained):
        arena = materialize(arena_spec)
        d = np.zeros(len(descs), dtype=O.DESC_DTYPE)
        for i, (off, ln, init, fl) in enumerate(descs):
            d[i] = (off, ln, init, fl)
        out_batch.append({"name": name, "arena": arena_spec, "chained": chained,
                          "desc": [list(x) for x in descs],
                          "want": [int(x) for x in O.py_batch(arena, d, chained)]})

    r = np.random.default_rng(5)
    descs = []
    for i in range(300):
        off = int(r.integers(0, 60000))
        ln = int(r.integers(0, 4097)) if i % 7 else int(r.integers(0, 40))
        ln = min(ln, 65536 - off)
        descs.append((off, ln, int(r.integers(0, 65536)), int(r.integers(0, 2))))
    add_batch("random_unaligned_300", {"splitmix": 42, "len": 65536}, descs, False)
    chain = []
    pos = 0
    for i in range(120):
        ln = int(r.integers(0, 600))
        cont = (i % 5) != 0
        chain.append((pos, ln, int(r.integers(0, 65536)), (2 if cont else 0) | (pos & 1)))
        pos += ln
    add_batch("chained_runs_120", {"splitmix": 43, "len": max(pos, 1)}, chain, True)
    add_batch("zero_len_and_edges", {"splitmix": 44, "len": 4096},
              [(0, 0, 0x1234, 0), (4096, 0, 7, 0), (4095, 1, 0, 0), (4095, 1, 0, 1),
               (0, 4096, 0xFFFF, 0), (1, 4095, 1, 1), (15, 17, 0, 0), (16, 16, 0, 1)], False)
    return {"checksum": out_single, "vv_with_offset": out_vv, "views_restart": out_restart,
            "pseudo_header": out_pseudo, "batch": out_batch}


def main():
    with open(os.path.join(HERE, "kat.json"), "w") as f:
        json.dump(kat(), f, indent=1)
    with open(os.path.join(HERE, "vectors.json"), "w") as f:
        json.dump(vectors(), f, indent=None, separators=(",", ":"))
    print("wrote", os.listdir(HERE))


if __name__ == "__main__":
    main()
