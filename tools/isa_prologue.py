#!/usr/bin/env python3
"""Instruction census of a kernel's prologue in a hipcc .s file: from the
kernel's entry to its first payload load (the first buffer_load_dwordx4
after the descriptor load, or the first at all with --first), by class —
SMEM (s_load: kernargs), SALU, VALU, VMEM (global/buffer loads), waitcnts —
plus the whole kernel's totals.  Used to compare the product's small-packet
instance with the floor kernels.

  python tools/isa_prologue.py FILE.s KERNEL_SYMBOL [--first]
"""
import re
import sys


def body(path, sym):
    lines, on = [], False
    for line in open(path):
        if line.startswith(sym + ":"):
            on = True
            continue
        if on:
            if line.strip().startswith(".Lfunc_end"):
                break
            lines.append(line.rstrip("\n"))
    return lines


def klass(ins):
    op = ins.split()[0]
    if op.startswith("s_waitcnt"):
        return "waitcnt"
    if op.startswith("s_load") or op.startswith("s_buffer_load") or op in ("s_memtime", "s_memrealtime"):
        return "smem"
    if op.startswith(("global_load", "buffer_load", "flat_load")):
        return "vmem_load"
    if op.startswith(("global_store", "buffer_store", "flat_store", "global_atomic", "buffer_atomic")):
        return "vmem_store"
    if op.startswith("ds_"):
        return "lds"
    if op.startswith("v_"):
        return "valu"
    if op.startswith("s_"):
        return "salu"
    return "other"


def census(instrs):
    c = {}
    for i in instrs:
        k = klass(i)
        c[k] = c.get(k, 0) + 1
    return c


def main():
    path, sym = sys.argv[1], sys.argv[2]
    first = "--first" in sys.argv
    ins = [l.strip() for l in body(path, sym) if l.strip() and not l.strip().startswith((";", ".", "//"))
           and not re.match(r"^[.\w]+:", l.strip())]
    loads = [k for k, i in enumerate(ins) if klass(i) == "vmem_load"]
    # the first payload load: the first buffer_load (descriptors come through global_load)
    stop = next((k for k in loads if ins[k].startswith("buffer_load")), len(ins)) if not first else \
        (loads[0] if loads else len(ins))
    pro = ins[:stop + 1]
    print(f"{sym[:90]}")
    print(f"  prologue to the first payload load: {len(pro)} instructions {census(pro)}")
    print(f"  first loads: {[ins[k].split()[0] for k in loads[:6]]}")
    print(f"  whole kernel (static): {len(ins)} instructions {census(ins)}")


if __name__ == "__main__":
    main()
