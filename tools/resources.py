#!/usr/bin/env python3
"""Print hipcc's kernel resource report (netstack_amd/lib/csum_kernels.resources.txt,
kept by the Makefile) as one line per kernel: VGPRs, scratch, occupancy, LDS."""
import os
import re
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def parse(path):
    ks, cur = {}, None
    for line in open(path):
        m = re.search(r"Function Name: (\S+)", line)
        if m:
            cur = m.group(1)
            ks[cur] = {}
            continue
        m = re.search(r"remark: ([A-Za-z ]+?)(?: \[[^\]]*\])?: (\d+)", line)
        if m and cur:
            ks[cur][m.group(1).strip()] = int(m.group(2))
    return ks


def demangle(names):
    out = subprocess.run(["c++filt"], input="\n".join(names), capture_output=True, text=True).stdout
    return out.splitlines()


if __name__ == "__main__":
    path = sys.argv[1] if len(sys.argv) > 1 else os.path.join(ROOT, "netstack_amd", "lib", "csum_kernels.resources.txt")
    ks = parse(path)
    for (k, v), d in zip(ks.items(), demangle(list(ks))):
        d = re.sub(r"\(.*", "", d)
        print(f"{d:70s} vgpr {v.get('VGPRs', '?'):>3} scratch {v.get('ScratchSize', '?'):>3} "
              f"occ {v.get('Occupancy', '?')} lds {v.get('LDS Size', '?')}")
