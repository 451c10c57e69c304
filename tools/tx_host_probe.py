"""ns_csum_tcp_tx_host on the box: host-inclusive time per call for cfg8's
1M x 1460-B segments (sendTCPBatch's layout) from a pinned and from a
pageable host arena, as 1 call and as 23,832 calls of 64 KiB, at a few
staging sizes.  Medians of --reps calls after one warm-up.  No checking
here (tests/test_gpu_tx_host.py and bench.py --mode host --config 8 do it).
  python tools/tx_host_probe.py [--reps 5] [--out FILE]"""

import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=5)
    ap.add_argument("--out", default=None)
    args = ap.parse_args()
    import torch

    import bench
    from netstack_amd import Engine
    from netstack_amd import workloads as W
    from netstack_amd.engine import tx_table

    n = 1 << 20
    geo = W.tx_struct_geometry(n)
    src = W.tx_split_batch(n, 7000, "cuda:0")[0].cpu()
    pinned = torch.empty(src.numel(), dtype=torch.uint8).pin_memory()
    pinned.copy_(src)
    pageable = src.numpy().copy()
    del src
    tables = {1: tx_table([geo]), 23832: tx_table(bench.tx_calls(geo, 23832))}
    rows = []
    for staging in (16 << 20, 64 << 20, 256 << 20):
        with Engine(0, staging_bytes=staging) as eng:
            for mem, a in (("pinned", pinned.numpy()), ("pageable", pageable)):
                for calls, tab in tables.items():
                    eng.tcp_tx_host(a, tab)  # warm-up: staging allocated
                    ts = []
                    for _ in range(args.reps):
                        t0 = time.perf_counter()
                        eng.tcp_tx_host(a, tab)
                        ts.append(time.perf_counter() - t0)
                    ms = sorted(ts)[len(ts) // 2] * 1e3
                    rows.append({"staging_mib": staging >> 20, "memory": mem, "calls": calls, "ms": ms,
                                 "gib_s": n * W.RX_PKT / (ms / 1e3) / 2**30,
                                 "pcie_gb_s": (geo["size"] + n * geo["slot"]) / (ms / 1e3) / 1e9})
                    print(json.dumps(rows[-1]), flush=True)
    if args.out:
        with open(args.out, "w") as f:
            json.dump(rows, f, indent=1)


if __name__ == "__main__":
    main()
