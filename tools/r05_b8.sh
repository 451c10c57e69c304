#!/bin/bash
# Round 5, batch 8: the packet-mode benches over two rotating batches (as
# cfg2), and the ring probe rotating vs re-reading one ring.
set -euo pipefail
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
cd "$R"
export TMPDIR=/tmp
mkdir -p gpurun_out/b8
timeout -k 10 300 python3 tools/rx_ring_probe.py --only 0 --rounds 7 --rotate 1 > gpurun_out/b8/ring_rot.json 2> gpurun_out/b8/ring_rot.err
timeout -k 10 300 python3 tools/rx_ring_probe.py --only 0 --rounds 7 --rotate 0 > gpurun_out/b8/ring_norot.json 2> gpurun_out/b8/ring_norot.err
timeout -k 10 300 python3 bench.py --config 7 --rx-layout ring > gpurun_out/b8/bench_cfg7_ring.json 2> gpurun_out/b8/bench_cfg7_ring.err
timeout -k 10 300 python3 bench.py --config 7 > gpurun_out/b8/bench_cfg7.json 2> gpurun_out/b8/bench_cfg7.err
timeout -k 10 300 python3 bench.py --config 8 --tx-layout split > gpurun_out/b8/bench_cfg8_split.json 2> gpurun_out/b8/bench_cfg8_split.err
echo done
