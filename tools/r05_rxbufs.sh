#!/bin/bash
# Round 5: ns_csum_rx_bufs (buffer lists) beside the ring tests it shares the
# kernel with, then the ring bench line (the kernel's LIST = 0 instance).
set -euo pipefail
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
cd "$R"
O=gpurun_out/rxbufs
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_rx_bufs.py tests/test_gpu_rx_ring.py tests/test_gpu_rx_ring_host.py \
  -x -v --timeout 120 --timeout-method thread > $O/tests.log 2>&1
timeout -k 10 300 python -u bench.py --config 7 --rx-layout ring --no-cpu > $O/bench_cfg7_ring.json 2> $O/bench_cfg7_ring.err
echo done
