#!/bin/bash
# Round 5: ns_csum_rx_ring_host — its GPU tests beside the device ring's, the
# host TX tests, then the host-inclusive ring bench line.
set -euo pipefail
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
cd "$R"
O=gpurun_out/rxhost
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_rx_ring_host.py tests/test_gpu_rx_ring.py tests/test_gpu_tx_host.py \
  -x -v --timeout 120 --timeout-method thread > $O/tests.log 2>&1
timeout -k 10 300 python -u bench.py --config 7 --rx-layout ring --mode host --steps 10 --warmup 2 \
  > $O/bench_host7_ring.json 2> $O/bench_host7_ring.err
echo done
