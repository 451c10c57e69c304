#!/bin/bash
# Round 5: receive tests, then the buffer list at several buffer spacings
# (ring order and shuffled) beside the ring.
set -euo pipefail
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
cd "$R"
O=gpurun_out/bufs_stride
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_rx_bufs.py tests/test_gpu_rx_ring.py tests/test_gpu_rx_ring_host.py \
  -x -q --timeout 120 --timeout-method thread > $O/tests.log 2>&1
timeout -k 10 200 python -u bench.py --config 7 --rx-layout ring --no-cpu > $O/ring.json 2>/dev/null
for st in 1504 1536 1664 2048; do
  for order in ring shuffled; do
    timeout -k 10 200 python -u bench.py --config 7 --rx-layout bufs --bufs-stride $st --bufs-order $order --no-cpu \
      > $O/bufs_${st}_${order}.json 2>/dev/null
  done
done
echo done
