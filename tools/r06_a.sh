#!/bin/bash
# Round 6, first GPU call: the receive tests with the minimum-size rows
# (ICMPv6 8 B), the packet-buffer tests, the host TX tests, smoke(), and the
# small-pass latency test with 3 and 4 host pipeline slots (the pipeline's
# streams and zstream share the greatest-priority hardware queues).
set -euo pipefail
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
cd "$R"
O=gpurun_out/r06a
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_rx_ring.py tests/test_gpu_rx_bufs.py tests/test_gpu_rx_ring_host.py \
  tests/test_gpu_packet.py tests/test_gpu_tx_host.py -x -v --timeout 120 --timeout-method thread > $O/tests.log 2>&1
timeout -k 10 200 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1
for sl in 3 4; do
  NS_CSUM_HOST_SLOTS=$sl timeout -k 10 200 python -u -m pytest tests/test_gpu_tx_host.py -k does_not_block -v -s \
    --timeout 150 --timeout-method thread > $O/lat_s$sl.log 2>&1 || true
  NS_CSUM_HOST_SLOTS=$sl timeout -k 10 200 python -u -m pytest tests/test_gpu_tx_host.py -k does_not_block -v -s \
    --timeout 150 --timeout-method thread > $O/lat_s${sl}_b.log 2>&1 || true
done
echo done
