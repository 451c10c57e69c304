#!/bin/bash
# The receive ring and buffer list over IPv6/TCP frames beside IPv4/TCP.
set -eo pipefail
echo "v6 probe: start"
mkdir -p gpurun_out/rxv6
timeout -k 10 240 python -u tools/rx_ring_probe.py --only 0 2>&1 | tee gpurun_out/rxv6/ring_v4.json
timeout -k 10 240 python -u tools/rx_ring_probe.py --only 0 --ipv6 2>&1 | tee gpurun_out/rxv6/ring_v6.json
timeout -k 10 240 python -u tools/rx_ring_probe.py --bufs ring --only 20 --ipv6 2>&1 | tee gpurun_out/rxv6/bufs_ring_v6.json
timeout -k 10 200 python -u -m pytest tests/test_gpu_rx_ring.py -x -q --timeout 120 --timeout-method thread -m gpu -k full_size_ring 2>&1 | tee gpurun_out/rxv6/full_size_test.log
