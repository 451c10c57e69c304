#!/bin/bash
# Receive-path GPU tests with 4-lane groups on short-slot rings, then smoke.
set -eo pipefail
echo "g4 tests: start"
mkdir -p gpurun_out/rxg4
timeout -k 10 500 python -u -m pytest tests/test_gpu_rx_ring.py tests/test_gpu_rx_ring_host.py tests/test_gpu_rx_bufs.py tests/test_gpu_packet.py -x -q --timeout 200 --timeout-method thread -m gpu 2>&1 | tee gpurun_out/rxg4/tests.log
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" 2>&1 | tee gpurun_out/rxg4/smoke.log
