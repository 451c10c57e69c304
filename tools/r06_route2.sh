#!/bin/bash
# The header pass at 5-8 chunks per lane: TX parity, then the routes again.
set -eo pipefail
echo "route2: start"
mkdir -p gpurun_out/txroute2
timeout -k 10 400 python -u -m pytest tests/test_gpu_tx_struct.py tests/test_gpu_tx_host.py tests/test_gpu_tcp.py -x -q --timeout 200 --timeout-method thread -m gpu 2>&1 | tee gpurun_out/txroute2/tests.log
timeout -k 10 300 python -u tools/tx_route_probe.py 2>&1 | tee gpurun_out/txroute2/routes.jsonl
