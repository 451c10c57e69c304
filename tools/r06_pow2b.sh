#!/bin/bash
# After the stride rule: the receive tests, then 1536/2048-B strides again.
set -eo pipefail
echo "pow2b: start"
mkdir -p gpurun_out/rxpow2b
timeout -k 10 400 python -u -m pytest tests/test_gpu_rx_ring.py tests/test_gpu_rx_ring_host.py -x -q --timeout 200 --timeout-method thread -m gpu 2>&1 | tee gpurun_out/rxpow2b/tests.log
timeout -k 10 300 python -u tools/rx_size_probe.py --frames 1512,2032 --variants 0 --rounds 7 2>&1 | tee gpurun_out/rxpow2b/v4.jsonl
