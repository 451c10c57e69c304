#!/bin/bash
# 4-lane groups on rings of short frames (tools/rx_ring_variants.hip 40, 41).
set -eo pipefail
echo "g4: start"
mkdir -p gpurun_out/rxg4
timeout -k 10 400 python -u tools/rx_size_probe.py --frames 64,128,256,576 --variants 40,41 2>&1 | tee gpurun_out/rxg4/v4.jsonl
timeout -k 10 300 python -u tools/rx_size_probe.py --frames 64,256 --variants 40,41 --v6 2>&1 | tee gpurun_out/rxg4/v6.jsonl
