#!/bin/bash
# 4-lane groups with 16 units per batch on mid-size frames.
set -eo pipefail
echo "g4b: start"
mkdir -p gpurun_out/rxg4b
timeout -k 10 400 python -u tools/rx_size_probe.py --frames 256,400,576,800,1000,1500 --variants 41,42 2>&1 | tee gpurun_out/rxg4b/v4.jsonl
