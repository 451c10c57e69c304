#!/bin/bash
# cfg2 with shifted packet starts.
set -eo pipefail
echo "align: start"
mkdir -p gpurun_out/align
timeout -k 10 300 python -u tools/align_probe.py 2>&1 | tee gpurun_out/align/align.jsonl
