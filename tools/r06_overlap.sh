#!/bin/bash
# TX passes over parts of the batch, header passes on a second stream.
set -eo pipefail
echo "overlap probe: start"
mkdir -p gpurun_out/txoverlap
timeout -k 10 240 python -u tools/tx_overlap_probe.py --parts 1,2,4,8 2>&1 | tee gpurun_out/txoverlap/normal.jsonl
timeout -k 10 240 python -u tools/tx_overlap_probe.py --parts 1,2,4,8 --prio 2>&1 | tee gpurun_out/txoverlap/prio.jsonl
