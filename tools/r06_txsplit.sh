#!/bin/bash
# The TX passes one by one across segment sizes: 8-lane (28) and 4-lane (93)
# payload passes.
set -eo pipefail
echo "txsplit: start"
mkdir -p gpurun_out/txsplit
timeout -k 10 500 python -u tools/tx_route_probe.py --mss 64,128,256,536 --split --rounds 3 --reps 10 2>&1 | tee gpurun_out/txsplit/pay28.jsonl
timeout -k 10 500 python -u tools/tx_route_probe.py --mss 64,128,256,536 --split --pay-variant 93 --rounds 3 --reps 10 2>&1 | tee gpurun_out/txsplit/pay93.jsonl
