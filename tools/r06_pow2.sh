#!/bin/bash
# Power-of-two slot strides: the product (line 0 nontemporal on 128-B-aligned
# slots) against variant 0 (line 0 default policy).
set -eo pipefail
echo "pow2: start"
mkdir -p gpurun_out/rxpow2
timeout -k 10 400 python -u tools/rx_size_probe.py --frames 1000,1512,2032,4080 --variants 0,14 --rounds 7 2>&1 | tee gpurun_out/rxpow2/v4.jsonl
