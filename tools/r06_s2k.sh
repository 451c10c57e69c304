#!/bin/bash
# MTU frames in 1504-, 2048- and 4096-B slots: the product against the
# layout's read floor (variant 50) and all-nontemporal lines (2).
set -eo pipefail
echo "s2k: start"
mkdir -p gpurun_out/s2k
for st in 1504 2048 3072 4096; do
  timeout -k 10 300 python -u tools/rx_ring_probe.py --stride $st --only 0,2,50 2>&1 | tee gpurun_out/s2k/s$st.json
done
