#!/bin/bash
# The receive ring across frame sizes (IPv4, and IPv6 at 1500 / 9000 B).
set -eo pipefail
echo "sizes: start"
mkdir -p gpurun_out/rxsizes
timeout -k 10 400 python -u tools/rx_size_probe.py 2>&1 | tee gpurun_out/rxsizes/v4.jsonl
timeout -k 10 300 python -u tools/rx_size_probe.py --v6 --frames 1500,9000 2>&1 | tee gpurun_out/rxsizes/v6.jsonl
