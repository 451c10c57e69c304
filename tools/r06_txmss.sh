#!/bin/bash
# ns_csum_tcp_tx across segment sizes (IPv4 route).
set -eo pipefail
echo "tx mss: start"
mkdir -p gpurun_out/txmss
timeout -k 10 500 python -u tools/tx_route_probe.py --mss 64,256,536,1460,8960 2>&1 | tee gpurun_out/txmss/mss.jsonl
