#!/bin/bash
# The receive ring behind Ethernet headers (link_hdr 14) against TUN framing.
set -eo pipefail
echo "eth: start"
mkdir -p gpurun_out/rxeth
timeout -k 10 300 python -u tools/rx_size_probe.py --frames 64,1500,9000 2>&1 | tee gpurun_out/rxeth/tun.jsonl
timeout -k 10 300 python -u tools/rx_size_probe.py --frames 64,1500,9000 --eth 2>&1 | tee gpurun_out/rxeth/eth.jsonl
