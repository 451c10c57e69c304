#!/bin/bash
# TX over IPv4 and IPv6 routes; the oracle-free cross-checks of two tools.
set -eo pipefail
echo "route probe: start"
mkdir -p gpurun_out/txroute
timeout -k 10 300 python -u tools/tx_route_probe.py 2>&1 | tee gpurun_out/txroute/routes.jsonl
timeout -k 10 120 python -u tools/tx_multi_probe.py --calls 200 --rounds 3 2>&1 | tee gpurun_out/txroute/multi.log
timeout -k 10 120 python -u tools/single_buffer_probe.py 2>&1 | tee gpurun_out/txroute/single.log
