#!/bin/bash
# Round 5, batch 5: the TX bench-vs-probe gap: 100 back-to-back product calls
# timed one by one (events), then bench cfg8 under a kernel trace.
set -euo pipefail
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
cd "$R"
export TMPDIR=/tmp
mkdir -p gpurun_out/b5
timeout -k 10 300 python3 tools/tx_struct_probe.py --rounds 2 --only struct --trend 100 > gpurun_out/b5/trend.json 2> gpurun_out/b5/trend.err
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/b5/trace -o run -- python3 bench.py --config 8 --no-cpu > gpurun_out/b5/bench8.json 2> gpurun_out/b5/bench8.err
echo done
