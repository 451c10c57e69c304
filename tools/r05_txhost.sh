#!/bin/bash
# Round 5: ns_csum_tcp_tx_host — its GPU tests, the device multi-call tests
# beside them, then the host-inclusive TX bench lines (one call; one call per
# 64 KiB GSO write) and a copy/kernel trace of the latter.
set -euo pipefail
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
cd "$R"
O=gpurun_out/txhost
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_tx_host.py tests/test_gpu_tx_struct.py -x -v --timeout 120 \
  --timeout-method thread > $O/tests.log 2>&1
timeout -k 10 300 python -u bench.py --config 8 --mode host --steps 10 --warmup 2 --cpu-seconds 5 \
  > $O/bench_host8_1call.json 2> $O/bench_host8_1call.err
timeout -k 10 300 python -u bench.py --config 8 --mode host --tx-calls 23832 --steps 10 --warmup 2 --no-cpu \
  > $O/bench_host8_23832calls.json 2> $O/bench_host8_23832calls.err
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --memory-copy-trace --stats -d "$R/$O/trace" -o run -- \
  python -u "$R/bench.py" --config 8 --mode host --tx-calls 23832 --steps 5 --warmup 1 --no-cpu > "$R/$O/trace.log" 2>&1
echo done
