#!/bin/bash
# Round 6: production with the one-shot header pass: TX tests, then bench
# cfg8 interleaved against variant 7 (persistent header pass).
set -euo pipefail
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
cd "$R"
O=gpurun_out/r06n
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_tx_struct.py tests/test_gpu_tx_host.py tests/test_gpu_proto.py tests/test_gpu_tcp.py -x -q --timeout 120 --timeout-method thread > $O/tests.log 2>&1
for r in 1 2 3; do
  for v in 0 7; do
    NS_CSUM_TX_VARIANT=$v timeout -k 10 200 python3 bench.py --config 8 --no-cpu > $O/bench_cfg8_v${v}_$r.json 2> $O/bench_cfg8_v${v}_$r.err
  done
done
echo done
