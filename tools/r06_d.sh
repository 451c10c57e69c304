#!/bin/bash
# Round 6: the one-pass group TX variants (7: written-through slot stores,
# 8: default-policy stores) against production, bench cfg8 interleaved.
set -euo pipefail
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
cd "$R"
O=gpurun_out/r06d
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_tx_struct.py -x -q --timeout 120 --timeout-method thread > $O/tests.log 2>&1
for r in 1 2 3; do
  for v in 0 7 8; do
    NS_CSUM_TX_VARIANT=$v timeout -k 10 200 python3 bench.py --config 8 --no-cpu > $O/bench_cfg8_v${v}_$r.json 2> $O/bench_cfg8_v${v}_$r.err
  done
done
echo done
