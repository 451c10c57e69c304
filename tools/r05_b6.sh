#!/bin/bash
# Round 5, batch 6: csum_grp (MTU-sized tables in 8-lane groups): its parity
# tests and the batch parity suite, then cfg2 / cfg7 / cfg5-shard A/B against
# the previous library (netstack_amd/lib_prev, csum_hyb for every table).
set -euo pipefail
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
cd "$R"
export TMPDIR=/tmp
mkdir -p gpurun_out/b6
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_grp.py tests/test_gpu_parity.py > gpurun_out/b6/t.log 2>&1
timeout -k 10 600 bash tools/ab_lib.sh 2 4 > gpurun_out/b6/ab2.log 2>&1
echo done
