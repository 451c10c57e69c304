#!/bin/bash
# Round 5, batch 4: the windowed payload pass back as the default (group
# pass = variant 5): TX tests, the probe (rotating and not), bench cfg8 over
# two rotating batches.
set -euo pipefail
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
cd "$R"
export TMPDIR=/tmp
mkdir -p gpurun_out/b4
timeout -k 10 400 python -u -m pytest -x -q --timeout 180 --timeout-method thread tests/test_gpu_tx_struct.py > gpurun_out/b4/t.log 2>&1
timeout -k 10 300 python3 tools/tx_struct_probe.py --rounds 5 --only struct,struct_grppay,struct_norot,txv_2p_group_norot,txv_pay_group,txv_pay_window,txv_hdr_pass > gpurun_out/b4/probe.json 2> gpurun_out/b4/probe.err
timeout -k 10 200 python3 bench.py --config 8 > gpurun_out/b4/bench8.json 2> gpurun_out/b4/bench8.err
echo done
