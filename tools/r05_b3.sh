#!/bin/bash
# Round 5, batch 3: why the group payload pass slows when the header pass
# runs between calls (rotating batches): A/B of cache policies, kernel trace.
set -euo pipefail
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
cd "$R"
export TMPDIR=/tmp
mkdir -p gpurun_out/b3
timeout -k 10 300 python3 tools/tx_struct_probe.py --rounds 5 --only struct,struct_winpay,struct_norot,txv_2p_window,txv_2p_window_norot,txv_2p_group,txv_2p_group_norot,txv_2p_grp_ntwb,txv_2p_grp_ntwb_norot > gpurun_out/b3/probe.json 2> gpurun_out/b3/probe.err
echo done
