#!/bin/bash
# Round 6: the TX fill's two passes timed one by one under every header-store
# policy, payload-pass shape, rotation and between-call gap
# (tools/tx_drain_probe.py), then per-dispatch PMC passes over five of them.
set -euo pipefail
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
cd "$R"
export TMPDIR=/tmp
O=gpurun_out/r06b
mkdir -p $O
timeout -k 10 300 python3 -u tools/tx_drain_probe.py > $O/drain.jsonl 2> $O/drain.err
SC=win:0:2:none,grp:0:2:none,grp:0:1:none,grp:1:2:none,grp:0:2:flush
i=0
for pmc in "FETCH_SIZE" "WRITE_SIZE" \
           "TCC_EA0_RDREQ_DRAM_CREDIT_STALL_sum TCC_EA0_WRREQ_DRAM_CREDIT_STALL_sum TCC_EA0_WRREQ_STALL_sum" \
           "TCC_NORMAL_WRITEBACK_sum TCC_ALL_TC_OP_WB_WRITEBACK_sum TCC_EA0_WRREQ_64B_sum"; do
  i=$((i + 1))
  timeout -s KILL 180 rocprofv3 --pmc $pmc -d $O/pmc$i -o run --output-format csv -- \
    python3 tools/tx_drain_probe.py --only $SC --calls 6 --warmup 2 --no-check > $O/pmc$i.log 2>&1
done
python3 tools/tx_drain_parse.py --only $SC --calls 6 --warmup 2 $O/pmc1 $O/pmc2 $O/pmc3 $O/pmc4 > $O/pmc.jsonl
echo done
