#!/bin/bash
# Round 6: cfg4's counters per byte beside the two access shapes it reads in
# (tools/pmc_run.py --set cfg4probe), one --pmc pass per counter group.
set -euo pipefail
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
cd "$R"
export TMPDIR=/tmp
O=gpurun_out/r06e
mkdir -p $O
i=0
for pmc in "FETCH_SIZE" \
           "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_VMEM_RD GRBM_GUI_ACTIVE" \
           "TCP_READ_TAGCONFLICT_STALL_CYCLES_sum TCP_PENDING_STALL_CYCLES_sum TCP_TCC_READ_REQ_sum TCP_TOTAL_READ_sum TD_TC_STALL_sum TA_BUSY_avr" \
           "TCC_HIT_sum TCC_MISS_sum TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_DRAM_CREDIT_STALL_sum"; do
  i=$((i + 1))
  timeout -s KILL 240 rocprofv3 --pmc $pmc -d $O/p$i -o run --output-format csv -- \
    python3 tools/pmc_run.py --set cfg4probe > $O/p$i.log 2>&1
  python3 tools/pmc_parse.py $O/p$i $O/p$i.log > $O/p$i.json
done
timeout -k 10 300 python3 tools/cfg4_split.py --rounds 5 --json $O/cfg4_split.json > $O/cfg4_split.log 2>&1
echo done
