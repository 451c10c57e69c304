#!/bin/bash
# Round 6: SQ / LDS counters of the TX header pass in situ (per dispatch).
set -euo pipefail
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
cd "$R"
export TMPDIR=/tmp
O=gpurun_out/r06j
mkdir -p $O
SC=grp:4:2:none
i=0
for pmc in "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_INSTS_VALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT" \
           "SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_SALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VALU SQ_INST_CYCLES_VMEM_WR SQ_WAIT_INST_LDS SQ_LDS_IDX_ACTIVE" \
           "TCP_PENDING_STALL_CYCLES_sum TCP_TCC_WRITE_REQ_sum TCP_TCC_READ_REQ_sum TD_TC_STALL_sum TA_BUSY_avr GRBM_GUI_ACTIVE"; do
  i=$((i + 1))
  timeout -s KILL 180 rocprofv3 --pmc $pmc -d $O/p$i -o run --output-format csv -- \
    python3 tools/tx_drain_probe.py --only $SC --calls 6 --warmup 2 --no-check > $O/p$i.log 2>&1
done
python3 tools/tx_drain_parse.py --only $SC --calls 6 --warmup 2 $O/p1 $O/p2 $O/p3 > $O/sq.jsonl
echo done
