#!/bin/bash
# rocprofv3 --pmc passes over the receive paths only (tools/pmc_run.py --set
# rx): FETCH_SIZE, WRITE_SIZE, the SQ wave/instruction counters.  Each pass in
# its own run, counters never combined with tracing domains.
#   tools/pmc_rx.sh TAG
set -euo pipefail
TAG=${1:-r05}
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
OUT=$R/gpurun_out/pmcrx_$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
cd "$R"
run() {  # name, counters...
  local name=$1; shift
  timeout -k 10 300 rocprofv3 --pmc "$@" -d "$OUT/$name" -o run --output-format csv \
    -- python3 tools/pmc_run.py --set rx > "$OUT/$name.log" 2>&1
  python3 tools/pmc_parse.py "$OUT/$name" "$OUT/$name.log" > "$OUT/${name}_summary.json"
}
run fetch FETCH_SIZE
run write WRITE_SIZE
run sq SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS
run inst SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_SMEM SQ_LDS_BANK_CONFLICT GRBM_GUI_ACTIVE
echo "pmc rx $TAG done"
