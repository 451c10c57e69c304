#!/bin/bash
# Collect the rocprofv3 evidence for one round on the GPU box:
#   tools/profile.sh TAG
# 1. kernel trace + stats of the default bench.py run (timing)
# 2. separate --pmc passes over tools/pmc_run.py — counters are never
#    combined with tracing domains:
#    FETCH_SIZE and WRITE_SIZE over every bench config (--set main), the SQ
#    wave / instruction counters, and the SQ counters of cfg3's product
#    instance beside the floor kernels (--set cfg3probe).
set -euo pipefail
TAG=${1:-r03}
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
OUT=$R/gpurun_out/prof_$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
cd "$R"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$OUT/trace" -o run --output-format csv \
  -- python3 bench.py --steps 50 --warmup 5 --no-cpu > "$OUT/bench_traced.log" 2>&1
python3 tools/trace_summary.py "$OUT/trace" --warmup 5 --steps 50 > "$OUT/trace_summary.json"
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE -d "$OUT/pmc_fetch" -o run --output-format csv \
  -- python3 tools/pmc_run.py > "$OUT/pmc_fetch.log" 2>&1
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE -d "$OUT/pmc_write" -o run --output-format csv \
  -- python3 tools/pmc_run.py > "$OUT/pmc_write.log" 2>&1
timeout -k 10 300 rocprofv3 --pmc SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS \
  -d "$OUT/pmc_sq" -o run --output-format csv -- python3 tools/pmc_run.py > "$OUT/pmc_sq.log" 2>&1
timeout -k 10 300 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE GRBM_GUI_ACTIVE \
  -d "$OUT/pmc_inst" -o run --output-format csv -- python3 tools/pmc_run.py > "$OUT/pmc_inst.log" 2>&1
timeout -k 10 300 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_INSTS_SALU SQ_INSTS_VALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_SMEM \
  -d "$OUT/pmc_cfg3" -o run --output-format csv -- python3 tools/pmc_run.py --set cfg3probe > "$OUT/pmc_cfg3.log" 2>&1
python3 tools/pmc_parse.py "$OUT/pmc_fetch" "$OUT/pmc_fetch.log" > "$OUT/fetch_summary.json"
python3 tools/pmc_parse.py "$OUT/pmc_write" "$OUT/pmc_write.log" > "$OUT/write_summary.json"
python3 tools/pmc_parse.py "$OUT/pmc_sq" "$OUT/pmc_sq.log" > "$OUT/sq_summary.json"
python3 tools/pmc_parse.py "$OUT/pmc_inst" "$OUT/pmc_inst.log" > "$OUT/inst_summary.json"
python3 tools/pmc_parse.py "$OUT/pmc_cfg3" "$OUT/pmc_cfg3.log" > "$OUT/cfg3_sq_summary.json"
echo "profile $TAG done"
