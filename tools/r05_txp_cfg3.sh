#!/bin/bash
# Round 5: the TX payload pass in 8-lane groups (tests, A/B probe, bench
# cfg8), then cfg3's product instance beside the floor kernels: a kernel
# trace for durations and one SQ counter pass (tools/pmc_run.py --set
# cfg3probe), then the host-inclusive cfg3 pipeline under a copy + kernel
# trace (tools/host_timeline.py); each step under its own time limit.
set -euo pipefail
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
cd "$R"
export TMPDIR=/tmp
mkdir -p gpurun_out/txp gpurun_out/c3
timeout -k 10 400 python -u -m pytest -x -q --timeout 180 --timeout-method thread tests/test_gpu_tx_struct.py tests/test_gpu_parity.py::test_fold_carry_walk_path > gpurun_out/txp/t.log 2>&1
timeout -k 10 300 python3 tools/tx_struct_probe.py --rounds 7 --only struct,struct_winpay,txv_pay_group,txv_pay_window,txv_hdr_pass > gpurun_out/txp/probe.json 2> gpurun_out/txp/probe.err
timeout -k 10 200 python3 bench.py --config 8 > gpurun_out/txp/bench8.json 2> gpurun_out/txp/bench8.err
timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/c3/trace -o run -- python3 tools/pmc_run.py --set cfg3probe > gpurun_out/c3/trace.log 2>&1
timeout -k 10 200 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_VMEM_RD -d gpurun_out/c3/sq -o run --output-format csv -- python3 tools/pmc_run.py --set cfg3probe > gpurun_out/c3/sq.log 2>&1
mkdir -p gpurun_out/h3
timeout -k 10 200 rocprofv3 --kernel-trace --memory-copy-trace --output-format csv -d gpurun_out/h3/trace -o run -- python3 bench.py --mode host --config 3 --steps 10 --warmup 3 --no-cpu > gpurun_out/h3/bench.json 2> gpurun_out/h3/bench.err
for sl in 2 3 4; do
  for ch in 131072 262144; do
    NS_CSUM_HOST_SLOTS=$sl NS_CSUM_HOST_CHUNK=$ch timeout -k 10 120 python3 bench.py --mode host --config 3 --steps 20 --warmup 3 --no-cpu > gpurun_out/h3/ab_s${sl}_c${ch}.json 2> gpurun_out/h3/ab_s${sl}_c${ch}.err
  done
done
echo done
