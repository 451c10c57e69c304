#!/bin/bash
# Round 5, batch 2: the host pipeline with results written straight to mapped
# memory (parity tests, then cfg3 host-inclusive A/B over slots and the D2H
# knob, and a copy trace), and the TX probe's two-pass shapes under a kernel
# trace (with and without d_out).  Each step under its own time limit.
set -euo pipefail
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
cd "$R"
export TMPDIR=/tmp
mkdir -p gpurun_out/b2
timeout -k 10 500 python -u -m pytest -x -q --timeout 180 --timeout-method thread tests/test_gpu_parity.py > gpurun_out/b2/t.log 2>&1
timeout -k 10 600 bash tools/ab_lib.sh 3 4 > gpurun_out/b2/ab_cfg3.log 2>&1
timeout -k 10 200 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_VMEM_RD -d gpurun_out/b2/c3sq -o run --output-format csv -- python3 tools/pmc_run.py --set cfg3probe > gpurun_out/b2/c3sq.log 2>&1
for sl in 2 3 4; do
  NS_CSUM_HOST_SLOTS=$sl timeout -k 10 120 python3 bench.py --mode host --config 3 --steps 20 --warmup 3 --no-cpu > gpurun_out/b2/h3_s${sl}.json 2> gpurun_out/b2/h3_s${sl}.err
  NS_CSUM_HOST_D2H=1 NS_CSUM_HOST_SLOTS=$sl timeout -k 10 120 python3 bench.py --mode host --config 3 --steps 20 --warmup 3 --no-cpu > gpurun_out/b2/h3_s${sl}_d2h.json 2> gpurun_out/b2/h3_s${sl}_d2h.err
done
timeout -k 10 120 python3 bench.py --mode host --config 2 --steps 10 --warmup 2 --no-cpu > gpurun_out/b2/h2.json 2> gpurun_out/b2/h2.err
timeout -k 10 200 rocprofv3 --kernel-trace --memory-copy-trace --output-format csv -d gpurun_out/b2/h3trace -o run -- python3 bench.py --mode host --config 3 --steps 10 --warmup 3 --no-cpu > gpurun_out/b2/h3trace.json 2> gpurun_out/b2/h3trace.err
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/b2/txtrace -o run -- python3 tools/tx_struct_probe.py --rounds 3 --only struct,struct_out,struct_winpay,struct_norot > gpurun_out/b2/txprobe.json 2> gpurun_out/b2/txprobe.err
echo done
