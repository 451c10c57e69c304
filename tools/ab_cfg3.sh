set -e
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 300 --timeout-method thread > gpurun_out/r3_parity_quad.log 2>&1 || { tail -30 gpurun_out/r3_parity_quad.log; exit 1; }
tail -2 gpurun_out/r3_parity_quad.log
bash tools/ab_lib.sh 3 4
python3 - <<'PY'
import json,glob,statistics
for v in ("prev","cur"):
    xs=[json.load(open(f))["roofline"]["avg_launch_us"] for f in sorted(glob.glob(f"gpurun_out/ab/cfg3.{v}.*.json"))]
    print(v, [round(x,2) for x in xs], "median", round(statistics.median(xs),2))
PY
timeout -k 10 120 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_INSTS_SALU SQ_INSTS_VALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_ACTIVE_INST_VALU -d gpurun_out/pmc_cfg3b -o run --output-format csv -- python3 tools/pmc_run.py --set cfg3probe > gpurun_out/pmc_cfg3b.log 2>&1
python3 tools/pmc_parse.py gpurun_out/pmc_cfg3b gpurun_out/pmc_cfg3b.log > gpurun_out/cfg3b_sq.json
