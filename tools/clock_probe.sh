#!/bin/bash
# Effective shader clock per launch over a bench run (the
# TX run-long slowdown): one rocprofv3 --pmc pass of GRBM_GUI_ACTIVE (summed
# over the 8 XCDs) with the kernel trace, over bench.py --config 8 (TX fill,
# ns_csum_tcp_tx) and --config 7 --rx-layout ring; tools/clock_parse.py
# divides each dispatch's GRBM_GUI_ACTIVE / 8 by its duration
# (MI355X_MICROARCH.md, DVFS give-back).
#   tools/clock_probe.sh TAG
set -euo pipefail
TAG=${1:-r05}
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
OUT=$R/gpurun_out/clock_$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
cd "$R"
timeout -k 10 300 rocprofv3 --pmc GRBM_GUI_ACTIVE GRBM_COUNT --kernel-trace -d "$OUT/cfg8" -o run --output-format csv \
  -- python3 bench.py --config 8 --steps 50 --warmup 5 --no-cpu > "$OUT/cfg8.log" 2>&1
python3 tools/clock_parse.py "$OUT/cfg8" > "$OUT/cfg8_clock.json"
timeout -k 10 300 rocprofv3 --pmc GRBM_GUI_ACTIVE GRBM_COUNT --kernel-trace -d "$OUT/ring" -o run --output-format csv \
  -- python3 bench.py --config 7 --rx-layout ring --steps 50 --warmup 5 --no-cpu > "$OUT/ring.log" 2>&1
python3 tools/clock_parse.py "$OUT/ring" > "$OUT/ring_clock.json"
echo "clock probe $TAG done"
