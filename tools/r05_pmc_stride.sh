#!/bin/bash
# Round 5: FETCH_SIZE of the ring kernel at 1504- and 1536-B slot spacing
# (tools/rx_ring_probe.py, product shape only), one pass each.
set -euo pipefail
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
OUT=$R/gpurun_out/pmc_stride
mkdir -p "$OUT"
export TMPDIR=/tmp
cd "$R"
for st in 1504 1536; do
  timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE -d "$OUT/f$st" -o run --output-format csv \
    -- python3 tools/rx_ring_probe.py --stride $st --only 0 --rounds 2 --reps 10 > "$OUT/f$st.log" 2>&1
done
echo done
