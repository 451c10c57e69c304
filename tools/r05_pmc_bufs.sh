#!/bin/bash
# Round 5: HBM traffic of the receive paths, the buffer list included
# (FETCH_SIZE and WRITE_SIZE in passes of their own over pmc_run.py --set rx).
set -euo pipefail
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
OUT=$R/gpurun_out/pmc_bufs
mkdir -p "$OUT"
export TMPDIR=/tmp
cd "$R"
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE -d "$OUT/fetch" -o run --output-format csv \
  -- python3 tools/pmc_run.py --set rx > "$OUT/fetch.log" 2>&1
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE -d "$OUT/write" -o run --output-format csv \
  -- python3 tools/pmc_run.py --set rx > "$OUT/write.log" 2>&1
python3 tools/pmc_parse.py "$OUT/fetch" "$OUT/fetch.log" > "$OUT/fetch_summary.json"
python3 tools/pmc_parse.py "$OUT/write" "$OUT/write.log" > "$OUT/write_summary.json"
echo done
