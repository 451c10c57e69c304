#!/bin/bash
# Round 6: the header pass with 3 tiles in flight per wave (txv 91) against
# 2 (production), in situ, fresh slots; the first run checks the fill.
set -euo pipefail
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
cd "$R"
O=gpurun_out/r06i
mkdir -p $O
: > $O/depth.jsonl
timeout -k 10 150 python3 -u tools/tx_drain_probe.py --only grp:4:2:none --calls 24 --depth 3 --per-cu 24 >> $O/depth.jsonl 2>> $O/depth.err
for r in 1 2; do
  for d in 2 3; do
    for pc in 16 24; do
      timeout -k 10 120 python3 -u tools/tx_drain_probe.py --only grp:4:2:none --calls 24 --depth $d --per-cu $pc --no-check >> $O/depth.jsonl 2>> $O/depth.err
    done
  done
done
echo done
