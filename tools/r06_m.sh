#!/bin/bash
# Round 6: the one-shot header pass at 1 / 2 / 4 waves per workgroup against
# the persistent pass and the copy floor, in situ, interleaved rounds.
set -euo pipefail
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
cd "$R"
O=gpurun_out/r06m
mkdir -p $O
: > $O/oneshot.jsonl
for wpg in 1 2; do
  timeout -k 10 150 python3 -u tools/tx_drain_probe.py --only grp:4:2:none --calls 8 --depth 1 --per-cu $wpg >> $O/oneshot.jsonl 2>> $O/oneshot.err
done
for r in 1 2 3; do
  for v in "" "--depth 1 --per-cu 1" "--depth 1 --per-cu 2" "--depth 1 --per-cu 4" "--hfloor"; do
    timeout -k 10 120 python3 -u tools/tx_drain_probe.py --only grp:4:2:none --calls 24 --no-check $v >> $O/oneshot.jsonl 2>> $O/oneshot.err
  done
done
echo done
