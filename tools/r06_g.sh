#!/bin/bash
# Round 6: the production header pass's shape (tile x waves per CU) in situ:
# group payload pass, nt sc1 header stores, fresh slots every call.
set -euo pipefail
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
cd "$R"
O=gpurun_out/r06g
mkdir -p $O
: > $O/sweep.jsonl
for ht in 64 32 16; do
  for pc in 24 12 32 48; do
    timeout -k 10 120 python3 -u tools/tx_drain_probe.py --only grp:4:2:none --calls 24 --htile $ht --per-cu $pc --no-check \
      >> $O/sweep.jsonl 2>> $O/sweep.err
  done
done
echo done
