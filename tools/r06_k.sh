#!/bin/bash
# Round 6: the TX header pass against a plain copy of its slots with the same
# written-through stores, in situ (after the payload pass, fresh slots).
set -euo pipefail
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
cd "$R"
O=gpurun_out/r06k
mkdir -p $O
: > $O/floor.jsonl
for r in 1 2; do
  timeout -k 10 120 python3 -u tools/tx_drain_probe.py --only grp:4:2:none --calls 24 --no-check >> $O/floor.jsonl 2>> $O/floor.err
  timeout -k 10 120 python3 -u tools/tx_drain_probe.py --only grp:4:2:none --calls 24 --no-check --hfloor >> $O/floor.jsonl 2>> $O/floor.err
done
echo done
