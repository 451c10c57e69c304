#!/bin/bash
# Round 6: the TX header pass one tile per wave on a one-shot grid (txv 92)
# against the persistent production pass and the copy floor, in situ.
set -euo pipefail
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
cd "$R"
O=gpurun_out/r06l
mkdir -p $O
: > $O/oneshot.jsonl
timeout -k 10 150 python3 -u tools/tx_drain_probe.py --only grp:4:2:none --calls 24 --depth 1 >> $O/oneshot.jsonl 2>> $O/oneshot.err
for r in 1 2; do
  timeout -k 10 120 python3 -u tools/tx_drain_probe.py --only grp:4:2:none --calls 24 --no-check >> $O/oneshot.jsonl 2>> $O/oneshot.err
  timeout -k 10 120 python3 -u tools/tx_drain_probe.py --only grp:4:2:none --calls 24 --no-check --depth 1 >> $O/oneshot.jsonl 2>> $O/oneshot.err
  timeout -k 10 120 python3 -u tools/tx_drain_probe.py --only grp:4:2:none --calls 24 --no-check --hfloor >> $O/oneshot.jsonl 2>> $O/oneshot.err
done
echo done
