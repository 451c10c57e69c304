#!/bin/bash
# Round 5: the ring and the buffer list in ring order, interleaved on one box.
set -euo pipefail
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
cd "$R"
O=gpurun_out/bufs_ab
mkdir -p $O
for i in 1 2; do
  timeout -k 10 200 python -u bench.py --config 7 --rx-layout ring --no-cpu > $O/ring_$i.json 2>/dev/null
  timeout -k 10 200 python -u bench.py --config 7 --rx-layout bufs --bufs-order ring --no-cpu > $O/bufs_$i.json 2>/dev/null
done
echo done
