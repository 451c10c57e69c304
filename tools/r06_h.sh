#!/bin/bash
# Round 6: buffer lists, last line default, the other lines >= 1 under each
# cache-policy combination (does any keep the interior out of the MALL?).
set -euo pipefail
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
cd "$R"
O=gpurun_out/r06h
mkdir -p $O
timeout -k 10 300 python3 tools/rx_ring_probe.py --bufs shuffled --rounds 5 --only 20,24,26,27,28,29 > $O/bufs_shuffled_policies.json 2> $O/bufs.err
echo done
