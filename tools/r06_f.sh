#!/bin/bash
# Round 6: buffer lists with each packet's last line at the default policy
# (variants 24 / 25) against the product list shape, shuffled and ring order.
set -euo pipefail
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
cd "$R"
O=gpurun_out/r06f
mkdir -p $O
timeout -k 10 300 python3 tools/rx_ring_probe.py --bufs shuffled --rounds 5 --only 20,24,25,21 > $O/bufs_shuffled_ll.json 2> $O/bufs_shuffled_ll.err
timeout -k 10 200 python3 tools/rx_ring_probe.py --bufs ring --rounds 3 --only 20,24 > $O/bufs_ring_ll.json 2> $O/bufs_ring_ll.err
echo done
