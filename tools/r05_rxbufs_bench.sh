#!/bin/bash
# Round 5: the buffer-list receive line (ns_csum_rx_bufs, shuffled buffers)
# beside the ring line, and a kernel trace of it.
set -euo pipefail
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
cd "$R"
O=gpurun_out/rxbufs
mkdir -p $O
timeout -k 10 300 python -u bench.py --config 7 --rx-layout bufs --no-cpu > $O/bench_cfg7_bufs.json 2> $O/bench_cfg7_bufs.err
timeout -k 10 300 python -u bench.py --config 7 --rx-layout ring --no-cpu > $O/bench_cfg7_ring.json 2> $O/bench_cfg7_ring.err
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$R/$O/trace" -o run --output-format csv -- \
  python -u "$R/bench.py" --config 7 --rx-layout bufs --no-cpu --steps 20 > "$R/$O/trace.log" 2>&1
echo done
