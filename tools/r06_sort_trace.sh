#!/bin/bash
# Per-kernel durations of the bucket-sorted buffer list (variant 30).
set -e
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out/rxsort
for o in shuffled ring; do
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/rxsort/trace_$o -o run -- python3 $R/tools/rx_ring_probe.py --bufs $o --only 30 --rounds 2 --reps 10 > $R/gpurun_out/rxsort/trace_$o.json
done
