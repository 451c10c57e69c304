#!/bin/bash
# Round 6: the TX fill with the group payload pass and written-through header
# stores as production: its GPU tests, bench cfg8 (rotating) three times
# beside round 5's production (variant 6), a kernel trace of the bench, and
# the per-dispatch PMC passes over the new production scenario; buffer-list
# cache-policy variants.
set -euo pipefail
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
cd "$R"
export TMPDIR=/tmp
O=gpurun_out/r06c
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_tx_struct.py tests/test_gpu_tx_host.py tests/test_gpu_proto.py \
  -x -v --timeout 120 --timeout-method thread > $O/tests.log 2>&1
for r in 1 2 3; do
  timeout -k 10 200 python3 bench.py --config 8 --no-cpu > $O/bench_cfg8_$r.json 2> $O/bench_cfg8_$r.err
  NS_CSUM_TX_VARIANT=6 timeout -k 10 200 python3 bench.py --config 8 --no-cpu > $O/bench_cfg8_v6_$r.json 2> $O/bench_cfg8_v6_$r.err
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/trace8 -o run --output-format csv \
  -- python3 bench.py --config 8 --steps 50 --warmup 5 --no-cpu > $O/bench_cfg8_traced.json 2> $O/bench_cfg8_traced.err
timeout -k 10 300 python3 -u tools/tx_drain_probe.py --only grp:4:2:none,win:0:2:none,grp:4:1:none,win:4:2:none,grp:4:2:flush \
  > $O/drain.jsonl 2> $O/drain.err
SC=grp:4:2:none,grp:6:2:none,win:0:2:none
i=0
for pmc in "FETCH_SIZE" "WRITE_SIZE" \
           "TCC_EA0_RDREQ_DRAM_CREDIT_STALL_sum TCC_EA0_WRREQ_DRAM_CREDIT_STALL_sum TCC_EA0_WRREQ_STALL_sum" \
           "TCC_NORMAL_WRITEBACK_sum TCC_ALL_TC_OP_WB_WRITEBACK_sum TCC_EA0_WRREQ_64B_sum"; do
  i=$((i + 1))
  timeout -s KILL 180 rocprofv3 --pmc $pmc -d $O/pmc$i -o run --output-format csv -- \
    python3 tools/tx_drain_probe.py --only $SC --calls 6 --warmup 2 --no-check > $O/pmc$i.log 2>&1
done
python3 tools/tx_drain_parse.py --only $SC --calls 6 --warmup 2 $O/pmc1 $O/pmc2 $O/pmc3 $O/pmc4 > $O/pmc.jsonl
# buffer lists: cache policies of lines >= 1 over a shuffled pool (and the ring order)
timeout -k 10 300 python3 tools/rx_ring_probe.py --bufs shuffled --rounds 5 > $O/bufs_shuffled.json 2> $O/bufs_shuffled.err
timeout -k 10 200 python3 tools/rx_ring_probe.py --bufs ring --rounds 3 --only 20,21 > $O/bufs_ring.json 2> $O/bufs_ring.err
echo done
