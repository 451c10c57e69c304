set -e
# Every bench line of a round, on the GPU box: tools/final_round.sh TAG
TAG=${1:-r06}
OUT=gpurun_out/final_$TAG
mkdir -p $OUT
for c in 1 2 3 4 5 7 8; do
  echo "bench cfg$c"
  timeout -k 10 300 python bench.py --config $c > $OUT/bench_cfg$c.json 2> $OUT/bench_cfg$c.err
done
echo "bench cfg7 as a receive ring (ns_csum_rx_ring) and as a buffer list (ns_csum_rx_bufs), shuffled and in ring order"
timeout -k 10 300 python bench.py --config 7 --rx-layout ring > $OUT/bench_cfg7_ring.json 2> $OUT/bench_cfg7_ring.err
timeout -k 10 300 python bench.py --config 7 --rx-layout bufs --no-cpu > $OUT/bench_cfg7_bufs.json 2> $OUT/bench_cfg7_bufs.err
timeout -k 10 300 python bench.py --config 7 --rx-layout bufs --bufs-order ring --no-cpu > $OUT/bench_cfg7_bufs_ring.json 2> $OUT/bench_cfg7_bufs_ring.err
echo "bench cfg8 paired table and wire layout"
timeout -k 10 300 python bench.py --config 8 --tx-layout split > $OUT/bench_cfg8_split.json 2> $OUT/bench_cfg8_split.err
timeout -k 10 300 python bench.py --config 8 --tx-layout wire > $OUT/bench_cfg8_wire.json 2> $OUT/bench_cfg8_wire.err
echo "host modes"
for c in 2 3 4; do
  timeout -k 10 200 python bench.py --mode host --config $c --no-cpu --no-parity > $OUT/bench_host$c.json 2>/dev/null
done
echo "host RX ring (ns_csum_rx_ring_host)"
timeout -k 10 300 python bench.py --mode host --config 7 --rx-layout ring --steps 10 --warmup 2 \
  > $OUT/bench_host7_ring.json 2>/dev/null
echo "host TX (ns_csum_tcp_tx_host): one call, and one call per 64 KiB GSO write"
timeout -k 10 300 python bench.py --mode host --config 8 --steps 10 --warmup 2 --cpu-seconds 5 > $OUT/bench_host8.json 2>/dev/null
timeout -k 10 300 python bench.py --mode host --config 8 --tx-calls 23832 --steps 10 --warmup 2 --no-cpu \
  > $OUT/bench_host8_23832calls.json 2>/dev/null
echo done
