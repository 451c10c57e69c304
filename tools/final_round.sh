set -e
mkdir -p gpurun_out/final
for c in 2 3 4 5 7 8; do
  echo "bench cfg$c"
  timeout -k 10 300 python bench.py --config $c > gpurun_out/final/bench_cfg$c.json 2> gpurun_out/final/bench_cfg$c.err
done
echo "host modes"
timeout -k 10 200 python bench.py --mode host --config 2 --no-cpu > gpurun_out/final/bench_host2.json 2>/dev/null
timeout -k 10 200 python bench.py --mode host --config 4 --no-cpu > gpurun_out/final/bench_host4.json 2>/dev/null
echo "profile"
timeout -k 10 900 bash tools/profile.sh r01
echo done
