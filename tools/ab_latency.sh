set -e
# Same-box A/B of two builds of the product library on tools/latency.cc:
#   tools/ab_latency.sh ROUNDS ITERS   (A = netstack_amd/lib_prev/, B = the current build)
# Writes gpurun_out/ab_lat/{prev,cur}.N.json, interleaved rounds.
R=${1:-5}; I=${2:-2000}
OUT=gpurun_out/ab_lat
mkdir -p $OUT
cp netstack_amd/lib/libnetstack_csum.so /tmp/cur.so
trap 'cp /tmp/cur.so netstack_amd/lib/libnetstack_csum.so' EXIT
for r in $(seq $R); do
  for v in prev cur; do
    if [ $v = prev ]; then cp netstack_amd/lib_prev/libnetstack_csum.so netstack_amd/lib/libnetstack_csum.so; else cp /tmp/cur.so netstack_amd/lib/libnetstack_csum.so; fi
    timeout -k 10 120 netstack_amd/lib/latency $I > $OUT/$v.$r.json
  done
done
