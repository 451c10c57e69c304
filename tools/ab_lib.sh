set -e
# Same-box A/B of two builds of the product library on one bench config:
#   tools/ab_lib.sh CONFIG ROUNDS   (A = netstack_amd/lib_prev/, B = the current build)
C=${1:-3}; R=${2:-3}
OUT=gpurun_out/ab
mkdir -p $OUT
cp netstack_amd/lib/libnetstack_csum.so /tmp/cur.so
for r in $(seq $R); do
  for v in prev cur; do
    if [ $v = prev ]; then cp netstack_amd/lib_prev/libnetstack_csum.so netstack_amd/lib/libnetstack_csum.so; else cp /tmp/cur.so netstack_amd/lib/libnetstack_csum.so; fi
    timeout -k 10 200 python bench.py --config $C --no-cpu > $OUT/cfg$C.$v.$r.json 2>/dev/null
  done
done
cp /tmp/cur.so netstack_amd/lib/libnetstack_csum.so
