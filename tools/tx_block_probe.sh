set -e
# TX fill timing probe: product 2-B stores vs whole aligned 64-B / 128-B block
# stores (wrong bytes; timing only), interleaved rounds on one box.
# The probe libraries were csum_kernels.hip with, at the top of store_result, a
# block of NSK_PROBE_BLOCK bytes written with uint4 stores instead of the field
# (reverted after the measurement), built with -DNSK_PROBE_BLOCK=64 / 128 into
# netstack_amd/lib_probe64/ and lib_probe128/.  Result:
# profiles/r02/tx_store_sector_probe.txt.
OUT=gpurun_out/txp
mkdir -p $OUT
cp netstack_amd/lib/libnetstack_csum.so /tmp/prod.so
timeout -k 10 200 python bench.py --config 7 --no-cpu > $OUT/rx.json 2>/dev/null
for round in 1 2 3; do
  for v in prod 64 128; do
    if [ $v = prod ]; then cp /tmp/prod.so netstack_amd/lib/libnetstack_csum.so; else cp netstack_amd/lib_probe$v/libnetstack_csum.so netstack_amd/lib/libnetstack_csum.so; fi
    timeout -k 10 200 python bench.py --config 8 --no-cpu > $OUT/$v.$round.json 2>/dev/null
    echo "$v $round done"
  done
done
cp /tmp/prod.so netstack_amd/lib/libnetstack_csum.so
