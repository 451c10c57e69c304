#!/bin/bash
# Buffer lists sorted into address buckets (tools/rx_ring_variants.hip 30-34)
# against the product list kernel (20), shuffled and ring order.
set -e
mkdir -p gpurun_out/rxsort
O=gpurun_out/rxsort
timeout -k 10 240 python -u tools/rx_ring_probe.py --bufs shuffled --only 20,30,31,32,33,34 > $O/shuffled2.json
timeout -k 10 240 python -u tools/rx_ring_probe.py --bufs ring --only 20,30,31,32,33,34 > $O/ring2.json
