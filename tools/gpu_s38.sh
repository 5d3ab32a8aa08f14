#!/bin/bash
# Guessed thresholds at the headline size (1M x 10M, d=128; the product scans
# plain above 2^23 rows): stride 64 / 128 and a 4.5-sigma margin.
set -e
mkdir -p gpurun_out
LIBS=product,g24st64,g24st64s45,g24st128s45
timeout -k 10 400 python -u tools/variant_bench.py --libs $LIBS --users 1000000 --items 10000000 --dim 128 --rounds 2 > gpurun_out/s38_10m.json 2> gpurun_out/s38.err
