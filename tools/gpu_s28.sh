#!/bin/bash
# Stagger of SIMD partners (waves 4-7 half a stage behind) vs the product.
set -e
mkdir -p gpurun_out
LIBS=product,stag,w48r3
timeout -k 10 200 python -u tools/variant_bench.py --libs $LIBS --users 262144 --items 10000000 --dim 128 --rounds 3 > gpurun_out/s28_10m.json 2> gpurun_out/s28.err
timeout -k 10 200 python -u tools/variant_bench.py --libs $LIBS --users 250000 --items 5000000 --dim 128 --rounds 3 > gpurun_out/s28_5m.json 2>> gpurun_out/s28.err
