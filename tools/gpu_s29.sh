#!/bin/bash
# d <= 64: eight user tiles per wave (2048 users per workgroup, two groups of
# four scored against each item tile) vs the product's four.
set -e
mkdir -p gpurun_out
LIBS=product,nut8,nut8d
timeout -k 10 200 python -u tools/variant_bench.py --libs $LIBS --users 1000000 --items 1000000 --dim 64 --rounds 3 > gpurun_out/s29_d64.json 2> gpurun_out/s29.err
timeout -k 10 200 python -u tools/variant_bench.py --libs $LIBS --users 262144 --items 4000000 --dim 64 --rounds 3 > gpurun_out/s29_d64_4m.json 2>> gpurun_out/s29.err
timeout -k 10 200 python -u tools/variant_bench.py --libs $LIBS --users 300000 --items 1000000 --dim 32 --rounds 3 > gpurun_out/s29_d32.json 2>> gpurun_out/s29.err
