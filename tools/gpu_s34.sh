#!/bin/bash
# Staged survivor path (d <= 64): tiles whose hitting lanes hold one survivor
# each store the keys directly, vs the product (always staged).
set -e
mkdir -p gpurun_out
LIBS=product,sfast
timeout -k 10 250 python -u tools/variant_bench.py --libs $LIBS --users 1000000 --items 1000000 --dim 64 --rounds 3 > gpurun_out/s34_d64.json 2> gpurun_out/s34.err
timeout -k 10 250 python -u tools/variant_bench.py --libs $LIBS --users 262144 --items 4000000 --dim 64 --rounds 3 > gpurun_out/s34_d64_4m.json 2>> gpurun_out/s34.err
timeout -k 10 250 python -u tools/variant_bench.py --libs $LIBS --users 300000 --items 1000000 --dim 32 --rounds 3 > gpurun_out/s34_d32.json 2>> gpurun_out/s34.err
