#!/bin/bash
# Guessed thresholds: sample stride 16 / 64 and a 4.5-sigma margin vs the
# product (stride 32, 6 sigma).
set -e
mkdir -p gpurun_out
LIBS=product,st16,st64,sig45,st64s45
timeout -k 10 250 python -u tools/variant_bench.py --libs $LIBS --users 1000000 --items 1000000 --dim 64 --rounds 3 > gpurun_out/s37_d64.json 2> gpurun_out/s37.err
timeout -k 10 250 python -u tools/variant_bench.py --libs $LIBS --users 250000 --items 5000000 --dim 128 --rounds 3 > gpurun_out/s37_5m.json 2>> gpurun_out/s37.err
timeout -k 10 250 python -u tools/variant_bench.py --libs $LIBS --users 1000000 --items 1250000 --dim 128 --rounds 3 > gpurun_out/s37_1m25.json 2>> gpurun_out/s37.err
