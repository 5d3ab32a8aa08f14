#!/bin/bash
# Staged survivors (d <= 64): short blocks (a one-survivor lane stages its max
# only) vs the product's 16-score blocks.
set -e
mkdir -p gpurun_out
LIBS=product,short
timeout -k 10 250 python -u tools/variant_bench.py --libs $LIBS --users 1000000 --items 1000000 --dim 64 --rounds 3 > gpurun_out/s43_d64.json 2> gpurun_out/s43.err
timeout -k 10 250 python -u tools/variant_bench.py --libs $LIBS --users 300000 --items 1000000 --dim 32 --rounds 3 > gpurun_out/s43_d32.json 2>> gpurun_out/s43.err
timeout -k 10 250 python -u tools/variant_bench.py --libs $LIBS --users 262144 --items 4000000 --dim 64 --rounds 3 > gpurun_out/s43_d64_4m.json 2>> gpurun_out/s43.err
