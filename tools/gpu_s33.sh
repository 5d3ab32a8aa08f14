#!/bin/bash
# Direct survivor enqueue (d = 128): one-survivor lanes store their max without
# the 16-way value select, vs the product.
set -e
mkdir -p gpurun_out
LIBS=product,fast
timeout -k 10 250 python -u tools/variant_bench.py --libs $LIBS --users 262144 --items 10000000 --dim 128 --rounds 3 > gpurun_out/s33_10m.json 2> gpurun_out/s33.err
timeout -k 10 250 python -u tools/variant_bench.py --libs $LIBS --users 250000 --items 5000000 --dim 128 --rounds 3 > gpurun_out/s33_5m.json 2>> gpurun_out/s33.err
timeout -k 10 250 python -u tools/variant_bench.py --libs $LIBS --users 1000000 --items 1250000 --dim 128 --rounds 3 > gpurun_out/s33_1m25.json 2>> gpurun_out/s33.err
