#!/bin/bash
# GPU tests on the new stage geometry + A/B of d=128 stage sizes:
# product (2 x 64 KB) vs w32r3 (3 x 32 KB, the previous product) vs w48r3 (3 x 48 KB).
set -e
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/s10_gpu_tests.log 2>&1
LIBS=product,w32r3,w48r3
timeout -k 10 200 python -u tools/variant_bench.py --libs $LIBS --users 1000000 --items 1250000 --dim 128 --rounds 3 > gpurun_out/s10_shard8.json 2> gpurun_out/s10_shard8.err
timeout -k 10 200 python -u tools/variant_bench.py --libs $LIBS --users 262144 --items 10000000 --dim 128 --rounds 3 > gpurun_out/s10_d128.json 2> gpurun_out/s10_d128.err
timeout -k 10 200 python -u tools/variant_bench.py --libs $LIBS --users 1000000 --items 2500000 --dim 128 --rounds 3 > gpurun_out/s10_shard4.json 2> gpurun_out/s10_shard4.err
