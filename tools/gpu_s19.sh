#!/bin/bash
# Survivor slots per hit event (product) vs an LDS atomic per key (atomic);
# d=64 also against the direct path (stagedoff).
set -e
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/s19_gpu_tests.log 2>&1
LIBS=product,atomic,stagedoff
timeout -k 10 200 python -u tools/variant_bench.py --libs $LIBS --users 262144 --items 10000000 --dim 128 --rounds 3 > gpurun_out/s19_d128.json 2> gpurun_out/s19.err
timeout -k 10 200 python -u tools/variant_bench.py --libs $LIBS --users 250000 --items 5000000 --dim 128 --rounds 3 > gpurun_out/s19_grid8.json 2>> gpurun_out/s19.err
timeout -k 10 200 python -u tools/variant_bench.py --libs $LIBS --users 1000000 --items 1000000 --dim 64 --rounds 3 > gpurun_out/s19_d64.json 2>> gpurun_out/s19.err
timeout -k 10 200 python -u tools/variant_bench.py --libs $LIBS --users 1000000 --items 1250000 --dim 128 --rounds 3 > gpurun_out/s19_shard8.json 2>> gpurun_out/s19.err
