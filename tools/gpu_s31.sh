#!/bin/bash
# Compaction slack (keys kept beyond k) 32 (product) vs 0 / 8 / 16.
set -e
mkdir -p gpurun_out
LIBS=product,slack0,slack8,slack16,slack8g64
timeout -k 10 200 python -u tools/variant_bench.py --libs $LIBS --users 1000000 --items 1000000 --dim 64 --rounds 3 > gpurun_out/s31_d64.json 2> gpurun_out/s31.err
timeout -k 10 250 python -u tools/variant_bench.py --libs $LIBS --users 262144 --items 10000000 --dim 128 --rounds 3 > gpurun_out/s31_10m.json 2>> gpurun_out/s31.err
timeout -k 10 250 python -u tools/variant_bench.py --libs $LIBS --users 250000 --items 5000000 --dim 128 --rounds 3 > gpurun_out/s31_5m.json 2>> gpurun_out/s31.err
