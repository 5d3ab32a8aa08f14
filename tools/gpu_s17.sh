#!/bin/bash
set -e
mkdir -p gpurun_out
LIBS=product,noguess
timeout -k 10 200 python -u tools/variant_bench.py --libs $LIBS --users 1000000 --items 1000000 --dim 64 --rounds 3 > gpurun_out/s17_d64.json 2> gpurun_out/s17.err
timeout -k 10 200 python -u tools/variant_bench.py --libs $LIBS --users 1000000 --items 1250000 --dim 128 --rounds 3 > gpurun_out/s17_shard8.json 2>> gpurun_out/s17.err
timeout -k 10 200 python -u tools/variant_bench.py --libs $LIBS --users 262144 --items 10000000 --dim 128 --rounds 3 > gpurun_out/s17_d128.json 2>> gpurun_out/s17.err
