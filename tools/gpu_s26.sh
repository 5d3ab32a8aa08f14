#!/bin/bash
set -e
mkdir -p gpurun_out
LIBS=product,g23,g24
timeout -k 10 200 python -u tools/variant_bench.py --libs $LIBS --users 250000 --items 5000000 --dim 128 --rounds 3 > gpurun_out/s26_5m.json 2> gpurun_out/s26.err
timeout -k 10 200 python -u tools/variant_bench.py --libs $LIBS --users 262144 --items 10000000 --dim 128 --rounds 3 > gpurun_out/s26_10m.json 2>> gpurun_out/s26.err
