#!/bin/bash
set -e
mkdir -p gpurun_out
LIBS=product,w72,gap64,gap160
timeout -k 10 200 python -u tools/variant_bench.py --libs $LIBS --users 262144 --items 10000000 --dim 128 --rounds 3 > gpurun_out/s21_d128.json 2> gpurun_out/s21.err
timeout -k 10 200 python -u tools/variant_bench.py --libs $LIBS --users 250000 --items 5000000 --dim 128 --rounds 3 > gpurun_out/s21_grid8.json 2>> gpurun_out/s21.err
