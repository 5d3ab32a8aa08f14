#!/bin/bash
# d <= 64: per-user thresholds in LDS (frees 8 VGPRs, spills 64 -> 16 B) vs
# registers (product).
set -e
mkdir -p gpurun_out
LIBS=product,thrlds
timeout -k 10 250 python -u tools/variant_bench.py --libs $LIBS --users 1000000 --items 1000000 --dim 64 --rounds 3 > gpurun_out/s44_d64.json 2> gpurun_out/s44.err
timeout -k 10 250 python -u tools/variant_bench.py --libs $LIBS --users 300000 --items 1000000 --dim 32 --rounds 3 > gpurun_out/s44_d32.json 2>> gpurun_out/s44.err
timeout -k 10 250 python -u tools/variant_bench.py --libs $LIBS --users 262144 --items 4000000 --dim 64 --rounds 3 > gpurun_out/s44_d64_4m.json 2>> gpurun_out/s44.err
