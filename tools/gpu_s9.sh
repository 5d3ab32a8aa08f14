#!/bin/bash
# A/B of the stage hand-off: s_barrier (product) vs decoupled LDS counters
# (sync1, sync1r4) vs 64-KB stages with a 2-slot ring (s64r2).
set -e
mkdir -p gpurun_out
export TMPDIR=/tmp
LIBS=product,sync1,sync1r4,s64r2
timeout -k 10 200 python -u tools/variant_bench.py --libs $LIBS --users 1000000 --items 1250000 --dim 128 --rounds 3 > gpurun_out/s9_shard8.json 2> gpurun_out/s9_shard8.err
timeout -k 10 200 python -u tools/variant_bench.py --libs $LIBS --users 262144 --items 10000000 --dim 128 --rounds 3 > gpurun_out/s9_d128.json 2> gpurun_out/s9_d128.err
timeout -k 10 200 python -u tools/variant_bench.py --libs $LIBS --users 1000000 --items 1000000 --dim 64 --rounds 3 > gpurun_out/s9_d64.json 2> gpurun_out/s9_d64.err
