#!/bin/bash
# Round-4 A/B 7: the stagger of MI355X_MICROARCH.md (two waves per SIMD, item 9):
# waves 4-7 pass each stage barrier right after their MFMAs of the stage's
# last tile and run its epilogue behind the barrier (DR_DEFER=1,
# libdivrec_hip_defer.so), against the product. One process per shape,
# outputs bit-identical.
set -e
export TMPDIR=/tmp
O=gpurun_out/ab7
mkdir -p $O
timeout -k 10 400 python3 -u tools/variant_bench.py --libs product,defer --users 1000000 --items 10000000 --dim 128 --rounds 2 > $O/ab_10m.json 2> $O/ab_10m.err
timeout -k 10 300 python3 -u tools/variant_bench.py --libs product,defer --users 1000000 --items 1000000 --dim 64 --rounds 3 > $O/ab_cfg2.json 2> $O/ab_cfg2.err
timeout -k 10 300 python3 -u tools/variant_bench.py --libs product,defer --users 262144 --items 10000000 --dim 128 --k 1000 --rounds 2 > $O/ab_k1000.json 2> $O/ab_k1000.err
