#!/bin/bash
# Round-5 A/B 3: more waves per SIMD at d <= 64, one process, outputs
# bit-identical: w12 = 12 waves (3 per SIMD, <= 168 VGPRs) x 3 user tiles,
# 24-KB stages; w16 = 16 waves (4 per SIMD, 128 VGPRs) x 2 user tiles,
# 16-KB stages; against the product's 8 waves x 8 tiles (2 groups of 4).
set -e
export TMPDIR=/tmp
O=gpurun_out/r05ab3
mkdir -p $O
timeout -k 10 300 python3 -u tools/variant_bench.py --libs product,w12,w16 --users 1000000 --items 1000000 --dim 64 --rounds 3 > $O/ab_cfg2.json 2> $O/ab_cfg2.err
timeout -k 10 300 python3 -u tools/variant_bench.py --libs product,w12,w16 --users 262144 --items 4000000 --dim 64 --rounds 3 > $O/ab_4m.json 2> $O/ab_4m.err
timeout -k 10 300 python3 -u tools/variant_bench.py --libs product,w12,w16 --users 1000000 --items 1000000 --dim 32 --rounds 3 > $O/ab_d32.json 2> $O/ab_d32.err
