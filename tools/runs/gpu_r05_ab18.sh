#!/bin/bash
# Round-5 A/B 18: the d <= 64 ring: three 32-KB stages (product) against two
# 48-KB stages (a barrier every 12 tiles at d = 64) and four 24-KB stages
# (three in flight, every 6 tiles); config 2 and d = 32; lists bit-identical.
set -e
export TMPDIR=/tmp
O=gpurun_out/r05ab18
mkdir -p $O
timeout -k 10 400 python3 -u tools/variant_bench.py --libs product,n2x48,n4x24 --users 1000000 --items 1000000 --dim 64 --rounds 4 > $O/ab_cfg2.json 2> $O/ab_cfg2.err
timeout -k 10 300 python3 -u tools/variant_bench.py --libs product,n2x48,n4x24 --users 1000000 --items 1000000 --dim 32 --rounds 3 > $O/ab_d32.json 2> $O/ab_d32.err
