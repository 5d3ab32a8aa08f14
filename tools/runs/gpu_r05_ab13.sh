#!/bin/bash
# Round-5 A/B 13: with the dense sample scan (a sample row now costs about
# the main scan's), the guess's planner knobs at config 2: stride 16 (twice
# the sample, ks 25 / ks1 15) and the first-tier margin z1 = 2.5.
set -e
export TMPDIR=/tmp
O=gpurun_out/r05ab13
mkdir -p $O
timeout -k 10 400 python3 -u tools/variant_bench.py --libs product,product@guess_stride=16,product@guess_z1=2.5,product@guess_stride=16+guess_z1=2.5,product@guess_z1=2.0 --users 1000000 --items 1000000 --dim 64 --rounds 4 > $O/ab_cfg2.json 2> $O/ab_cfg2.err
timeout -k 10 500 python3 -u tools/variant_bench.py --libs product,product@guess_z1=2.5,product@guess_z1=2.0 --users 1000000 --items 10000000 --dim 128 --rounds 2 > $O/ab_10m.json 2> $O/ab_10m.err
