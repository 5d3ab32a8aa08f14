#!/bin/bash
# Round-5 A/B 23: d <= 64 LDS split: two 56-KB stages with 64 staged blocks
# per wave (product) against two 48-KB stages with 96 (n48sb96: fewer
# in-loop resolutions of a full staging area); config 2 and d = 32.
set -e
export TMPDIR=/tmp
O=gpurun_out/r05ab23
mkdir -p $O
timeout -k 10 300 python3 -u tools/variant_bench.py --libs product,n48sb96 --users 1000000 --items 1000000 --dim 64 --rounds 5 > $O/ab_cfg2.json 2> $O/ab_cfg2.err
timeout -k 10 300 python3 -u tools/variant_bench.py --libs product,n48sb96 --users 1000000 --items 1000000 --dim 32 --rounds 4 > $O/ab_d32.json 2> $O/ab_d32.err
