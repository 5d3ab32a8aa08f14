#!/bin/bash
# Round-5 A/B 19: config 2's guess after the ring change: stride 24 / 20 and
# the first-tier margin z1 = 2.5, alone and together; lists bit-identical.
set -e
export TMPDIR=/tmp
O=gpurun_out/r05ab19
mkdir -p $O
timeout -k 10 500 python3 -u tools/variant_bench.py --libs product,product@guess_stride=24,product@guess_z1=2.5,product@guess_stride=24+guess_z1=2.5,product@guess_stride=20 --users 1000000 --items 1000000 --dim 64 --rounds 5 > $O/ab_cfg2.json 2> $O/ab_cfg2.err
