#!/bin/bash
# Round-4 A/B 4: the guess's planner knobs re-measured on the final kernels
# (two tiers + group-max sample), one process per shape, outputs bit-identical:
# the sample stride (config 2 at 64; k = 1000 at 64) and the first-tier margin
# z1 (2.5 / 3.5 against 3.0) at config 2, k = 1000 and the headline shape.
set -e
export TMPDIR=/tmp
O=gpurun_out/ab4
mkdir -p $O
timeout -k 10 400 python3 -u tools/variant_bench.py --libs product,product@DIVREC_GUESS_STRIDE=64,product@DIVREC_GUESS_Z1=2.5,product@DIVREC_GUESS_Z1=3.5 --users 1000000 --items 1000000 --dim 64 --rounds 3 > $O/ab_cfg2.json 2> $O/ab_cfg2.err
timeout -k 10 500 python3 -u tools/variant_bench.py --libs product,product@DIVREC_GUESS_STRIDE=64,product@DIVREC_GUESS_Z1=2.5,product@DIVREC_GUESS_Z1=3.5 --users 262144 --items 10000000 --dim 128 --k 1000 --rounds 2 > $O/ab_k1000.json 2> $O/ab_k1000.err
timeout -k 10 500 python3 -u tools/variant_bench.py --libs product,product@DIVREC_GUESS_Z1=2.5,product@DIVREC_GUESS_Z1=3.5,product@DIVREC_GUESS_STRIDE=128 --users 1000000 --items 10000000 --dim 128 --rounds 2 > $O/ab_10m.json 2> $O/ab_10m.err
