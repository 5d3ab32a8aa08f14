#!/bin/bash
# Round 6: k = 1000 (1M x 10M, d = 128) planner knobs on the staged build:
# sample stride 64 / 16, first-tier ranks 44 / 47 (guess_z1 / guess_c1).
set -e
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r06k1000
mkdir -p $O
cd $R
timeout -k 10 600 python3 -u tools/variant_bench.py --libs product,product@guess_stride=64,product@guess_stride=64+sample_dense=24,product@guess_stride=128,product@guess_stride=96+sample_dense=24 --users 1000000 --items 10000000 --dim 128 --k 1000 --rounds 3 > $O/ab_knobs2.json 2> $O/ab_knobs2.err
