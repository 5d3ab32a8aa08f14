#!/bin/bash
# Round 6: main-scan flush gap 32 / 64 against 96 (earlier first compaction:
# thresholds rise sooner, fewer survivors) at config 2, d = 32 and the headline.
set -e
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r06gap
mkdir -p $O
cd $R
timeout -k 10 300 python3 -u tools/variant_bench.py --libs product,gap32,gap64 --users 1000000 --items 1000000 --dim 64 --k 100 --rounds 5 > $O/ab_cfg2.json 2> $O/ab_cfg2.err
timeout -k 10 300 python3 -u tools/variant_bench.py --libs product,gap32,gap64 --users 1000000 --items 1000000 --dim 32 --k 100 --rounds 5 > $O/ab_d32.json 2> $O/ab_d32.err
timeout -k 10 400 python3 -u tools/variant_bench.py --libs product,gap32,gap64 --users 1000000 --items 10000000 --dim 128 --k 100 --rounds 3 > $O/ab_head.json 2> $O/ab_head.err
