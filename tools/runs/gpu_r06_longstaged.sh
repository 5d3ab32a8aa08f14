#!/bin/bash
# Round 6: the d = 128 long-list staging on the product sources (region split
# removed): score_topk / k = 1000 tests, then A/B against the round-5 build.
set -e
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r06ls
mkdir -p $O
cd $R
timeout -k 10 900 python3 -u -m pytest tests/test_real_plans.py tests/test_hip_kernels.py -k "score_topk or 1000 or split or second_tier or config" -x -v --timeout 400 --timeout-method thread -p no:cacheprovider > $O/tests.log 2>&1
timeout -k 10 400 python3 -u tools/variant_bench.py --libs product,r06base --users 1000000 --items 10000000 --dim 128 --k 1000 --rounds 3 > $O/ab_k1000.json 2> $O/ab_k1000.err
timeout -k 10 300 python3 -u tools/variant_bench.py --libs product,r06base --users 1000000 --items 1000000 --dim 64 --k 100 --rounds 5 > $O/ab_cfg2.json 2> $O/ab_cfg2.err
