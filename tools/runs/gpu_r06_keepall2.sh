#!/bin/bash
# Round 6: keep-all plan adopted (<= 2048 rows, <= 16384 users): its edge
# tests and the score_topk / API subsets again.
set -e
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r06ka2
mkdir -p $O
cd $R
timeout -k 10 600 python3 -u -m pytest tests/test_hip_kernels.py tests/test_api_gpu.py tests/test_distributed_gpu.py tests/test_real_plans.py -k "score_topk or recommend or api or drop or golden or shard or exclusion or keeps_every" -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > $O/tests.log 2>&1
