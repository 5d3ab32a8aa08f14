#!/bin/bash
# Round 6: config 1's host plumbing (cached exclusion CSR, one rank-metrics
# launch per evaluation loop): the API / metric tests, the ml100k line and
# the per-part profile.
set -e
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r06c1
mkdir -p $O
cd $R
timeout -k 10 600 python3 -u -m pytest tests/test_api_gpu.py tests/test_hip_kernels.py -k "api or metric or rank or golden or loop or precision or recall or ndcg or map or entropy or pri or ild" -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > $O/tests.log 2>&1
timeout -k 10 200 python3 bench.py --workload ml100k --steps 5 --warmup 2 --no-cpu-baseline > $O/ml100k.jsonl 2> $O/ml100k.err
timeout -k 10 200 python3 tools/ml100k_profile.py > $O/prof.txt 2>&1
