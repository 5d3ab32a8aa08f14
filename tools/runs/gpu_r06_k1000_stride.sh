#!/bin/bash
# Round 6: k = 1000 samples at stride 128 (dense tile maxima) on the staged
# build: the k = 1000 / config-5 / sharded tests, A/B against the round-5
# build, and the config-5 (mmr) workload line.
set -e
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r06k1000s
mkdir -p $O
cd $R
timeout -k 10 900 python3 -u -m pytest tests/test_real_plans.py tests/test_hip_kernels.py tests/test_distributed_gpu.py -k "1000 or config5 or shard or mmr" -x -v --timeout 600 --timeout-method thread -p no:cacheprovider > $O/tests.log 2>&1
timeout -k 10 400 python3 -u tools/variant_bench.py --libs product,r06base --users 1000000 --items 10000000 --dim 128 --k 1000 --rounds 3 > $O/ab_k1000.json 2> $O/ab_k1000.err
timeout -k 10 400 python3 bench.py --workload mmr --no-cpu-baseline > $O/bench_mmr.jsonl 2> $O/bench_mmr.err
