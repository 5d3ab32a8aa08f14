#!/bin/bash
# Round 6: small catalogs keep every key (CAP >= n_items, no compaction):
# score_topk / API tests, then A/B against the compacting plan (nokeep) at
# small shapes and config 1's drop-in evaluation step.
set -e
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r06ka
mkdir -p $O
cd $R
timeout -k 10 600 python3 -u -m pytest tests/test_hip_kernels.py tests/test_api_gpu.py tests/test_distributed_gpu.py -k "score_topk or recommend or api or drop or golden or shard or exclusion" -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > $O/tests.log 2>&1
for shape in "943 1682 32 10" "943 1682 64 10" "6040 3706 128 10" "10000 2000 64 100" "60000 2048 64 10" "1000 1500 128 1000"; do
  set -- $shape
  timeout -k 10 200 python3 -u tools/variant_bench.py --libs product,nokeep --users $1 --items $2 --dim $3 --k $4 --rounds 5 >> $O/ab_small.jsonl 2>> $O/ab_small.err
done
timeout -k 10 200 python3 bench.py --workload ml100k --steps 5 --warmup 2 --no-cpu-baseline > $O/ml100k_product.jsonl 2> $O/ml100k_product.err
DIVREC_HIP_LIB=$R/diversity-recommendations_amd/divrec/_lib/libdivrec_hip_nokeep.so timeout -k 10 200 python3 bench.py --workload ml100k --steps 5 --warmup 2 --no-cpu-baseline > $O/ml100k_nokeep.jsonl 2> $O/ml100k_nokeep.err
timeout -k 10 200 python3 tools/ml100k_profile.py > $O/prof.txt 2>&1
