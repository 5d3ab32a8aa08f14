#!/bin/bash
# Round 6: keep-all plans split the catalog into stage-long chunks: tests,
# A/B against the unsplit keep-all plan (scan_split = 1), config 1's line.
set -e
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r06ka3
mkdir -p $O
cd $R
timeout -k 10 600 python3 -u -m pytest tests/test_hip_kernels.py tests/test_api_gpu.py tests/test_distributed_gpu.py -k "score_topk or recommend or api or drop or golden or shard or exclusion or keeps_every or loop" -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > $O/tests.log 2>&1
for shape in "943 1682 32 10" "943 1682 64 10" "10000 2000 64 100" "16000 2048 128 10" "300 700 128 50"; do
  set -- $shape
  timeout -k 10 200 python3 -u tools/variant_bench.py --libs product,product@scan_split=1 --users $1 --items $2 --dim $3 --k $4 --rounds 5 >> $O/ab_split.jsonl 2>> $O/ab_split.err
done
timeout -k 10 200 python3 bench.py --workload ml100k --steps 5 --warmup 2 --no-cpu-baseline > $O/ml100k.jsonl 2> $O/ml100k.err
