#!/bin/bash
# Round-5: dense Adam with 16-B accesses: its tests, then the BPR bench line
# (config 3: fused step + Adam).
set -e
export TMPDIR=/tmp
O=gpurun_out/r05adam
mkdir -p $O
timeout -k 10 300 python3 -u -m pytest tests/test_hip_kernels.py tests/test_api_gpu.py -k "adam or bpr or pairwise" -q -x --timeout 200 --timeout-method thread -p no:cacheprovider > $O/tests.log 2>&1
timeout -k 10 300 python3 bench.py --workload bpr --steps 5 --warmup 2 --no-cpu-baseline > $O/bpr.jsonl 2> $O/bpr.err
timeout -k 10 300 python3 bench.py --workload bpr --steps 5 --warmup 2 --no-cpu-baseline >> $O/bpr.jsonl 2>> $O/bpr.err
