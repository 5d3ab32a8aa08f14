#!/bin/bash
# Round-5 A/B 5: the direct (d >= 128) survivor enqueue with one ballot per
# score register and value / row selected on the ballots (product) against
# the per-lane bit mask + 16-way max of round 4 (eb0), one process per shape,
# outputs bit-identical; then the top-k GPU tests.
set -e
export TMPDIR=/tmp
O=gpurun_out/r05ab5
mkdir -p $O
timeout -k 10 300 python3 -u tools/variant_bench.py --libs product,eb0 --users 1000000 --items 10000000 --dim 128 --rounds 3 > $O/ab_10m.json 2> $O/ab_10m.err
timeout -k 10 400 python3 -u tools/variant_bench.py --libs product,eb0 --users 1000000 --items 10000000 --dim 128 --k 1000 --rounds 2 > $O/ab_k1000_1m.json 2> $O/ab_k1000_1m.err
timeout -k 10 300 python3 -u tools/variant_bench.py --libs product,eb0 --users 1000000 --items 1250000 --dim 128 --rounds 3 > $O/ab_shard8.json 2> $O/ab_shard8.err
timeout -k 10 900 python3 -u -m pytest tests/test_hip_kernels.py tests/test_real_plans.py -k "topk or plan or second_tier or forced" -x -q --timeout 500 --timeout-method thread > $O/tests.log 2>&1
