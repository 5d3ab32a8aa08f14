#!/bin/bash
# Round-5 A/B 16: the d = 128 ring geometry: two 64-KB stages (product)
# against three 48-KB stages (two in flight, a barrier every 6 tiles) and two
# 72-KB stages (a barrier every 9 tiles); headline, k = 1000 and an 8-way
# shard's 1.25M rows; lists bit-identical; then the new dense-sample test.
set -e
export TMPDIR=/tmp
O=gpurun_out/r05ab16
mkdir -p $O
timeout -k 10 600 python3 -u -m pytest tests/test_hip_kernels.py -k "dense_sample" -x -q --timeout 300 --timeout-method thread > $O/tests.log 2>&1
timeout -k 10 500 python3 -u tools/variant_bench.py --libs product,w3x48,w2x72 --users 1000000 --items 10000000 --dim 128 --rounds 2 > $O/ab_10m.json 2> $O/ab_10m.err
timeout -k 10 300 python3 -u tools/variant_bench.py --libs product,w3x48,w2x72 --users 1000000 --items 1250000 --dim 128 --rounds 3 > $O/ab_shard8.json 2> $O/ab_shard8.err
timeout -k 10 400 python3 -u tools/variant_bench.py --libs product,w3x48,w2x72 --users 262144 --items 10000000 --dim 128 --k 1000 --rounds 2 > $O/ab_k1000.json 2> $O/ab_k1000.err
