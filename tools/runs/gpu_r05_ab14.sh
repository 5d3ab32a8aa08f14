#!/bin/bash
# Round-5 A/B 14: the dense threshold kernel with per-lane LDS lists and
# batched merges (product) against the per-tile insertion network (dnet) and
# the compaction path; config 2 and the headline; k = 1000 with the dense
# sample (a 39-GB matrix: budget 48 GiB) against its compaction path; lists
# bit-identical; then the guess / threshold tests.
set -e
export TMPDIR=/tmp
O=gpurun_out/r05ab14
mkdir -p $O
timeout -k 10 600 python3 -u -m pytest tests/test_hip_kernels.py -k "dense_sample or sample_thresholds or guess" -x -q --timeout 300 --timeout-method thread > $O/tests.log 2>&1
timeout -k 10 300 python3 -u tools/variant_bench.py --libs product,dnet,product@sample_dense=0 --users 1000000 --items 1000000 --dim 64 --rounds 4 > $O/ab_cfg2.json 2> $O/ab_cfg2.err
timeout -k 10 400 python3 -u tools/variant_bench.py --libs product,dnet --users 1000000 --items 10000000 --dim 128 --rounds 2 > $O/ab_10m.json 2> $O/ab_10m.err
timeout -k 10 500 python3 -u tools/variant_bench.py --libs product,product@sample_dense=48 --users 1000000 --items 10000000 --dim 128 --k 1000 --rounds 2 > $O/ab_k1000.json 2> $O/ab_k1000.err
