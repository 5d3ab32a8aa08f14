#!/bin/bash
# Round-5 A/B 12: the sample scan's dense tile maxima (product) against its
# compaction path (sample_dense = 0), config 2, the headline and d = 32;
# lists bit-identical; then the guess / threshold / plan tests.
set -e
export TMPDIR=/tmp
O=gpurun_out/r05ab12
mkdir -p $O
timeout -k 10 600 python3 -u -m pytest tests/test_hip_kernels.py -k "dense_sample or sample_thresholds or guess or nan_rows" -x -q --timeout 300 --timeout-method thread > $O/tests.log 2>&1
timeout -k 10 300 python3 -u tools/variant_bench.py --libs product,product@sample_dense=0 --users 1000000 --items 1000000 --dim 64 --rounds 4 > $O/ab_cfg2.json 2> $O/ab_cfg2.err
timeout -k 10 400 python3 -u tools/variant_bench.py --libs product,product@sample_dense=0 --users 1000000 --items 10000000 --dim 128 --rounds 2 > $O/ab_10m.json 2> $O/ab_10m.err
timeout -k 10 300 python3 -u tools/variant_bench.py --libs product,product@sample_dense=0 --users 1000000 --items 1000000 --dim 32 --rounds 3 > $O/ab_d32.json 2> $O/ab_d32.err
