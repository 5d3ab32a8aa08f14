#!/bin/bash
# Round-5 A/B 10: the d = 128 sample scans (tile maxima; the headline's
# stride-128 sample and config 5's stride-32 one) on the per-user-tile
# pipeline (product) against their group epilogue (g128), outputs
# bit-identical; then the threshold / guess tests.
set -e
export TMPDIR=/tmp
O=gpurun_out/r05ab10
mkdir -p $O
timeout -k 10 400 python3 -u tools/variant_bench.py --libs product,g128 --users 1000000 --items 10000000 --dim 128 --k 1000 --rounds 2 > $O/ab_k1000_1m.json 2> $O/ab_k1000_1m.err
timeout -k 10 300 python3 -u tools/variant_bench.py --libs product,g128 --users 1000000 --items 10000000 --dim 128 --rounds 2 > $O/ab_10m.json 2> $O/ab_10m.err
timeout -k 10 600 python3 -u -m pytest tests/test_hip_kernels.py tests/test_real_plans.py -k "k1000 or sample_thresholds or headline or config5 or second_tier" -x -q --timeout 500 --timeout-method thread > $O/tests.log 2>&1
