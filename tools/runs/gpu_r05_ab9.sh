#!/bin/bash
# Round-5 A/B 9: the sample scan (tile maxima) on the per-user-tile pipeline
# too at d <= 64 (product) against its group epilogue (sgrp), config 2 and
# d = 32, outputs bit-identical; then the guess / threshold tests.
set -e
export TMPDIR=/tmp
O=gpurun_out/r05ab9
mkdir -p $O
timeout -k 10 300 python3 -u tools/variant_bench.py --libs product,sgrp --users 1000000 --items 1000000 --dim 64 --rounds 4 > $O/ab_cfg2.json 2> $O/ab_cfg2.err
timeout -k 10 300 python3 -u tools/variant_bench.py --libs product,sgrp --users 1000000 --items 1000000 --dim 32 --rounds 3 > $O/ab_d32.json 2> $O/ab_d32.err
timeout -k 10 900 python3 -u -m pytest tests/test_hip_kernels.py tests/test_real_plans.py tests/test_distributed_gpu.py -k "topk or sample_thresholds or plan or second_tier or forced or sharded" -x -q --timeout 500 --timeout-method thread > $O/tests.log 2>&1
