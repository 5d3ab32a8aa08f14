#!/bin/bash
# Round-5 A/B 4: the sample scan keeping one max per user and TILE (the two
# half-waves merged by v_permlane32_swap, per-user counters with one writer,
# no LDS atomics) against one max per 16-row half-tile with an LDS atomic per
# hitting lane (g16 = the previous build), one process per shape, outputs
# bit-identical; then the guess / threshold GPU tests.
set -e
export TMPDIR=/tmp
O=gpurun_out/r05ab4
mkdir -p $O
timeout -k 10 300 python3 -u tools/variant_bench.py --libs product,g16 --users 1000000 --items 1000000 --dim 64 --rounds 4 > $O/ab_cfg2.json 2> $O/ab_cfg2.err
timeout -k 10 300 python3 -u tools/variant_bench.py --libs product,g16 --users 262144 --items 10000000 --dim 128 --k 1000 --rounds 3 > $O/ab_k1000.json 2> $O/ab_k1000.err
timeout -k 10 300 python3 -u tools/variant_bench.py --libs product,g16 --users 1000000 --items 10000000 --dim 128 --rounds 2 > $O/ab_10m.json 2> $O/ab_10m.err
timeout -k 10 900 python3 -u -m pytest tests/test_hip_kernels.py tests/test_real_plans.py tests/test_distributed_gpu.py tests/test_rccl_gpu.py -k "topk or sample_thresholds or plan or second_tier or forced or sharded or rccl" -x -q --timeout 500 --timeout-method thread > $O/tests.log 2>&1
