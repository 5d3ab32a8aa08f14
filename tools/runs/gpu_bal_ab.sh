#!/bin/bash
# A/B of DR_BALANCE (SIMD-pair progress priority) against the product scan,
# in one process per shape, plus the per-wave diag shares of both builds.
set -e
export TMPDIR=/tmp
O=gpurun_out/bal
mkdir -p $O
timeout -k 10 300 python -u tools/diag_topk.py --lib=diag --users 262144 --items 10000000 --dim 128 --k 100 > $O/diag.json 2> $O/diag.err
timeout -k 10 300 python -u tools/diag_topk.py --lib=baldiag --users 262144 --items 10000000 --dim 128 --k 100 > $O/baldiag.json 2> $O/baldiag.err
timeout -k 10 400 python -u tools/variant_bench.py --libs product,bal --users 262144 --items 10000000 --dim 128 --rounds 3 > $O/ab_10m.json 2> $O/ab_10m.err
timeout -k 10 400 python -u tools/variant_bench.py --libs product,bal --users 1000000 --items 1250000 --dim 128 --rounds 3 > $O/ab_1m25.json 2> $O/ab_1m25.err
timeout -k 10 400 python -u tools/variant_bench.py --libs product,bal --users 262144 --items 10000000 --dim 128 --k 1000 --rounds 2 > $O/ab_k1000.json 2> $O/ab_k1000.err
