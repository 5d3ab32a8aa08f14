#!/bin/bash
# Round-4 A/B 1 (one process per shape, outputs must be bit-identical):
#   product  = group-max sample scan (GMAX) over the tile-transposed sample
#   nogmax   = the round-3 sample scan (every survivor)
#   bal      = product + DR_BALANCE (SIMD-pair progress priority)
#   product@DIVREC_GUESS_STRIDE=16 = a denser sample, now that it is cheap
# plus the per-wave diag shares of the scan with and without DR_BALANCE, and
# the GPU tests of the scan (the guess paths changed).
set -e
export TMPDIR=/tmp
O=gpurun_out/ab1
mkdir -p $O
timeout -k 10 600 python3 -u -m pytest tests/test_real_plans.py tests/test_hip_kernels.py -m gpu -x -q --timeout 300 --timeout-method thread -k "score_topk or plan or tier or rescan or stride or thresholds" > $O/tests.log 2>&1
timeout -k 10 300 python3 -u tools/diag_topk.py --lib=diag --users 262144 --items 10000000 --dim 128 --k 100 > $O/diag.json 2> $O/diag.err
timeout -k 10 300 python3 -u tools/diag_topk.py --lib=baldiag --users 262144 --items 10000000 --dim 128 --k 100 > $O/baldiag.json 2> $O/baldiag.err
timeout -k 10 400 python3 -u tools/variant_bench.py --libs product,nogmax,bal,product@DIVREC_GUESS_STRIDE=16,product@DIVREC_GUESS_STRIDE=8 --users 1000000 --items 1000000 --dim 64 --rounds 3 > $O/ab_cfg2.json 2> $O/ab_cfg2.err
timeout -k 10 400 python3 -u tools/variant_bench.py --libs product,nogmax,bal,balinv,bal1 --users 1000000 --items 10000000 --dim 128 --rounds 2 > $O/ab_10m.json 2> $O/ab_10m.err
timeout -k 10 400 python3 -u tools/variant_bench.py --libs product,nogmax,bal --users 262144 --items 10000000 --dim 128 --k 1000 --rounds 2 > $O/ab_k1000.json 2> $O/ab_k1000.err
timeout -k 10 400 python3 -u tools/variant_bench.py --libs product,bal --users 1000000 --items 1250000 --dim 128 --rounds 3 > $O/ab_1m25.json 2> $O/ab_1m25.err
timeout -k 10 300 python3 -u tools/shard_thr_ab.py --shards 8 > $O/shard8.json 2> $O/shard8.err
