#!/bin/bash
# Round-5 A/B 2, one process per shape, outputs bit-identical: long lists
# ending each whole-catalog unit compacted to 1024 keys (product) against no
# end compaction (nokeep), and the candidate-key store policy (st1: sc1
# write-through, st2: nt) against plain stores; then the k = 1000 GPU tests.
set -e
export TMPDIR=/tmp
O=gpurun_out/r05ab2
mkdir -p $O
timeout -k 10 400 python3 -u tools/variant_bench.py --libs product,nokeep,st1,st2 --users 1000000 --items 10000000 --dim 128 --k 1000 --rounds 2 > $O/ab_k1000_1m.json 2> $O/ab_k1000_1m.err
timeout -k 10 300 python3 -u tools/variant_bench.py --libs product,st1,st2 --users 1000000 --items 1000000 --dim 64 --rounds 3 > $O/ab_cfg2.json 2> $O/ab_cfg2.err
timeout -k 10 300 python3 -u tools/variant_bench.py --libs product,st1,st2 --users 1000000 --items 10000000 --dim 128 --rounds 2 > $O/ab_10m.json 2> $O/ab_10m.err
timeout -k 10 600 python3 -u -m pytest tests/test_hip_kernels.py tests/test_real_plans.py -k "k1000 or config5 or forced_stride or second_tier" -x -q --timeout 500 --timeout-method thread > $O/tests.log 2>&1
