#!/bin/bash
# Round-5 A/B 1: the hot test on v_maximum3_f32 with the ballots kept in SGPR
# pairs, and staged blocks with one 8-B record, against the round-4 kernels
# (libdivrec_hip_r04.so), one process per shape, outputs bit-identical; then
# the top-k GPU tests of the new build.
set -e
export TMPDIR=/tmp
O=gpurun_out/r05ab1
mkdir -p $O
timeout -k 10 300 python3 -u tools/variant_bench.py --libs product,r04 --users 1000000 --items 1000000 --dim 64 --rounds 4 > $O/ab_cfg2.json 2> $O/ab_cfg2.err
timeout -k 10 300 python3 -u tools/variant_bench.py --libs product,r04 --users 1000000 --items 10000000 --dim 128 --rounds 2 > $O/ab_10m.json 2> $O/ab_10m.err
timeout -k 10 300 python3 -u tools/variant_bench.py --libs product,r04 --users 262144 --items 10000000 --dim 128 --k 1000 --rounds 2 > $O/ab_k1000.json 2> $O/ab_k1000.err
timeout -k 10 600 python3 -u -m pytest tests/test_hip_kernels.py -k "topk or sample_thresholds" -x -q --timeout 300 --timeout-method thread > $O/tests.log 2>&1
