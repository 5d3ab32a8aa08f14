#!/bin/bash
# Round-4 A/B 2: SIMD-pair MFMA turns (DR_TURNS, libdivrec_hip_turns.so)
# against the product scan, one process per shape, lists must be identical;
# per-wave diag shares of both. Each step under its own time limit (a spin
# that never got its turn would be capped in-kernel, but bound it anyway).
set -e
export TMPDIR=/tmp
O=gpurun_out/ab2
mkdir -p $O
timeout -k 10 200 python3 -u tools/variant_bench.py --libs product,turns --users 131072 --items 1250000 --dim 128 --rounds 2 > $O/ab_small.json 2> $O/ab_small.err
timeout -k 10 300 python3 -u tools/diag_topk.py --lib=diag --users 262144 --items 10000000 --dim 128 --k 100 > $O/diag.json 2> $O/diag.err
timeout -k 10 300 python3 -u tools/diag_topk.py --lib=turnsdiag --users 262144 --items 10000000 --dim 128 --k 100 > $O/turnsdiag.json 2> $O/turnsdiag.err
timeout -k 10 400 python3 -u tools/variant_bench.py --libs product,turns --users 1000000 --items 10000000 --dim 128 --rounds 2 > $O/ab_10m.json 2> $O/ab_10m.err
timeout -k 10 300 python3 -u tools/variant_bench.py --libs product,turns --users 1000000 --items 1000000 --dim 64 --rounds 3 > $O/ab_cfg2.json 2> $O/ab_cfg2.err
timeout -k 10 300 python3 -u tools/variant_bench.py --libs product,turns --users 262144 --items 10000000 --dim 128 --k 1000 --rounds 2 > $O/ab_k1000.json 2> $O/ab_k1000.err
timeout -k 10 300 python3 -u tools/variant_bench.py --libs product,turns --users 1000000 --items 1250000 --dim 128 --rounds 3 > $O/ab_1m25.json 2> $O/ab_1m25.err
