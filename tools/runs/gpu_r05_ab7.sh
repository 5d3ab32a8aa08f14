#!/bin/bash
# Round-5 A/B 7: the per-user-tile software-pipelined epilogue (product:
# each (item tile, user tile) job's hot test runs under the next job's MFMA
# chain, two accumulators, the tile's A fragments read once) against the
# group epilogue (grp: DR_UTPIPE=0, the round-4 structure), one process per
# shape, outputs bit-identical; then the top-k GPU tests.
set -e
export TMPDIR=/tmp
O=gpurun_out/r05ab7
mkdir -p $O
timeout -k 10 300 python3 -u tools/variant_bench.py --libs product,grp --users 1000000 --items 1000000 --dim 64 --rounds 4 > $O/ab_cfg2.json 2> $O/ab_cfg2.err
timeout -k 10 300 python3 -u tools/variant_bench.py --libs product,grp --users 1000000 --items 10000000 --dim 128 --rounds 2 > $O/ab_10m.json 2> $O/ab_10m.err
timeout -k 10 300 python3 -u tools/variant_bench.py --libs product,grp --users 262144 --items 10000000 --dim 128 --k 1000 --rounds 3 > $O/ab_k1000.json 2> $O/ab_k1000.err
timeout -k 10 300 python3 -u tools/variant_bench.py --libs product,grp --users 1000000 --items 1000000 --dim 32 --rounds 3 > $O/ab_d32.json 2> $O/ab_d32.err
timeout -k 10 900 python3 -u -m pytest tests/test_hip_kernels.py tests/test_real_plans.py -k "topk or plan or second_tier or forced" -x -q --timeout 500 --timeout-method thread > $O/tests.log 2>&1
