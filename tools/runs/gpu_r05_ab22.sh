#!/bin/bash
# Round-5 A/B 22: with the compaction histogram aliased into the staging area
# (product), two 56-KB stages at d <= 64 (n2x56: a barrier every 14 tiles at
# d = 64) against the product's 48-KB stages; config 2 and d = 32; lists
# bit-identical; then the GPU suite on the product.
set -e
export TMPDIR=/tmp
O=gpurun_out/r05ab22
mkdir -p $O
timeout -k 10 300 python3 -u tools/variant_bench.py --libs product,n2x56 --users 1000000 --items 1000000 --dim 64 --rounds 5 > $O/ab_cfg2.json 2> $O/ab_cfg2.err
timeout -k 10 300 python3 -u tools/variant_bench.py --libs product,n2x56 --users 1000000 --items 1000000 --dim 32 --rounds 4 > $O/ab_d32.json 2> $O/ab_d32.err
timeout -k 10 600 python3 -u -m pytest tests -m gpu -q -x --timeout 300 --timeout-method thread -p no:cacheprovider > $O/gpu_tests.log 2>&1
