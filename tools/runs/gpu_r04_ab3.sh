#!/bin/bash
# Round-4 A/B 3: the new long-list ILD tests and the whole GPU suite on the
# product build, then the 16-way max without canonicalising copies
# (DR_MAX3_ASM, libdivrec_hip_max3.so) against the product in one process.
set -e
export TMPDIR=/tmp
O=gpurun_out/ab3
mkdir -p $O
timeout -k 10 300 python3 -u -m pytest tests/test_hip_kernels.py -m gpu -x -q --timeout 200 --timeout-method thread -k "long_lists or drop_in_long" > $O/new_tests.log 2>&1
timeout -k 10 600 python3 -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread > $O/gpu_tests.log 2>&1
timeout -k 10 300 python3 -u tools/variant_bench.py --libs product,max3 --users 1000000 --items 1000000 --dim 64 --rounds 3 > $O/ab_cfg2.json 2> $O/ab_cfg2.err
timeout -k 10 300 python3 -u tools/variant_bench.py --libs product,max3 --users 262144 --items 10000000 --dim 128 --rounds 3 > $O/ab_10m.json 2> $O/ab_10m.err
