#!/bin/bash
# Round-5 A/B 21: the 0.5 % Poisson-tail first-tier rank (product) against
# the round-3 rule mu + 3 sigma + 1 (guess_z1=3) at config 2, d = 32, the
# 8-way shard rows and the headline (same ranks there); then the GPU suite.
set -e
export TMPDIR=/tmp
O=gpurun_out/r05ab21
mkdir -p $O
timeout -k 10 300 python3 -u tools/variant_bench.py --libs product,product@guess_z1=3 --users 1000000 --items 1000000 --dim 64 --rounds 5 > $O/ab_cfg2.json 2> $O/ab_cfg2.err
timeout -k 10 300 python3 -u tools/variant_bench.py --libs product,product@guess_z1=3 --users 1000000 --items 1250000 --dim 128 --rounds 4 > $O/ab_shard8.json 2> $O/ab_shard8.err
timeout -k 10 400 python3 -u tools/variant_bench.py --libs product,product@guess_z1=3 --users 1000000 --items 10000000 --dim 128 --rounds 2 > $O/ab_10m.json 2> $O/ab_10m.err
timeout -k 10 600 python3 -u -m pytest tests -m gpu -q -x --timeout 300 --timeout-method thread -p no:cacheprovider > $O/gpu_tests.log 2>&1
