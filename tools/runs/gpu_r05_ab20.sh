#!/bin/bash
# Round-5 A/B 20: first-tier rank at a 0.5 % Poisson tail instead of 3 sigma:
# k = 1000 (ks1 50 -> 48: z1 = 2.7) and the 8-way shard's 1.25M rows at
# d = 128 (ks1 10 -> 9: z1 = 2.5); lists bit-identical.
set -e
export TMPDIR=/tmp
O=gpurun_out/r05ab20
mkdir -p $O
timeout -k 10 500 python3 -u tools/variant_bench.py --libs product,product@guess_z1=2.7 --users 1000000 --items 10000000 --dim 128 --k 1000 --rounds 2 > $O/ab_k1000.json 2> $O/ab_k1000.err
timeout -k 10 300 python3 -u tools/variant_bench.py --libs product,product@guess_z1=2.5 --users 1000000 --items 1250000 --dim 128 --rounds 4 > $O/ab_shard8.json 2> $O/ab_shard8.err
timeout -k 10 300 python3 -u tools/variant_bench.py --libs product,product@guess_z1=2.5 --users 1000000 --items 1000000 --dim 32 --rounds 4 > $O/ab_d32.json 2> $O/ab_d32.err
