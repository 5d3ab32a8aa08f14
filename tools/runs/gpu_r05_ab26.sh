#!/bin/bash
# Round-5 A/B 26: d = 128 with ONE wave per SIMD (4 waves of 512 VGPRs,
# 8 user tiles each, same 1024 users per workgroup) and the per-user-tile
# pipeline (w4utp) against the product's two waves per SIMD; headline,
# an 8-way shard's rows and k = 1000; lists bit-identical.
set -e
export TMPDIR=/tmp
O=gpurun_out/r05ab26
mkdir -p $O
timeout -k 10 500 python3 -u tools/variant_bench.py --libs product,w4utp --users 1000000 --items 10000000 --dim 128 --rounds 2 > $O/ab_10m.json 2> $O/ab_10m.err
timeout -k 10 300 python3 -u tools/variant_bench.py --libs product,w4utp --users 1000000 --items 1250000 --dim 128 --rounds 3 > $O/ab_shard8.json 2> $O/ab_shard8.err
timeout -k 10 400 python3 -u tools/variant_bench.py --libs product,w4utp --users 262144 --items 10000000 --dim 128 --k 1000 --rounds 2 > $O/ab_k1000.json 2> $O/ab_k1000.err
