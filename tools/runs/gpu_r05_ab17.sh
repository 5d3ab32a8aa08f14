#!/bin/bash
# Round-5 A/B 17: confirmation run of the d = 128 ring (two 72-KB stages,
# w2x72) against the product's two 64-KB stages on another box: headline
# (3 rounds) and the full-size k = 1000 scan.
set -e
export TMPDIR=/tmp
O=gpurun_out/r05ab17
mkdir -p $O
timeout -k 10 600 python3 -u tools/variant_bench.py --libs product,w2x72 --users 1000000 --items 10000000 --dim 128 --rounds 3 > $O/ab_10m.json 2> $O/ab_10m.err
timeout -k 10 500 python3 -u tools/variant_bench.py --libs product,w2x72 --users 1000000 --items 10000000 --dim 128 --k 1000 --rounds 1 > $O/ab_k1000.json 2> $O/ab_k1000.err
