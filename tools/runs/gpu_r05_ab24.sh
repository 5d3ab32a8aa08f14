#!/bin/bash
# Round-5 A/B 24: k = 1000 with the dense sample at stride 64 (a 19.5-GB
# matrix: budget 24 GiB) against the product's compaction sample at stride 32;
# full size; lists bit-identical.
set -e
export TMPDIR=/tmp
O=gpurun_out/r05ab24
mkdir -p $O
timeout -k 10 600 python3 -u tools/variant_bench.py --libs product,product@guess_stride=64+sample_dense=24,product@sample_dense=48 --users 1000000 --items 10000000 --dim 128 --k 1000 --rounds 2 > $O/ab_k1000.json 2> $O/ab_k1000.err
