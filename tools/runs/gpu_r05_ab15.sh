#!/bin/bash
# Round-5 A/B 15: the headline's guess stride with the dense sample scan:
# stride 128 (product) against 64 (a 19.5-GB matrix: budget 24 GiB) and
# config 2 at stride 24; lists bit-identical.
set -e
export TMPDIR=/tmp
O=gpurun_out/r05ab15
mkdir -p $O
timeout -k 10 500 python3 -u tools/variant_bench.py --libs product,product@guess_stride=64+sample_dense=24 --users 1000000 --items 10000000 --dim 128 --rounds 3 > $O/ab_10m.json 2> $O/ab_10m.err
timeout -k 10 300 python3 -u tools/variant_bench.py --libs product,product@guess_stride=24 --users 1000000 --items 1000000 --dim 64 --rounds 4 > $O/ab_cfg2.json 2> $O/ab_cfg2.err
