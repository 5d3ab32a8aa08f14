#!/bin/bash
# Round-5 A/B 6: staged hits taking the lane bit from the ballot (inverse
# ballot, product) against re-deriving it from the compare (noib), config 2,
# outputs bit-identical.
set -e
export TMPDIR=/tmp
O=gpurun_out/r05ab6
mkdir -p $O
timeout -k 10 300 python3 -u tools/variant_bench.py --libs product,noib --users 1000000 --items 1000000 --dim 64 --rounds 5 > $O/ab_cfg2.json 2> $O/ab_cfg2.err
timeout -k 10 300 python3 -u tools/variant_bench.py --libs product,noib --users 262144 --items 4000000 --dim 64 --rounds 3 > $O/ab_4m.json 2> $O/ab_4m.err
