#!/bin/bash
# Round-5 A/B 29: the compaction slack (keys kept past k): 32 (product)
# against 16 and 48; config 2 and the headline; lists bit-identical.
set -e
export TMPDIR=/tmp
O=gpurun_out/r05ab29
mkdir -p $O
timeout -k 10 300 python3 -u tools/variant_bench.py --libs product,sl16,sl48 --users 1000000 --items 1000000 --dim 64 --rounds 4 > $O/ab_cfg2.json 2> $O/ab_cfg2.err
timeout -k 10 500 python3 -u tools/variant_bench.py --libs product,sl16,sl48 --users 1000000 --items 10000000 --dim 128 --rounds 2 > $O/ab_10m.json 2> $O/ab_10m.err
