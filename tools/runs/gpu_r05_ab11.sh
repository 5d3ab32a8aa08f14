#!/bin/bash
# Round-5 A/B 11: the sample scan's compaction (slack kept past ks, flush
# gap): product (slack 32, gap 96) against tighter compactions, which raise
# each user's running threshold sooner and so store fewer tile-max keys.
# Config 2, the headline 1M x 10M and k = 1000; lists bit-identical.
set -e
export TMPDIR=/tmp
O=gpurun_out/r05ab11
mkdir -p $O
timeout -k 10 300 python3 -u tools/variant_bench.py --libs product,s0g32,s0g64,s8g24 --users 1000000 --items 1000000 --dim 64 --rounds 4 > $O/ab_cfg2.json 2> $O/ab_cfg2.err
timeout -k 10 400 python3 -u tools/variant_bench.py --libs product,s0g32,s8g24 --users 1000000 --items 10000000 --dim 128 --rounds 2 > $O/ab_10m.json 2> $O/ab_10m.err
timeout -k 10 400 python3 -u tools/variant_bench.py --libs product,s0g32,s8g24 --users 262144 --items 10000000 --dim 128 --k 1000 --rounds 3 > $O/ab_k1000.json 2> $O/ab_k1000.err
