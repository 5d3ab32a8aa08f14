#!/bin/bash
# Round-5 A/B 31: the small-grid split (8192-row minimum chunk) at two more
# mid sizes against no split (scan_split=1); lists bit-identical.
set -e
export TMPDIR=/tmp
O=gpurun_out/r05ab31
mkdir -p $O
timeout -k 10 300 python3 -u tools/variant_bench.py --libs product,product@scan_split=1 --users 5000 --items 20000 --dim 64 --k 10 --rounds 5 > $O/ab_5k_20k.json 2> $O/ab_5k_20k.err
timeout -k 10 300 python3 -u tools/variant_bench.py --libs product,product@scan_split=1 --users 2000 --items 50000 --dim 128 --k 100 --rounds 5 > $O/ab_2k_50k.json 2> $O/ab_2k_50k.err
timeout -k 10 300 python3 -u tools/variant_bench.py --libs product,product@scan_split=1 --users 943 --items 16500 --dim 32 --k 10 --rounds 5 > $O/ab_943_16k.json 2> $O/ab_943_16k.err
