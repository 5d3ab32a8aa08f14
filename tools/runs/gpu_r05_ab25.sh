#!/bin/bash
# Round-5 A/B 25: main-scan flush gap 124 (flush at 256 keys, the finalize's
# 256-key sort still holds them) against 96 (228) at d <= 64, where CAP 1024
# leaves room; config 2 and d = 32; lists bit-identical.
set -e
export TMPDIR=/tmp
O=gpurun_out/r05ab25
mkdir -p $O
timeout -k 10 300 python3 -u tools/variant_bench.py --libs product,gap124 --users 1000000 --items 1000000 --dim 64 --rounds 5 > $O/ab_cfg2.json 2> $O/ab_cfg2.err
timeout -k 10 300 python3 -u tools/variant_bench.py --libs product,gap124 --users 1000000 --items 1000000 --dim 32 --rounds 4 > $O/ab_d32.json 2> $O/ab_d32.err
