#!/bin/bash
# Round-4 A/B 5: two 4-wave scan workgroups per CU (wg2: DR_WAVES=4,
# DR_WG_PER_CU=2, 32-KB stages at d = 128, 16-KB stages otherwise; each group
# has its own LDS ring and barrier, the two waves of a SIMD belong to
# different groups) against the product's one 8-wave workgroup per CU. One
# process per shape, outputs bit-identical.
set -e
export TMPDIR=/tmp
O=gpurun_out/ab5
mkdir -p $O
timeout -k 10 400 python3 -u tools/variant_bench.py --libs product,wg2 --users 1000000 --items 10000000 --dim 128 --rounds 2 > $O/ab_10m.json 2> $O/ab_10m.err
timeout -k 10 300 python3 -u tools/variant_bench.py --libs product,wg2 --users 1000000 --items 1000000 --dim 64 --rounds 3 > $O/ab_cfg2.json 2> $O/ab_cfg2.err
timeout -k 10 300 python3 -u tools/variant_bench.py --libs product,wg2 --users 262144 --items 10000000 --dim 128 --k 1000 --rounds 2 > $O/ab_k1000.json 2> $O/ab_k1000.err
