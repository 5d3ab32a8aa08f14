#!/bin/bash
# Round 6: second-tier rescan split up to 128 catalog chunks per failing user
# block (rc128) against 64, at the headline, config 2 and k = 1000; and the
# k = 1000 first-tier rank at stride 128 (17 by the Poisson rule; 15 / 19).
set -e
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r06rc
mkdir -p $O
cd $R
timeout -k 10 400 python3 -u tools/variant_bench.py --libs product,rc128 --users 1000000 --items 10000000 --dim 128 --k 100 --rounds 4 > $O/ab_head.json 2> $O/ab_head.err
timeout -k 10 300 python3 -u tools/variant_bench.py --libs product,rc128 --users 1000000 --items 1000000 --dim 64 --k 100 --rounds 5 > $O/ab_cfg2.json 2> $O/ab_cfg2.err
timeout -k 10 600 python3 -u tools/variant_bench.py --libs product,rc128,product@guess_z1=1.5+guess_c1=2.9,product@guess_z1=2.5+guess_c1=4 --users 1000000 --items 10000000 --dim 128 --k 1000 --rounds 3 > $O/ab_k1000.json 2> $O/ab_k1000.err
