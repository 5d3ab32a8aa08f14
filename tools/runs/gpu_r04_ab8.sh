#!/bin/bash
# Round-4 A/B 8: MMR probe threshold by a VALU bitonic network (DR_MMR_VSEL=1,
# libdivrec_hip_vsel.so) against the product's SALU radix select, one process
# per candidate kind, picks identical for every user (tools/mmr_ab.py).
set -e
export TMPDIR=/tmp
O=gpurun_out/ab8
mkdir -p $O
timeout -k 10 400 python3 -u tools/mmr_ab.py --libs product,vsel --real > $O/ab_real.json 2> $O/ab_real.err
timeout -k 10 300 python3 -u tools/mmr_ab.py --libs product,vsel > $O/ab_rand.json 2> $O/ab_rand.err
timeout -k 10 300 python3 -u tools/mmr_ab.py --libs product,vsel --lam 0 > $O/ab_lam0.json 2> $O/ab_lam0.err
timeout -k 10 300 python3 -u tools/mmr_ab.py --libs product,vsel --lam 1 > $O/ab_lam1.json 2> $O/ab_lam1.err
