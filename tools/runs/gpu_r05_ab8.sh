#!/bin/bash
# Round-5 A/B 8: the guess's planner knobs on the pipelined d = 64 scan
# (config 2), one process, outputs bit-identical: first-tier margin z1 and
# offset c1, and the sample stride.
set -e
export TMPDIR=/tmp
O=gpurun_out/r05ab8
mkdir -p $O
timeout -k 10 400 python3 -u tools/variant_bench.py --libs product,product@guess_z1=2.5,product@guess_z1=2.0,product@guess_c1=0,product@guess_stride=16,product@guess_stride=64 --users 1000000 --items 1000000 --dim 64 --rounds 3 > $O/ab_cfg2.json 2> $O/ab_cfg2.err
