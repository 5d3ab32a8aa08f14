#!/bin/bash
# Round-5: where config 2's time goes after the dense sample scan: kernel
# trace of the score1m workload (product) and the diag build's phase shares
# of the main scan.
set -e
export TMPDIR=/tmp
O=gpurun_out/r05diag2
mkdir -p $O
R=$GRAFT_REPO_ROOT
cd /tmp
timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d $R/$O/trace -o trace -- python3 $R/bench.py --workload score1m --steps 3 --warmup 1 --no-cpu-baseline > $R/$O/trace.log 2>&1
cd $R
timeout -k 10 300 python3 -u tools/diag_topk.py --users 1000000 --items 1000000 --dim 64 --k 100 > $O/diag_cfg2.json 2> $O/diag_cfg2.err
