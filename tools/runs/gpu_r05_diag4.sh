#!/bin/bash
# Round-5: phase shares of the k = 1000 main scan (diag build of the final tree).
set -e
export TMPDIR=/tmp
O=gpurun_out/r05diag4
mkdir -p $O
timeout -k 10 300 python3 -u tools/diag_topk.py --users 262144 --items 10000000 --dim 128 --k 1000 > $O/diag_k1000.json 2> $O/diag_k1000.err
timeout -k 10 300 python3 -u tools/diag_topk.py --users 262144 --items 10000000 --dim 128 --k 100 > $O/diag_k100.json 2> $O/diag_k100.err
