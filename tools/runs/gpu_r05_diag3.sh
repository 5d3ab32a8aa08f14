#!/bin/bash
# Round-5: phase shares of the headline's main scan (diag build), 1M x 10M d=128.
set -e
export TMPDIR=/tmp
O=gpurun_out/r05diag3
mkdir -p $O
timeout -k 10 300 python3 -u tools/diag_topk.py --users 1000000 --items 10000000 --dim 128 --k 100 > $O/diag_10m.json 2> $O/diag_10m.err
