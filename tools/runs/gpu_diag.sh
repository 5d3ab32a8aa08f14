#!/bin/bash
# Phase shares + in-kernel clock of the score scan (instrumented diag library).
set -e
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 200 python -u tools/diag_topk.py --users 131072 --items 10000000 --dim 128 --k 100 > gpurun_out/diag128.json 2> gpurun_out/diag128.err
timeout -k 10 200 python -u tools/diag_topk.py --users 262144 --items 1000000 --dim 64 --k 100 > gpurun_out/diag64.json 2> gpurun_out/diag64.err
