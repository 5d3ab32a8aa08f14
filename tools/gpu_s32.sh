#!/bin/bash
# Phase shares of the d=64 scan with eight user tiles per wave (diag build).
set -e
mkdir -p gpurun_out
timeout -k 10 200 python -u tools/diag_topk.py --users 1000000 --items 1000000 --dim 64 --k 100 > gpurun_out/s32_diag64.json 2> gpurun_out/s32.err
