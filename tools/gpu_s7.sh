#!/bin/bash
set -e
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/s7_gpu_tests.log 2>&1
LIBS=product,enqloop,enqloop4
timeout -k 10 300 python -u tools/variant_bench.py --libs $LIBS --users 131072 --items 10000000 --dim 128 --rounds 3 > gpurun_out/s7_bench128.json 2> gpurun_out/s7_bench128.err
timeout -k 10 300 python -u tools/variant_bench.py --libs $LIBS --users 262144 --items 1000000 --dim 64 --rounds 3 > gpurun_out/s7_bench64.json 2> gpurun_out/s7_bench64.err
bash tools/gpu_diag.sh
