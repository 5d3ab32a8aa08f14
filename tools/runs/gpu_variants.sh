#!/bin/bash
# GPU session: parity tests of the product library, then the in-process A/B
# of the score-scan variants (tools/build_variants.sh) at two shapes.
set -e
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/v_gpu_tests.log 2>&1
LIBS=product,base,nut2,prio,noapipe,pre,ring3,gap32,gap256
timeout -k 10 400 python -u tools/variant_bench.py --libs $LIBS --users 131072 --items 10000000 --dim 128 --rounds 3 > gpurun_out/v_bench128.json 2> gpurun_out/v_bench128.err
timeout -k 10 400 python -u tools/variant_bench.py --libs $LIBS --users 262144 --items 1000000 --dim 64 --rounds 3 > gpurun_out/v_bench64.json 2> gpurun_out/v_bench64.err
