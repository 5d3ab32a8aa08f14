#!/bin/bash
set -e
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/s6_gpu_tests.log 2>&1
timeout -k 10 300 python -u tools/variant_bench.py --libs product --users 1000000 --items 1000000 --dim 64 --rounds 2 > gpurun_out/s6_1m64.json 2> gpurun_out/s6_1m64.err
timeout -k 10 300 python -u tools/variant_bench.py --libs product --users 262144 --items 1000000 --dim 64 --rounds 2 > gpurun_out/s6_262k64.json 2> gpurun_out/s6_262k64.err
for w in bpr score1m; do
  timeout -k 10 300 python -u bench.py --workload $w --no-cpu-baseline > gpurun_out/s6_wl_$w.json 2> gpurun_out/s6_wl_$w.err
done
timeout -k 10 400 python -u bench.py --no-cpu-baseline > gpurun_out/s6_bench.json 2> gpurun_out/s6_bench.err
