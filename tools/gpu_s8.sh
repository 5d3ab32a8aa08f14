#!/bin/bash
# Re-entry check of the restored tree + shard-size scan scaling (the per-rank
# scan of the 8-GPU config is 1M users x 1.25M items).
set -e
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/s8_gpu_tests.log 2>&1
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/s8_smoke.log 2>&1
timeout -k 10 400 python bench.py > gpurun_out/s8_bench.json 2> gpurun_out/s8_bench.err
for n in 1250000 2500000 5000000; do
  timeout -k 10 300 python bench.py --items $n --no-cpu-baseline > gpurun_out/s8_bench_I$n.json 2>> gpurun_out/s8_bench.err
done
