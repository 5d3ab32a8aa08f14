#!/bin/bash
set -e
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/s18_gpu_tests.log 2>&1
timeout -k 10 300 python bench.py --workload score1m > gpurun_out/s18_score1m.json 2> gpurun_out/s18.err
timeout -k 10 300 python bench.py --items 1250000 --no-cpu-baseline > gpurun_out/s18_shard8.json 2>> gpurun_out/s18.err
