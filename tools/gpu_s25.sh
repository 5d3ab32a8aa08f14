#!/bin/bash
set -e
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/s25_gpu_tests.log 2>&1
timeout -k 10 300 python bench.py --workload bpr > gpurun_out/s25_bpr.json 2> gpurun_out/s25.err
