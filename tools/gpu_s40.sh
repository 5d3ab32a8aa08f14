#!/bin/bash
# Row-sparse (lazy) Adam: parity tests and the BPR workload line.
set -e
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_api_gpu.py -x -v --timeout 120 --timeout-method thread -k "adam_rows or sparse_adam or bpr or adam" > gpurun_out/s40_tests.log 2>&1
timeout -k 10 300 python bench.py --workload bpr > gpurun_out/s40_bpr.json 2> gpurun_out/s40.err
