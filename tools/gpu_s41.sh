#!/bin/bash
# Device pairwise sampler: parity/distribution tests, full GPU suite, BPR line.
set -e
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/s41_tests.log 2>&1
timeout -k 10 300 python bench.py --workload bpr > gpurun_out/s41_bpr.json 2> gpurun_out/s41.err
