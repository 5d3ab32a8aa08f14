#!/bin/bash
set -e
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_hip_kernels.py -k mmr -x -q --timeout 120 --timeout-method thread > gpurun_out/s12_mmr_tests.log 2>&1
timeout -k 10 300 python -u tools/mmr_sweep.py > gpurun_out/s12_mmr_sweep.jsonl 2> gpurun_out/s12.err
