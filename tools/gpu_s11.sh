#!/bin/bash
# MMR probe-batch kernel: parity tests, then the config-5 workload.
set -e
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_hip_kernels.py -k mmr -x -v --timeout 120 --timeout-method thread > gpurun_out/s11_mmr_tests.log 2>&1
timeout -k 10 300 python -u bench.py --workload mmr --steps 3 --warmup 1 > gpurun_out/s11_mmr.json 2> gpurun_out/s11_mmr.err
