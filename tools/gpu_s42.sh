#!/bin/bash
# gather_dot backward: contiguous 32-lane row layout (product) vs 16-B chunks.
set -e
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_hip_kernels.py -x -v --timeout 120 --timeout-method thread -k gather > gpurun_out/s42_tests.log 2>&1
timeout -k 10 300 python bench.py --workload gather --no-cpu-baseline > gpurun_out/s42_rows.json 2> gpurun_out/s42.err
DIVREC_HIP_LIB=$PWD/diversity-recommendations_amd/divrec/_lib/libdivrec_hip_bwdvec.so timeout -k 10 300 python bench.py --workload gather --no-cpu-baseline > gpurun_out/s42_vec.json 2>> gpurun_out/s42.err
