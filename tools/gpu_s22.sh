#!/bin/bash
set -e
mkdir -p gpurun_out
timeout -k 10 300 python bench.py --no-cpu-baseline --steps 2 > gpurun_out/s22_bench.json 2> gpurun_out/s22.err
timeout -k 10 300 python bench.py --workload gather --no-cpu-baseline > gpurun_out/s22_gather.json 2>> gpurun_out/s22.err
