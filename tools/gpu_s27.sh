#!/bin/bash
set -e
mkdir -p gpurun_out
timeout -k 10 400 python bench.py > gpurun_out/s27_bench.json 2> gpurun_out/s27.err
timeout -k 10 300 python bench.py --workload bpr --no-cpu-baseline > gpurun_out/s27_bpr.json 2>> gpurun_out/s27.err
