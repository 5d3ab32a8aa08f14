#!/bin/bash
# Parity suite (optionally a -k selection first), then the headline bench and
# the named secondary workload lines, each under its own time limit; the first
# failure ends the script.   usage: tools/runs/gpu_step.sh [-k EXPR] [workload ...]
set -e
mkdir -p gpurun_out
if [ "$1" = "-k" ]; then
  timeout -k 10 300 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread -k "$2" > gpurun_out/s_sel.log 2>&1
  shift 2
fi
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/s_all.log 2>&1
timeout -k 10 400 python bench.py --no-cpu-baseline > gpurun_out/s_bench.json 2> gpurun_out/s_bench.err
for w in "$@"; do
  timeout -k 10 300 python bench.py --workload $w --no-cpu-baseline > gpurun_out/s_$w.json 2> gpurun_out/s_$w.err
done
