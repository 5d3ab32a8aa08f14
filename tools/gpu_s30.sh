#!/bin/bash
# Product with eight user tiles per wave at d <= 64: parity suite, config-2
# workload line and its rocprof kernel summary.
set -e
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/s30_tests.log 2>&1
timeout -k 10 300 python bench.py --workload score1m > gpurun_out/s30_score1m.json 2> gpurun_out/s30.err
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/prof_s30 -o score1m -- python3 $GRAFT_REPO_ROOT/bench.py --workload score1m --steps 3 --warmup 1 --no-cpu-baseline > $GRAFT_REPO_ROOT/gpurun_out/s30_prof.log 2>&1
