#!/bin/bash
# One GPU session: parity tests, smoke, headline bench, rocprofv3 kernel
# summary of the headline step, and the secondary workload lines.
# Every GPU step has its own time limit; the first failure ends the script.
set -e
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1
timeout -k 10 400 python bench.py > gpurun_out/bench.log 2>&1
cd /tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/prof -o bench -- python3 $GRAFT_REPO_ROOT/bench.py --steps 2 --warmup 1 --no-cpu-baseline > $GRAFT_REPO_ROOT/gpurun_out/prof.log 2>&1
cd $GRAFT_REPO_ROOT
timeout -k 10 300 python bench.py --workload score1m > gpurun_out/wl_score1m.json 2> gpurun_out/wl_score1m.err
timeout -k 10 300 python bench.py --workload mmr > gpurun_out/wl_mmr.json 2> gpurun_out/wl_mmr.err
timeout -k 10 300 python bench.py --workload gather > gpurun_out/wl_gather.json 2> gpurun_out/wl_gather.err
timeout -k 10 300 python bench.py --workload bpr > gpurun_out/wl_bpr.json 2> gpurun_out/wl_bpr.err
