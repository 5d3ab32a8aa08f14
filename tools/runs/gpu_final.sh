#!/bin/bash
# End-of-session GPU pass, part 1: parity suite, smoke, headline bench with its
# CPU baseline, rocprofv3 kernel summary of the headline, every secondary
# workload line. Part 2 (PMC traffic): bash tools/gpu_pmc_kernels.sh catalog mmr
set -e
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/f_tests.log 2>&1
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/f_smoke.log 2>&1
timeout -k 10 400 python bench.py > gpurun_out/f_bench.log 2>&1
cd /tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/f_prof -o bench -- python3 $GRAFT_REPO_ROOT/bench.py --steps 2 --warmup 1 --no-cpu-baseline > $GRAFT_REPO_ROOT/gpurun_out/f_prof.log 2>&1
cd $GRAFT_REPO_ROOT
for w in score1m gather bpr mmr fp32 ml100k; do
  timeout -k 10 300 python bench.py --workload $w > gpurun_out/f_wl_$w.json 2> gpurun_out/f_wl_$w.err
done
