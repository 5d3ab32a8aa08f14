#!/bin/bash
# Full round check: GPU tests, smoke, headline bench, rocprof kernel summary,
# PMC HBM traffic passes, secondary workloads. First failure ends the script.
set -e
mkdir -p gpurun_out
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/s13_gpu_tests.log 2>&1
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/s13_smoke.log 2>&1
timeout -k 10 400 python bench.py > gpurun_out/s13_bench.json 2> gpurun_out/s13_bench.err
cd /tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/s13_prof -o bench -- python3 $R/bench.py --steps 2 --warmup 1 --no-cpu-baseline > $R/gpurun_out/s13_prof.log 2>&1
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $R/gpurun_out/s13_pmc_fetch -o fetch -- python3 $R/bench.py --steps 1 --warmup 0 --no-cpu-baseline > $R/gpurun_out/s13_pmc_fetch.log 2>&1
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $R/gpurun_out/s13_pmc_write -o write -- python3 $R/bench.py --steps 1 --warmup 0 --no-cpu-baseline > $R/gpurun_out/s13_pmc_write.log 2>&1
cd $R
for w in score1m mmr gather bpr; do
  timeout -k 10 300 python bench.py --workload $w >> gpurun_out/s13_workloads.jsonl 2>> gpurun_out/s13_workloads.err
done
