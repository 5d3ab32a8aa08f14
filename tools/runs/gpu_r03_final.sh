#!/bin/bash
# Round-3 final pass: GPU tests + smoke, the headline bench line (+ its rocprofv3
# kernel-trace summary), the secondary lines, the PMC traffic passes (catalog,
# config 2, config 5) and the MFMA-busy counter pass. Each GPU step has its own
# time limit; the first failure ends the script.
set -e
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r03f
mkdir -p $O
cd $R
timeout -k 10 600 python3 -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread > $O/gpu_tests.log 2>&1
timeout -k 10 120 python3 -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1
timeout -k 10 300 python3 bench.py > $O/bench.jsonl 2> $O/bench.err
for w in score1m mmr gather bpr fp32 ml100k excl; do
  timeout -k 10 300 python3 bench.py --workload $w --steps 3 --warmup 1 >> $O/workloads.jsonl 2>> $O/workloads.err
done
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace -o trace -- python3 $R/bench.py --steps 2 --warmup 1 --no-cpu-baseline > $O/trace.log 2>&1
cd $R
