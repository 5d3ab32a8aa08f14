#!/bin/bash
# Round-6 final measurement, part A2: the headline bench line, every
# secondary line, and rocprofv3 kernel-trace --stats summaries of the
# headline, config 2 and config 5 (program directly after --). Each GPU step has its own time limit; the
# first failure ends the script.
set -e
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r06fa
mkdir -p $O
cd $R
timeout -k 10 300 python3 -u -m pytest tests/test_hip_kernels.py -m gpu -k dense_sample_chunked_units -v --timeout 200 --timeout-method thread -p no:cacheprovider > $O/gpu_tests_rerun.log 2>&1
timeout -k 10 120 python3 -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1
timeout -k 10 300 python3 bench.py > $O/bench.jsonl 2> $O/bench.err
for w in score1m mmr gather bpr fp32 ml100k excl; do
  timeout -k 10 300 python3 bench.py --workload $w --steps 3 --warmup 1 >> $O/workloads.jsonl 2>> $O/workloads.err
done
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace -o trace -- python3 $R/bench.py --steps 2 --warmup 1 --no-cpu-baseline > $O/trace.log 2>&1
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/score1m_trace -o trace -- python3 $R/bench.py --workload score1m --steps 2 --warmup 1 --no-cpu-baseline > $O/score1m_trace.log 2>&1
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/mmr_trace -o trace -- python3 $R/bench.py --workload mmr --steps 2 --warmup 1 --no-cpu-baseline > $O/mmr_trace.log 2>&1
