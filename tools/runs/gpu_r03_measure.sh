#!/bin/bash
# Round-3 measurement pass on one MI355X: the headline bench line, its rocprofv3
# kernel-trace summary, the MFMA-utilisation counter pass (catalog + config 2),
# and the config-5 (mmr) and config-2 (score1m) lines. Each GPU step has its
# own time limit; the first failure ends the script.
set -e
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r03m
mkdir -p $O
cd $R
timeout -k 10 300 python3 bench.py > $O/bench.jsonl 2> $O/bench.err
timeout -k 10 300 python3 bench.py --workload mmr --steps 2 --warmup 1 > $O/mmr.jsonl 2> $O/mmr.err
timeout -k 10 300 python3 bench.py --workload score1m --steps 5 --warmup 2 > $O/score1m.jsonl 2> $O/score1m.err
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace -o trace -- python3 $R/bench.py --steps 2 --warmup 1 --no-cpu-baseline > $O/trace.log 2>&1
cd $R
bash tools/gpu_pmc_mfma.sh catalog score1m
