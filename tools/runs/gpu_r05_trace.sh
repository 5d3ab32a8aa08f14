#!/bin/bash
# Round 5: rocprofv3 kernel traces of config 2 and config 5 (top-1000 scan +
# MMR + ILD) on the current build.
set -e
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r05trace
mkdir -p $O
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/score1m -o trace -- python3 $R/bench.py --workload score1m --steps 2 --warmup 1 --no-cpu-baseline > $O/score1m.log 2>&1
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/mmr -o trace -- python3 $R/bench.py --workload mmr --steps 2 --warmup 1 --no-cpu-baseline > $O/mmr.log 2>&1
