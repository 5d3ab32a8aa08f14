#!/bin/bash
# Round 6: kernel-level time split of config 2 (bench.py --workload score1m).
set -e
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r06tr2
mkdir -p $O
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace -o trace -- python3 $R/bench.py --workload score1m --steps 3 --warmup 1 --no-cpu-baseline > $O/bench.jsonl 2> $O/bench.err
