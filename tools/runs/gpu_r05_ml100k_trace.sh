#!/bin/bash
# Round-5: kernel trace of config 1's evaluation step.
set -e
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r05ml100k
mkdir -p $O
cd /tmp
timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace -o t -- python3 $R/bench.py --workload ml100k --steps 5 --warmup 2 --no-cpu-baseline > $O/trace.log 2>&1
