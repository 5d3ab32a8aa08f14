#!/bin/bash
# Round 6: the new full-size tests (bench's own tables vs float64; config-3
# BPR step), the headline bench line with its fp64 check field, and the
# streamed/per-user ILD crossover at k = 40 / 64.
set -e
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r06chk1
mkdir -p $O
cd $R
timeout -k 10 600 python3 -u -m pytest tests/test_real_plans.py -k "bpr_config3" -x -v --timeout 500 --timeout-method thread -p no:cacheprovider > $O/tests.log 2>&1
timeout -k 10 300 python3 bench.py --no-cpu-baseline > $O/bench.jsonl 2> $O/bench.err
for k in 40 64; do
timeout -k 10 200 python3 -u tools/ild_ab.py --variants stream,ild_stream=0 --k $k --rounds 3 >> $O/ild.jsonl 2>> $O/ild.err || true
done
