#!/bin/bash
# Round 6: ILD producer/consumer waves (ild_stream = 2) against the streamed
# kernel (1) and the one-wave-per-user kernel (0): parity tests, then A/B at
# the config-4 shape, k = 10 / 40 / 64, d = 64.
set -e
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r06ild11
mkdir -p $O
cd $R
timeout -k 10 500 python3 -u -m pytest tests/test_hip_kernels.py tests/test_real_plans.py -k "ild_embedding or beyond_2_28" -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > $O/tests.log 2>&1
timeout -k 10 200 python3 -u tools/ild_ab.py --variants stream,ild_stream=2,ild_stream=0 --rounds 5 >> $O/ab.jsonl 2>> $O/ab.err || true
timeout -k 10 200 python3 -u tools/ild_ab.py --variants stream,ild_stream=2,ild_stream=0 --items 100000 --rounds 3 >> $O/ab.jsonl 2>> $O/ab.err || true
for k in 10 40 64; do
timeout -k 10 200 python3 -u tools/ild_ab.py --variants stream,ild_stream=2,ild_stream=0 --k $k --rounds 3 >> $O/ab.jsonl 2>> $O/ab.err || true
done
timeout -k 10 200 python3 -u tools/ild_ab.py --variants stream,ild_stream=2,ild_stream=0 --dim 64 --rounds 3 >> $O/ab.jsonl 2>> $O/ab.err || true
