#!/bin/bash
# Round 6: first run of the streamed ILD kernel: its parity tests (bit-identical
# to the one-wave-per-user kernel, float64 oracle), then in-process A/B at the
# config-4 shape (1M users x top-100, 10M x 128 bf16, cosine) and at k = 10.
set -e
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r06ild1
mkdir -p $O
cd $R
timeout -k 10 400 python3 -u -m pytest tests/test_hip_kernels.py -k "ild_embedding" -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > $O/tests.log 2>&1
timeout -k 10 200 python3 -u tools/ild_ab.py --variants stream,ild_stream=0 --rounds 5 > $O/ab_k100.json 2> $O/ab_k100.err
timeout -k 10 200 python3 -u tools/ild_ab.py --variants stream,ild_stream=0,ild_bufs=4,ild_bufs=2 --k 10 --rounds 5 > $O/ab_k10.json 2> $O/ab_k10.err
timeout -k 10 200 python3 -u tools/ild_ab.py --variants stream,ild_stream=0 --dim 64 --rounds 5 > $O/ab_k100_d64.json 2> $O/ab_k100_d64.err
