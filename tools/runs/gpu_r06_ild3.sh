#!/bin/bash
# Round 6: streamed ILD with the weighted-column epilogue: parity tests, then
# A/B against the one-wave-per-user kernel and the exp1 (no row DMA) / exp2
# (no compute) floors at the config-4 shape, k = 10, d = 64.
set -e
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r06ild3
mkdir -p $O
cd $R
timeout -k 10 400 python3 -u -m pytest tests/test_hip_kernels.py -k "ild_embedding" -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > $O/tests.log 2>&1
timeout -k 10 200 python3 -u tools/ild_ab.py --variants stream,ild_stream=0,exp1@stream,exp2@stream --rounds 5 >> $O/ab.jsonl 2>> $O/ab.err || true
timeout -k 10 200 python3 -u tools/ild_ab.py --variants stream,ild_stream=0,exp1@stream,exp2@stream --items 100000 --rounds 3 >> $O/ab.jsonl 2>> $O/ab.err || true
timeout -k 10 200 python3 -u tools/ild_ab.py --variants stream,ild_stream=0,exp1@stream,exp2@stream --k 10 --rounds 3 >> $O/ab.jsonl 2>> $O/ab.err || true
timeout -k 10 200 python3 -u tools/ild_ab.py --variants stream,ild_stream=0,exp1@stream,exp2@stream --dim 64 --rounds 3 >> $O/ab.jsonl 2>> $O/ab.err || true
timeout -k 10 200 python3 -u tools/ild_ab.py --variants stream,ild_stream=0 --kind euclidean --rounds 3 >> $O/ab.jsonl 2>> $O/ab.err || true
