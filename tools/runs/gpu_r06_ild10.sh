#!/bin/bash
# Round 6: streamed ILD (pieces issued up front, tile-by-tile Gram) and
# sched_group_barrier variants interleaving VALU into the MFMA chains.
set -e
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r06ild10
mkdir -p $O
cd $R
timeout -k 10 400 python3 -u -m pytest tests/test_hip_kernels.py -k "ild_embedding" -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > $O/tests.log 2>&1
timeout -k 10 200 python3 -u tools/ild_ab.py --variants stream,sgb2@stream,sgb4@stream,sgb6@stream,ild_stream=0,diag1@stream --rounds 5 >> $O/ab.jsonl 2>> $O/ab.err || true
timeout -k 10 200 python3 -u tools/ild_ab.py --variants stream,sgb2@stream,sgb4@stream,sgb6@stream,ild_stream=0 --items 100000 --rounds 3 >> $O/ab.jsonl 2>> $O/ab.err || true
timeout -k 10 200 python3 -u tools/ild_ab.py --variants stream,ild_stream=0,diag1@stream --k 10 --rounds 3 >> $O/ab.jsonl 2>> $O/ab.err || true
