#!/bin/bash
# Round 6: the piece ring's depth P (ild_bufs = ring slots per wave) at the
# config-4 shape: P = 25 (one list, the old NB = 1 depth), 28, 31, 34, 37 (default)
set -e
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r06ild6
mkdir -p $O
cd $R
timeout -k 10 200 python3 -u tools/ild_ab.py --variants stream,ild_bufs=25,ild_bufs=28,ild_bufs=31,ild_bufs=34,exp2@ild_bufs=25,exp1@ild_bufs=25 --rounds 3 >> $O/ab.jsonl 2>> $O/ab.err || true
timeout -k 10 200 python3 -u tools/ild_ab.py --variants stream,ild_bufs=3,ild_bufs=6,ild_bufs=12,ild_bufs=24 --k 10 --rounds 3 >> $O/ab.jsonl 2>> $O/ab.err || true
