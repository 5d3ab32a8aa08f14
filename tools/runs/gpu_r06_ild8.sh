#!/bin/bash
# Round 6: streamed ILD variants (lean id layout / MFMA-first) timed, and
# their diag builds' per-phase cycles per user (s_memtime), config-4 shape.
set -e
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r06ild8
mkdir -p $O
cd $R
timeout -k 10 200 python3 -u tools/ild_ab.py --variants stream,nl0mf1@stream,nl1mf0@stream,nl0mf0@stream,ild_stream=0 --rounds 5 >> $O/ab.jsonl 2>> $O/ab.err || true
timeout -k 10 200 python3 -u tools/ild_ab.py --variants lean1mf1@stream,lean0mf1@stream,lean1mf0@stream,lean0mf0@stream --rounds 2 >> $O/ab.jsonl 2>> $O/ab.err || true
timeout -k 10 200 python3 -u tools/ild_ab.py --variants lean1mf1@stream,lean0mf0@stream --k 10 --rounds 2 >> $O/ab.jsonl 2>> $O/ab.err || true
