#!/bin/bash
# Round 6: ILD routing (streamed only for d = 128 cosine / dot, k > 40):
# the ILD tests, and the default plan against both forced kernels at d = 64,
# euclidean d = 128 and the headline shape.
set -e
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r06ir
mkdir -p $O
cd $R
true

timeout -k 10 200 python3 -u tools/ild_ab.py --variants stream,ild_stream=0,ild_stream=1 --kind euclidean --rounds 3 > $O/euclid.json 2> $O/euclid.err || true
timeout -k 10 200 python3 -u tools/ild_ab.py --variants stream,ild_stream=0,ild_stream=1 --dim 32 --rounds 5 > $O/d32.json 2> $O/d32.err || true
timeout -k 10 200 python3 -u tools/ild_ab.py --variants stream,ild_stream=0 --rounds 5 > $O/d128.json 2> $O/d128.err || true
