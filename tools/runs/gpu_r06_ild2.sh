#!/bin/bash
# Round 6: where the streamed ILD's time goes: the product stream kernel, the
# one-wave-per-user kernel, exp1 (no row DMA: lists + compute only) and exp2
# (no compute: the DMA pipeline alone), over 10M / 1M / 100K-row tables.
set -e
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r06ild2
mkdir -p $O
cd $R
for it in 10000000 1000000 100000; do
  timeout -k 10 200 python3 -u tools/ild_ab.py --variants stream,ild_stream=0,exp1@stream,exp2@stream --items $it --rounds 3 >> $O/ab.jsonl 2>> $O/ab.err || true
done
timeout -k 10 200 python3 -u tools/ild_ab.py --variants stream,ild_stream=0,exp1@stream,exp2@stream --k 10 --rounds 3 >> $O/ab.jsonl 2>> $O/ab.err || true
