#!/bin/bash
# Round-5: lower bound of the non-resident-row MMR layout (tools/probes/mmr_fold.py).
set -e
export TMPDIR=/tmp
O=gpurun_out/r05mmrfold
mkdir -p $O
timeout -k 10 300 python3 -u tools/probes/mmr_fold.py > $O/mmr_fold.json 2> $O/mmr_fold.err
