#!/bin/bash
# Round-4 final measurement, part C (same build as parts A/B): PMC traffic of
# the secondary HBM-bound lines (gather, BPR, fp32 scoring), the one-GPU
# multi-rank rehearsal, and the headline bench line again now that the
# build-stamped PMC records of parts B and C are in profiles/.
set -e
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
cd $R
bash tools/gpu_pmc_kernels.sh gather bpr fp32
bash tools/runs/gpu_r04_rehearse.sh
mkdir -p gpurun_out/r04fc
timeout -k 10 300 python3 bench.py > gpurun_out/r04fc/bench.jsonl 2> gpurun_out/r04fc/bench.err
