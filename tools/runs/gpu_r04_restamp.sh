#!/bin/bash
# One-call re-measurement of a new build: the PMC traffic and MFMA-busy passes
# of every bench workload (stamped with this build's id), copied into
# profiles/ on the box so that the bench lines of part A carry them, then
# final part A (GPU tests, smoke, bench, workloads, kernel traces).
set -e
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
cd $R
bash tools/gpu_pmc_kernels.sh catalog score1m mmr gather bpr fp32
bash tools/gpu_pmc_mfma.sh catalog score1m
cp gpurun_out/pmck/pmc_*.json profiles/
cp gpurun_out/pmcm/pmc_mfma_*.json profiles/
bash tools/runs/gpu_r04_final_a.sh
