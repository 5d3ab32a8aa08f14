#!/bin/bash
# Round-4 final measurement, part B: build-id-stamped PMC records of the same
# tree — FETCH_SIZE / WRITE_SIZE passes (tools/gpu_pmc_kernels.sh) for the
# headline, config 2 and config 5, and the MFMA-busy pass
# (tools/gpu_pmc_mfma.sh) for the headline and config 2.
set -e
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
cd $R
bash tools/gpu_pmc_kernels.sh catalog score1m mmr
bash tools/gpu_pmc_mfma.sh catalog score1m
