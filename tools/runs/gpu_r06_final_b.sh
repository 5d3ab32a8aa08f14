#!/bin/bash
# Round-6 final measurement, part B1: build-id-stamped PMC records of the
# same tree (FETCH_SIZE / WRITE_SIZE passes, tools/gpu_pmc_kernels.sh) for the
# headline, config 2 and config 5.
set -e
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
cd $R
bash tools/gpu_pmc_kernels.sh catalog score1m mmr
