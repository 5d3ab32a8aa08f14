#!/bin/bash
# HBM traffic of the headline step from rocprofv3 PMC counters: one pass per
# counter group (FETCH_SIZE and WRITE_SIZE cannot share a pass on gfx950),
# each over one bench step at the full config (MI355X_MICROARCH.md, HBM).
set -e
mkdir -p gpurun_out
cd /tmp
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $R/gpurun_out/pmc_fetch -o fetch -- python3 $R/bench.py --steps 1 --warmup 0 --no-cpu-baseline > $R/gpurun_out/pmc_fetch.log 2>&1
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $R/gpurun_out/pmc_write -o write -- python3 $R/bench.py --steps 1 --warmup 0 --no-cpu-baseline > $R/gpurun_out/pmc_write.log 2>&1
