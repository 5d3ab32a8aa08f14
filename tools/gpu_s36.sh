#!/bin/bash
# HBM traffic (PMC, one counter group per pass) of one dr_score_topk call:
# headline config (1M x 10M, d=128) and config 2 (1M x 1M, d=64).
set -e
mkdir -p gpurun_out
cd /tmp
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
B="$R/bench.py --steps 1 --warmup 0 --no-cpu-baseline"
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $R/gpurun_out/pmc_fetch -o fetch -- python3 $B > $R/gpurun_out/pmc_fetch.log 2>&1
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $R/gpurun_out/pmc_write -o write -- python3 $B > $R/gpurun_out/pmc_write.log 2>&1
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $R/gpurun_out/pmc1m_fetch -o fetch -- python3 $B --workload score1m > $R/gpurun_out/pmc1m_fetch.log 2>&1
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $R/gpurun_out/pmc1m_write -o write -- python3 $B --workload score1m > $R/gpurun_out/pmc1m_write.log 2>&1
