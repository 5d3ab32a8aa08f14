#!/bin/bash
# Round-6 final measurement, part B2: PMC records of the other workloads with
# a traffic field, the MFMA-busy pass for the headline and config 2, the
# one-GPU multi-rank rehearsal, and the headline bench line again, now
# carrying the build-stamped counters (records of part B1 copied in first).
set -e
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
cd $R
bash tools/gpu_pmc_kernels.sh gather bpr fp32
bash tools/gpu_pmc_mfma.sh catalog score1m
O=gpurun_out/r06reh
mkdir -p $O
timeout -k 10 500 python3 bench.py --gpus 8 --backend gloo --same-device --check-users 1024 --steps 1 --warmup 0 --no-cpu-baseline > $O/catalog8.jsonl 2> $O/catalog8.err
timeout -k 10 400 python3 bench.py --workload mmr --gpus 2 --backend gloo --same-device --users 262144 --steps 1 --warmup 0 --no-cpu-baseline > $O/mmr2.jsonl 2> $O/mmr2.err
cp gpurun_out/pmck/pmc_*.json gpurun_out/pmcm/pmc_mfma_*.json profiles/
O=gpurun_out/r06fc
mkdir -p $O
timeout -k 10 300 python3 bench.py > $O/bench.jsonl 2> $O/bench.err
