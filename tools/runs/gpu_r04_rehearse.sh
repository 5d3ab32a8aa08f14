#!/bin/bash
# One-GPU rehearsal of the driver's multi-GPU bench with the final build:
# bench.py --gpus N launching its own ranks (gloo groups, every rank on
# cuda:0): 8 ranks in the default 8-way item-sharded layout plus the 4 x 2
# grid, with the multi-rank list check; and config 5 user-sharded over 2
# ranks. Throughput here is meaningless (the ranks share one GPU).
set -e
export TMPDIR=/tmp
O=gpurun_out/r04reh
mkdir -p $O
timeout -k 10 500 python3 bench.py --gpus 8 --backend gloo --same-device --check-users 1024 --steps 1 --warmup 0 --no-cpu-baseline > $O/catalog8.jsonl 2> $O/catalog8.err
timeout -k 10 400 python3 bench.py --workload mmr --gpus 2 --backend gloo --same-device --users 262144 --steps 1 --warmup 0 --no-cpu-baseline > $O/mmr2.jsonl 2> $O/mmr2.err
