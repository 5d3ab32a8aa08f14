#!/bin/bash
# Bench paths on one GPU: the headline line (with the CPU baseline), the
# config-5 MMR pipeline, and a 4-rank gloo rehearsal of the multi-GPU layouts
# (pure 4-way item sharding + the 2 x 2 alt grid) with list checks.
# Every GPU step has its own time limit; the first failure ends the script.
set -e
mkdir -p gpurun_out
timeout -k 10 300 python bench.py > gpurun_out/bc_bench.json 2> gpurun_out/bc_bench.err
timeout -k 10 300 python bench.py --workload mmr --no-cpu-baseline > gpurun_out/bc_mmr.json 2> gpurun_out/bc_mmr.err
timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 4 --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 4 --backend gloo --same-device --users 200000 --items 2000000 --steps 2 --warmup 1 --check-users 512 > gpurun_out/bc_rehearse4.json 2> gpurun_out/bc_rehearse4.err
