#!/bin/bash
# Multi-rank rehearsal of the bench on ONE GPU: gloo process groups, every rank
# on cuda:0 (RCCL needs one GPU per rank; the 8-GPU runs are the driver's).
# Exercises the grid layout, the all_to_all exchange + merge and the max-over-
# ranks timing, and checks each rank's final lists against a one-device scan.
set -e
mkdir -p gpurun_out
R="python -m torch.distributed.run --nnodes=1 --master-addr 127.0.0.1"
timeout -k 10 300 $R --nproc-per-node 2 --master-port 29511 bench.py --gpus 2 --backend gloo --same-device --users 200000 --items 2000000 --steps 2 --warmup 1 --check-users 1024 > gpurun_out/s35_n2.json 2> gpurun_out/s35_n2.err
timeout -k 10 300 $R --nproc-per-node 4 --master-port 29512 bench.py --gpus 4 --backend gloo --same-device --users 200000 --items 2000000 --steps 2 --warmup 1 --check-users 1024 > gpurun_out/s35_n4.json 2> gpurun_out/s35_n4.err
timeout -k 10 300 $R --nproc-per-node 8 --master-port 29513 bench.py --gpus 8 --backend gloo --same-device --users 200000 --items 2000000 --steps 2 --warmup 1 --check-users 1024 > gpurun_out/s35_n8.json 2> gpurun_out/s35_n8.err
timeout -k 10 300 $R --nproc-per-node 4 --master-port 29514 bench.py --gpus 4 --backend gloo --same-device --item-shards 4 --users 200000 --items 2000000 --steps 2 --warmup 1 --check-users 1024 > gpurun_out/s35_n4s4.json 2> gpurun_out/s35_n4s4.err
