# One-GPU rehearsal of the multi-rank bench paths on gloo (every rank on
# cuda:0) with the round-3 build: 8-way item sharding with global thresholds
# (the default --gpus 8 layout) with list checks, and the user-sharded
# config-5 pipeline (persistent MMR grid per rank) on 2 ranks.
set -e
mkdir -p gpurun_out/rh3
timeout -k 10 500 python -m torch.distributed.run --nnodes=1 --nproc-per-node 8 --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 8 --backend gloo --same-device --users 200000 --items 4000000 --steps 2 --warmup 1 --check-users 512 > gpurun_out/rh3/catalog8.json 2> gpurun_out/rh3/catalog8.err
timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29534 bench.py --workload mmr --gpus 2 --backend gloo --same-device --users 50000 --items 2000000 --steps 2 --warmup 1 > gpurun_out/rh3/mmr2.json 2> gpurun_out/rh3/mmr2.err
