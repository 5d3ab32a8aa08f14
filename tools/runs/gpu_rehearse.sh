# One-GPU rehearsal of the multi-rank bench paths on gloo (every rank on
# cuda:0): pure 4-way item sharding + the 2 x 2 alt grid with list checks,
# and the user-sharded config-5 pipeline on 2 ranks.
set -e
mkdir -p gpurun_out
timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 4 --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 4 --backend gloo --same-device --users 200000 --items 2000000 --steps 2 --warmup 1 --check-users 512 > gpurun_out/rh_catalog4.json 2> gpurun_out/rh_catalog4.err
timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29534 bench.py --workload mmr --gpus 2 --backend gloo --same-device --users 50000 --items 2000000 --steps 2 --warmup 1 > gpurun_out/rh_mmr2.json 2> gpurun_out/rh_mmr2.err
