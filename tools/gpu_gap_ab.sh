# Score-scan A/B of knob variants at config 2 (d=64) and the 8-way shard
# shape (d=128, 1M x 1.25M). Usage: bash tools/gpu_gap_ab.sh LIBS TAG
set -e
mkdir -p gpurun_out
timeout -k 10 300 python tools/variant_bench.py --libs $1 --users 1000000 --items 1000000 --dim 64 > gpurun_out/ab_$2_d64.json 2> gpurun_out/ab_$2_d64.err
timeout -k 10 300 python tools/variant_bench.py --libs $1 --users 1000000 --items 1250000 --dim 128 > gpurun_out/ab_$2_shard8.json 2> gpurun_out/ab_$2_shard8.err
