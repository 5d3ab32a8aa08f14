# Score-scan A/B at d=128 on the 8-way item-shard shape (1M x 1.25M) and the
# single-GPU shape (262144 x 10M). Usage: bash tools/gpu_scan_ab2.sh LIBS TAG
set -e
mkdir -p gpurun_out
L=$1; T=$2
timeout -k 10 300 python tools/variant_bench.py --libs $L --users 1000000 --items 1250000 --dim 128 > gpurun_out/ab_${T}_shard8.json 2> gpurun_out/ab_${T}_shard8.err
timeout -k 10 300 python tools/variant_bench.py --libs $L --users 262144 --items 10000000 --dim 128 > gpurun_out/ab_${T}_d128.json 2> gpurun_out/ab_${T}_d128.err
