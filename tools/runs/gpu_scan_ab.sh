# Score-scan A/B (tools/variant_bench.py, outputs must be identical) at
# config 2 (d=64, 1M x 1M), d=32 and the k=1000 shape; then the scan parity
# tests. Usage: bash tools/runs/gpu_scan_ab.sh product,VARIANT[,...] TAG
set -e
mkdir -p gpurun_out
L=$1; T=$2
timeout -k 10 300 python tools/variant_bench.py --libs $L --users 1000000 --items 1000000 --dim 64 > gpurun_out/ab_${T}_d64.json 2> gpurun_out/ab_${T}_d64.err
timeout -k 10 300 python tools/variant_bench.py --libs $L --users 1000000 --items 1000000 --dim 32 > gpurun_out/ab_${T}_d32.json 2> gpurun_out/ab_${T}_d32.err
timeout -k 10 300 python tools/variant_bench.py --libs $L --users 262144 --items 10000000 --dim 128 > gpurun_out/ab_${T}_d128.json 2> gpurun_out/ab_${T}_d128.err
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/ab_${T}_tests.log 2>&1
