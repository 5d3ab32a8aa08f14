set -e
mkdir -p gpurun_out/capab
timeout -k 10 400 python tools/variant_bench.py --libs product,cap1k,cap1kg3,gap124 --users 262144 --items 10000000 --dim 128 --k 100 > gpurun_out/capab/k100_262k.json 2> gpurun_out/capab/k100_262k.err
timeout -k 10 400 python tools/variant_bench.py --libs product,cap1k,cap1kg3 --users 1000000 --items 1000000 --dim 64 --k 100 > gpurun_out/capab/d64_1m.json 2> gpurun_out/capab/d64_1m.err
