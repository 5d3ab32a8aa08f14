set -e
mkdir -p gpurun_out
timeout -k 10 300 python -u tools/variant_bench.py --libs product,abi1base --users 1000000 --items 1000000 --dim 64 --rounds 3 > gpurun_out/ab_d64.json 2> gpurun_out/ab_d64.err
timeout -k 10 300 python -u tools/variant_bench.py --libs product,abi1base --users 262144 --items 10000000 --dim 128 --rounds 3 > gpurun_out/ab_d128.json 2> gpurun_out/ab_d128.err
timeout -k 10 300 python -u tools/variant_bench.py --libs product,abi1base --users 262144 --items 10000000 --dim 128 --k 1000 --rounds 2 > gpurun_out/ab_k1000.json 2> gpurun_out/ab_k1000.err
