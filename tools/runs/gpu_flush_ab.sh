set -e
mkdir -p gpurun_out/flush
V=product,oldflush,product@DIVREC_GUESS_Z1=2.5
timeout -k 10 300 python tools/variant_bench.py --libs $V --users 262144 --items 10000000 --dim 128 --k 1000 > gpurun_out/flush/k1000_262k.json 2> gpurun_out/flush/k1000_262k.err
timeout -k 10 400 python tools/variant_bench.py --libs product,oldflush --users 1000000 --items 10000000 --dim 128 --k 1000 --rounds 2 > gpurun_out/flush/k1000_1m.json 2> gpurun_out/flush/k1000_1m.err
