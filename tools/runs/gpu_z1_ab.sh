set -e
mkdir -p gpurun_out/z1
V=product,product@DIVREC_GUESS_Z1=1.5,product@DIVREC_GUESS_Z1=1.0,product@DIVREC_GUESS_Z1=0.5,product@DIVREC_GUESS_Z1=1.0+DIVREC_GUESS_C1=0
timeout -k 10 300 python tools/variant_bench.py --libs $V --users 1000000 --items 1000000 --dim 64 --k 100 > gpurun_out/z1/d64.json 2> gpurun_out/z1/d64.err
timeout -k 10 400 python tools/variant_bench.py --libs $V --users 1000000 --items 10000000 --dim 128 --k 100 --rounds 2 > gpurun_out/z1/10m.json 2> gpurun_out/z1/10m.err
timeout -k 10 300 python tools/variant_bench.py --libs $V --users 262144 --items 10000000 --dim 128 --k 1000 > gpurun_out/z1/k1000.json 2> gpurun_out/z1/k1000.err
