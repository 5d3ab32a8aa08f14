set -e
mkdir -p gpurun_out/z2
V=product,product@DIVREC_GUESS_Z1=3.0,product@DIVREC_GUESS_Z1=3.5,product@DIVREC_GUESS_Z1=2.0,product@DIVREC_GUESS_STRIDE=64,product@DIVREC_GUESS_STRIDE=64+DIVREC_GUESS_Z1=3.0
timeout -k 10 300 python tools/variant_bench.py --libs $V --users 1000000 --items 1000000 --dim 64 --k 100 > gpurun_out/z2/d64.json 2> gpurun_out/z2/d64.err
V2=product,product@DIVREC_GUESS_Z1=3.0,product@DIVREC_GUESS_Z1=3.5
timeout -k 10 400 python tools/variant_bench.py --libs $V2 --users 1000000 --items 10000000 --dim 128 --k 100 --rounds 3 > gpurun_out/z2/10m.json 2> gpurun_out/z2/10m.err
timeout -k 10 300 python tools/variant_bench.py --libs $V2 --users 262144 --items 10000000 --dim 128 --k 1000 > gpurun_out/z2/k1000.json 2> gpurun_out/z2/k1000.err
