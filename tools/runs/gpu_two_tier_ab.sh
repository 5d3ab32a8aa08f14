set -e
mkdir -p gpurun_out/t2
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread -k "score_topk or real_plans or recommendations or distributed_gpu" > gpurun_out/t2/tests.log 2>&1
timeout -k 10 300 python tools/variant_bench.py --libs product,product@DIVREC_GUESS_TIGHT=0 --users 1000000 --items 1000000 --dim 64 --k 100 > gpurun_out/t2/ab_d64.json 2> gpurun_out/t2/ab_d64.err
timeout -k 10 300 python tools/variant_bench.py --libs product,product@DIVREC_GUESS_TIGHT=0 --users 1000000 --items 10000000 --dim 128 --k 100 > gpurun_out/t2/ab_10m.json 2> gpurun_out/t2/ab_10m.err
timeout -k 10 300 python tools/variant_bench.py --libs product,product@DIVREC_GUESS_TIGHT=0 --users 262144 --items 10000000 --dim 128 --k 1000 > gpurun_out/t2/ab_k1000.json 2> gpurun_out/t2/ab_k1000.err
