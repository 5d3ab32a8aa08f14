set -e
mkdir -p gpurun_out/enq
timeout -k 10 600 python -u -m pytest tests/test_hip_kernels.py tests/test_real_plans.py -m gpu -x -q --timeout 300 --timeout-method thread -k "topk or plan or rescan or split or stride or second_tier" > gpurun_out/enq/tests.log 2>&1
timeout -k 10 400 python tools/variant_bench.py --libs product,scanprev --users 1000000 --items 10000000 --dim 128 --k 100 --rounds 3 > gpurun_out/enq/k100_1m.json 2> gpurun_out/enq/k100_1m.err
timeout -k 10 300 python tools/variant_bench.py --libs product,scanprev --users 262144 --items 10000000 --dim 128 --k 1000 > gpurun_out/enq/k1000.json 2> gpurun_out/enq/k1000.err
