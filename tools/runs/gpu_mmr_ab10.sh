set -e
mkdir -p gpurun_out/mmr10
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -k "mmr" > gpurun_out/mmr10/tests.log 2>&1
timeout -k 10 300 python tools/mmr_ab.py --libs product,mmrv9,mmrprev --users 262144 --real > gpurun_out/mmr10/ab_real.json 2> gpurun_out/mmr10/ab_real.err
timeout -k 10 300 python tools/mmr_ab.py --libs product,mmrv9,mmrprev --users 262144 > gpurun_out/mmr10/ab_rand.json 2> gpurun_out/mmr10/ab_rand.err
timeout -k 10 300 python tools/mmr_ab.py --libs product,mmrprev --users 262144 --lam 1.0 > gpurun_out/mmr10/ab_lam1.json 2> gpurun_out/mmr10/ab_lam1.err
timeout -k 10 300 python tools/mmr_ab.py --libs product,mmrprev --users 262144 --lam 0.0 > gpurun_out/mmr10/ab_lam0.json 2> gpurun_out/mmr10/ab_lam0.err
timeout -k 10 300 python tools/mmr_ab.py --libs product,mmrprev --users 1000 --real > gpurun_out/mmr10/ab_small.json 2> gpurun_out/mmr10/ab_small.err
timeout -k 10 300 python tools/mmr_diag.py --users 65536 --real > gpurun_out/mmr10/diag_real.json 2> gpurun_out/mmr10/diag_real.err
timeout -k 10 300 python -u -m pytest tests/test_hip_kernels.py -m gpu -x -q --timeout 120 --timeout-method thread -k "score_topk" > gpurun_out/mmr10/tests_topk.log 2>&1
timeout -k 10 300 python tools/variant_bench.py --libs product,enqold --users 262144 --items 10000000 --dim 128 --k 100 > gpurun_out/mmr10/enq_k100.json 2> gpurun_out/mmr10/enq_k100.err
timeout -k 10 300 python tools/variant_bench.py --libs product,enqold --users 262144 --items 10000000 --dim 128 --k 1000 > gpurun_out/mmr10/enq_k1000.json 2> gpurun_out/mmr10/enq_k1000.err
