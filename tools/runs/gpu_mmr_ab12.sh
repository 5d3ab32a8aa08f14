set -e
mkdir -p gpurun_out/mmr12
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -k "mmr" > gpurun_out/mmr12/tests.log 2>&1
timeout -k 10 300 python tools/mmr_ab.py --libs product,sel1,mmrv10,mmrprev --users 262144 --real > gpurun_out/mmr12/ab_real.json 2> gpurun_out/mmr12/ab_real.err
timeout -k 10 300 python tools/mmr_ab.py --libs product,sel1,mmrv10,mmrprev --users 262144 > gpurun_out/mmr12/ab_rand.json 2> gpurun_out/mmr12/ab_rand.err
timeout -k 10 300 python tools/mmr_ab.py --libs product,mmrprev --users 262144 --lam 1.0 > gpurun_out/mmr12/ab_lam1.json 2> gpurun_out/mmr12/ab_lam1.err
timeout -k 10 300 python tools/mmr_ab.py --libs product,mmrprev --users 262144 --lam 0.0 > gpurun_out/mmr12/ab_lam0.json 2> gpurun_out/mmr12/ab_lam0.err
timeout -k 10 300 python tools/mmr_ab.py --libs product,mmrprev --users 1000 --real > gpurun_out/mmr12/ab_small.json 2> gpurun_out/mmr12/ab_small.err
timeout -k 10 300 python tools/mmr_diag.py --users 65536 --real > gpurun_out/mmr12/diag_real.json 2> gpurun_out/mmr12/diag_real.err
