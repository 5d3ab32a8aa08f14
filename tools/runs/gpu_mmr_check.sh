set -e
mkdir -p gpurun_out/mmr4
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -k "mmr" > gpurun_out/mmr4/tests.log 2>&1
timeout -k 10 300 python tools/mmr_diag.py --users 65536 --real > gpurun_out/mmr4/diag_real.json 2> gpurun_out/mmr4/diag_real.err
timeout -k 10 300 python tools/mmr_ab.py --libs product,mmrlegacy --users 262144 --real > gpurun_out/mmr4/ab_real.json 2> gpurun_out/mmr4/ab_real.err
timeout -k 10 300 python tools/mmr_ab.py --libs product,mmrlegacy --users 262144 > gpurun_out/mmr4/ab_rand.json 2> gpurun_out/mmr4/ab_rand.err
