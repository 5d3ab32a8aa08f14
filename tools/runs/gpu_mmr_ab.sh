# MMR: parity tests and timing of the product kernel (add variant libraries to
# --libs for an A/B) on random and on real top-1000 candidates; fp32 scoring line.
set -e
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread -k "mmr" > gpurun_out/mmr_tests.log 2>&1
timeout -k 10 300 python tools/mmr_ab.py --libs product --users 262144 > gpurun_out/mmr_ab_rand.json 2> gpurun_out/mmr_ab_rand.err
timeout -k 10 300 python tools/mmr_ab.py --libs product --users 262144 --real > gpurun_out/mmr_ab_real.json 2> gpurun_out/mmr_ab_real.err
timeout -k 10 300 python tools/mmr_diag.py --users 65536 --real > gpurun_out/mmr_diag_real.json 2> gpurun_out/mmr_diag_real.err
