set -e
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -k "gather or range or forward or mf_ or bpr or train" > gpurun_out/q_tests.log 2>&1
timeout -k 10 300 python bench.py --workload gather > gpurun_out/q_gather.json 2> gpurun_out/q_gather.err
