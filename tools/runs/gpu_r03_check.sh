# Final-tree check: every GPU test, smoke and one headline bench line.
set -e
mkdir -p gpurun_out/r03c
timeout -k 10 600 python3 -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread > gpurun_out/r03c/gpu_tests.log 2>&1
timeout -k 10 120 python3 -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r03c/smoke.log 2>&1
timeout -k 10 300 python3 bench.py > gpurun_out/r03c/bench.jsonl 2> gpurun_out/r03c/bench.err
timeout -k 10 300 python3 bench.py --workload mmr --steps 3 --warmup 1 > gpurun_out/r03c/mmr.jsonl 2> gpurun_out/r03c/mmr.err
