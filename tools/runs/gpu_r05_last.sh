#!/bin/bash
# Round-5 last check of the tree the driver will run: GPU suite, smoke, bench.
set -e
export TMPDIR=/tmp
O=gpurun_out/r05last
mkdir -p $O
timeout -k 10 600 python3 -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread -p no:cacheprovider > $O/gpu_tests.log 2>&1
timeout -k 10 120 python3 -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1
timeout -k 10 300 python3 bench.py > $O/bench.jsonl 2> $O/bench.err
