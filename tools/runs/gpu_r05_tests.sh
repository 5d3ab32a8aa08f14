#!/bin/bash
# Round 5: the whole -m gpu suite (with the new RCCL world-1 test) and smoke,
# each under its own time limit; the first failure ends the script.
set -e
export TMPDIR=/tmp
O=gpurun_out/r05tests
mkdir -p $O
timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > $O/gpu_tests.log 2>&1
timeout -k 10 120 python3 -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1
