#!/bin/bash
# Round-5: the whole GPU suite on the current tree (after the ring changes).
set -e
export TMPDIR=/tmp
O=gpurun_out/r05tests2
mkdir -p $O
timeout -k 10 600 python3 -u -m pytest tests -m gpu -q -x --timeout 300 --timeout-method thread -p no:cacheprovider > $O/gpu_tests.log 2>&1
