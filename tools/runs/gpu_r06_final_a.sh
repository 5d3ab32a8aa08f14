#!/bin/bash
# Round-6 final measurement, part A1 (the tree the driver will run): every GPU
# test and the smoke. Each GPU step has its own time limit; the
# first failure ends the script.
set -e
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r06fa
mkdir -p $O
cd $R
timeout -k 10 1000 python3 -u -m pytest tests -m gpu -q --timeout 600 --timeout-method thread -p no:cacheprovider > $O/gpu_tests.log 2>&1
timeout -k 10 120 python3 -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1
