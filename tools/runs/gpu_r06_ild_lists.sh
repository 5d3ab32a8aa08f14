#!/bin/bash
# Round 6: why bench.py's ILD line (real top-100 lists, after the scan) reads
# slower than the uniform-list A/B: the three settings side by side.
set -e
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r06il
mkdir -p $O
cd $R
timeout -k 10 300 python3 -u -m pytest tests/test_hip_kernels.py -k "ild" -x -v --timeout 200 --timeout-method thread -p no:cacheprovider > $O/tests.log 2>&1
timeout -k 10 200 python3 -u tools/ild_ab.py --variants stream --rounds 5 > $O/uniform.json 2> $O/uniform.err
timeout -k 10 300 python3 -u tools/ild_ab.py --variants stream --rounds 5 --lists topk > $O/topk.json 2> $O/topk.err
timeout -k 10 400 python3 -u tools/ild_ab.py --variants stream --rounds 4 --lists topk --after-scan > $O/topk_after_scan.json 2> $O/topk_after_scan.err
