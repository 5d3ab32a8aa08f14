#!/bin/bash
# Round-5 A/B 27: the wave sort's cross-lane exchanges by DPP quad permutes
# and ds_swizzle (product) against ds_bpermute for every exchange (sortbp):
# config 2, the headline and k = 1000 (their finalize sorts); lists
# bit-identical; then the GPU suite.
set -e
export TMPDIR=/tmp
O=gpurun_out/r05ab27
mkdir -p $O
timeout -k 10 300 python3 -u tools/variant_bench.py --libs product,sortbp --users 1000000 --items 1000000 --dim 64 --rounds 5 > $O/ab_cfg2.json 2> $O/ab_cfg2.err
timeout -k 10 400 python3 -u tools/variant_bench.py --libs product,sortbp --users 262144 --items 10000000 --dim 128 --k 1000 --rounds 3 > $O/ab_k1000.json 2> $O/ab_k1000.err
timeout -k 10 600 python3 -u -m pytest tests -m gpu -q -x --timeout 300 --timeout-method thread -p no:cacheprovider > $O/gpu_tests.log 2>&1
cd /tmp
timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/$O/trace -o t -- python3 $GRAFT_REPO_ROOT/bench.py --workload score1m --steps 2 --warmup 1 --no-cpu-baseline > $GRAFT_REPO_ROOT/$O/trace.log 2>&1
