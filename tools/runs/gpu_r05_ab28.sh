#!/bin/bash
# Round-5 A/B 28: device-counted finalizes (second-tier stream finalize,
# third-tier finalize) on a bounded grid whose waves stride over the list
# (product) against a wave per possible user (f3, the round-5 final build);
# config 2, the headline and d = 32; lists bit-identical; then the GPU suite
# and a kernel trace of config 2.
set -e
export TMPDIR=/tmp
O=gpurun_out/r05ab28
mkdir -p $O
timeout -k 10 300 python3 -u tools/variant_bench.py --libs product,f3 --users 1000000 --items 1000000 --dim 64 --rounds 5 > $O/ab_cfg2.json 2> $O/ab_cfg2.err
timeout -k 10 300 python3 -u tools/variant_bench.py --libs product,f3 --users 1000000 --items 1000000 --dim 32 --rounds 4 > $O/ab_d32.json 2> $O/ab_d32.err
timeout -k 10 500 python3 -u tools/variant_bench.py --libs product,f3 --users 1000000 --items 10000000 --dim 128 --rounds 2 > $O/ab_10m.json 2> $O/ab_10m.err
timeout -k 10 600 python3 -u -m pytest tests -m gpu -q -x --timeout 300 --timeout-method thread -p no:cacheprovider > $O/gpu_tests.log 2>&1
cd /tmp
timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/$O/trace -o t -- python3 $GRAFT_REPO_ROOT/bench.py --workload score1m --steps 2 --warmup 1 --no-cpu-baseline > $GRAFT_REPO_ROOT/$O/trace.log 2>&1
