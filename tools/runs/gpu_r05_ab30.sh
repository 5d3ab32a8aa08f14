#!/bin/bash
# Round-5 A/B 30: small grids (fewer user blocks than CUs) split short
# catalogs down to one stage per chunk (product) against the 2^16-row minimum
# chunk (product@scan_split=1 has no split at these sizes either way);
# config 1's shape and two mid sizes; lists bit-identical; config 1's bench
# line; then the GPU suite.
set -e
export TMPDIR=/tmp
O=gpurun_out/r05ab30
mkdir -p $O
timeout -k 10 300 python3 -u tools/variant_bench.py --libs product,product@scan_split=1 --users 943 --items 1682 --dim 32 --k 10 --rounds 5 > $O/ab_ml100k.json 2> $O/ab_ml100k.err
timeout -k 10 300 python3 -u tools/variant_bench.py --libs product,product@scan_split=1 --users 1000 --items 100000 --dim 128 --k 100 --rounds 5 > $O/ab_1k_100k.json 2> $O/ab_1k_100k.err
timeout -k 10 300 python3 -u tools/variant_bench.py --libs product,product@scan_split=1 --users 40 --items 300001 --dim 32 --k 100 --rounds 5 > $O/ab_40_300k.json 2> $O/ab_40_300k.err
timeout -k 10 300 python3 bench.py --workload ml100k --steps 5 --warmup 2 --no-cpu-baseline > $O/ml100k.jsonl 2> $O/ml100k.err
timeout -k 10 600 python3 -u -m pytest tests -m gpu -q -x --timeout 300 --timeout-method thread -p no:cacheprovider > $O/gpu_tests.log 2>&1
