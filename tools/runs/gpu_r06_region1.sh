#!/bin/bash
# Round 6: region-mode tail split (config 2: 12 chunks in 85-key slices of the
# users' own buffers). Tests, A/B against the unsplit plan and the committed
# build, guess failure counts on the bench's tables, and the score1m line.
set -e
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r06reg1
mkdir -p $O
cd $R
timeout -k 10 600 python3 -u -m pytest tests/test_real_plans.py -k "region or config2 or second_tier or forced_stride" -x -v --timeout 300 --timeout-method thread -p no:cacheprovider > $O/tests.log 2>&1
timeout -k 10 300 python3 -u tools/variant_bench.py --libs product,product@scan_split=1,r06base --users 1000000 --items 1000000 --dim 64 --k 100 --rounds 5 > $O/ab_cfg2.json 2> $O/ab_cfg2.err
timeout -k 10 300 python3 -u tools/variant_bench.py --libs product,r06base --users 1000000 --items 1000000 --dim 32 --k 100 --rounds 5 > $O/ab_d32.json 2> $O/ab_d32.err
timeout -k 10 300 python3 -u tools/variant_bench.py --libs product,r06base --users 1000000 --items 10000000 --dim 128 --k 100 --rounds 3 > $O/ab_head.json 2> $O/ab_head.err
timeout -k 10 300 python3 -u - > $O/fails.txt 2>&1 <<'PY'
import sys; sys.path.insert(0, "diversity-recommendations_amd"); sys.path.insert(0, ".")
import torch
from bench import gen_table
from divrec import ops
for (U, I, d) in [(1_000_000, 1_000_000, 64), (1_000_000, 1_000_000, 32)]:
    users = gen_table(U, d, 1, "cuda"); items = gen_table(I, d, 2, "cuda")
    st = {}
    ops.score_topk(users, items, 100, stats=st)
    print((U, I, d), ops.score_topk_plan(U, I, torch.bfloat16, d, 100), st, flush=True)
PY
timeout -k 10 300 python3 bench.py --workload score1m --no-cpu-baseline > $O/bench_score1m.jsonl 2> $O/bench_score1m.err
