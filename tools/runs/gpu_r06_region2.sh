#!/bin/bash
# Round 6: region-mode tail split (config 2) and staged survivors for d = 128
# long lists (k = 1000). Tests first, then A/B against the committed build
# (r06base) and the no-long-staging variant, guess failure counts on the
# bench's tables, and the score1m line.
set -e
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r06reg2
mkdir -p $O
cd $R
timeout -k 10 900 python3 -u -m pytest tests/test_real_plans.py tests/test_hip_kernels.py -k "region or config5 or 1000 or split" -x -v --timeout 400 --timeout-method thread -p no:cacheprovider > $O/tests.log 2>&1
timeout -k 10 300 python3 -u tools/variant_bench.py --libs product,product@scan_split=1,r06base --users 1000000 --items 1000000 --dim 64 --k 100 --rounds 5 > $O/ab_cfg2.json 2> $O/ab_cfg2.err
timeout -k 10 400 python3 -u tools/variant_bench.py --libs product,nolong --users 1000000 --items 10000000 --dim 128 --k 1000 --rounds 3 > $O/ab_k1000.json 2> $O/ab_k1000.err
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
    del users, items
PY
timeout -k 10 300 python3 bench.py --workload score1m --no-cpu-baseline > $O/bench_score1m.jsonl 2> $O/bench_score1m.err
