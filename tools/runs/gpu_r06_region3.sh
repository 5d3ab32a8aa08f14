#!/bin/bash
# Round 6: config 2 — region split strided / contiguous against the unsplit
# plan, and first-tier ranks 8 / 7 (guess_z1 / guess_c1 knobs) on the unsplit
# plan; then the d = 128 stage-size FETCH record.
set -e
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r06reg3
mkdir -p $O
cd $R
timeout -k 10 400 python3 -u tools/variant_bench.py --libs product@scan_split=1,product,regcont,product@scan_split=1+guess_z1=1+guess_c1=3,product@scan_split=1+guess_z1=1+guess_c1=2 --users 1000000 --items 1000000 --dim 64 --k 100 --rounds 5 > $O/ab_cfg2.json 2> $O/ab_cfg2.err
bash tools/runs/gpu_r06_stagefetch.sh
