#!/bin/bash
# the headline scan's HBM FETCH / WRITE with 72-KB (product)
# and 64-KB (stage64) d = 128 stages, one PMC pass per counter per library
# (separate runs), then the in-process A/B timing of the two.
set -e
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r06sf
mkdir -p $O
VB="$R/tools/variant_bench.py --users 1000000 --items 10000000 --dim 128 --k 100"
for t in product stage64; do
  cd /tmp
  timeout -s KILL 240 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/$t/fetch -o fetch -- python3 $VB --libs $t --rounds 1 > $O/$t.fetch.log 2>&1
  timeout -s KILL 240 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/$t/write -o write -- python3 $VB --libs $t --rounds 1 > $O/$t.write.log 2>&1
done
cd $R
timeout -k 10 300 python3 -u $VB --libs product,stage64 --rounds 5 > $O/ab.json 2> $O/ab.err
python3 tools/stage_fetch.py --dir $O --ab $O/ab.json --out $O/stage_fetch.json > $O/summary.txt
