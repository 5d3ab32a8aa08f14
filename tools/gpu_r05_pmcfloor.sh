#!/bin/bash
# Round-5: HBM traffic of the product scan against the seeded scan from exact
# thresholds and from +inf, k = 1000 and k = 100 at 1M x 10M, d = 128
# (FETCH_SIZE and WRITE_SIZE in separate passes; tools/pmc_floor.py).
set -e
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r05pmcfloor
mkdir -p $O
cd /tmp
for k in 1000 100; do
  for c in FETCH_SIZE WRITE_SIZE; do
    timeout -s KILL 240 rocprofv3 --pmc $c --output-format csv -d $O/k$k/$c -o p -- python3 $R/tools/pmc_floor.py --k $k > $O/k$k.$c.log 2>&1
  done
done
cd $R
for k in 1000 100; do
  for c in FETCH_SIZE WRITE_SIZE; do
    python3 tools/pmc_floor.py --reduce $O/k$k/$c/p_counter_collection.csv $c > $O/k$k.$c.json
  done
done
