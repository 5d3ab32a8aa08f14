#!/bin/bash
# Round-5: kernel times of the sort kernels, product (DPP/swizzle exchanges)
# against sortbp (ds_bpermute), config 2 through tools/variant_bench.py.
set -e
export TMPDIR=/tmp
O=gpurun_out/r05prof27
R=$GRAFT_REPO_ROOT
mkdir -p $O
cd /tmp
for v in product sortbp; do
  timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $R/$O/$v -o t -- python3 $R/tools/variant_bench.py --libs $v --users 1000000 --items 1000000 --dim 64 --rounds 2 > $R/$O/$v.log 2>&1
done
