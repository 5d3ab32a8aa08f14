#!/bin/bash
# Round-5: kernel times of the dense threshold kernels (buffered merges in
# product, per-tile network in dnet) and of k = 1000's dense sample path.
set -e
export TMPDIR=/tmp
O=gpurun_out/r05prof14
R=$GRAFT_REPO_ROOT
mkdir -p $O
cd /tmp
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $R/$O/cfg2_product -o t -- python3 $R/tools/variant_bench.py --libs product --users 1000000 --items 1000000 --dim 64 --rounds 2 > $R/$O/cfg2_product.log 2>&1
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $R/$O/cfg2_dnet -o t -- python3 $R/tools/variant_bench.py --libs dnet --users 1000000 --items 1000000 --dim 64 --rounds 2 > $R/$O/cfg2_dnet.log 2>&1
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/$O/k1000_dense -o t -- python3 $R/tools/variant_bench.py --libs product@sample_dense=48 --users 1000000 --items 10000000 --dim 128 --k 1000 --rounds 1 > $R/$O/k1000_dense.log 2>&1
