#!/bin/bash
# Round-4 A/B 6: the next MFMA pass's first two A fragments read right after
# the current pass's last MFMA (DR_XPF=1, libdivrec_hip_xpf.so), so their LDS
# latency passes under the epilogue, against the product. One process per
# shape, outputs bit-identical. noieee: the bf16 scan compiled without IEEE
# mode (-fno-honor-nans -mno-amdgpu-ieee: no canonicalising v_max_f32 before
# the hot test's max3 chain).
set -e
export TMPDIR=/tmp
O=gpurun_out/ab6
mkdir -p $O
timeout -k 10 400 python3 -u tools/variant_bench.py --libs product,xpf,noieee --users 1000000 --items 10000000 --dim 128 --rounds 2 > $O/ab_10m.json 2> $O/ab_10m.err
timeout -k 10 300 python3 -u tools/variant_bench.py --libs product,xpf,noieee --users 1000000 --items 1000000 --dim 64 --rounds 3 > $O/ab_cfg2.json 2> $O/ab_cfg2.err
timeout -k 10 300 python3 -u tools/variant_bench.py --libs product,xpf,noieee --users 262144 --items 10000000 --dim 128 --k 1000 --rounds 2 > $O/ab_k1000.json 2> $O/ab_k1000.err
