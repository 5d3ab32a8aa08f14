#!/bin/bash
# Round 5: where config 2's scan time goes on the current kernels: the
# product call, the seeded scan from each user's TRUE k-th score (~k
# survivors), the seeded scan with +inf thresholds (no survivor: MFMA + hot
# test + stage pipeline only), and the diag build's phase shares of the main
# scan; the same floor at the headline's 8-way shard shape for reference.
set -e
export TMPDIR=/tmp
O=gpurun_out/r05floor
mkdir -p $O
timeout -k 10 300 python3 -u tools/scan_floor.py --users 1000000 --items 1000000 --dim 64 > $O/floor_cfg2.json 2> $O/floor_cfg2.err
timeout -k 10 300 python3 -u tools/diag_topk.py --users 1000000 --items 1000000 --dim 64 --k 100 > $O/diag_cfg2.json 2> $O/diag_cfg2.err
