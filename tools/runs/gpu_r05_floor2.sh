#!/bin/bash
# Round-5: survivor-path floors of the final build (product / exact seeded
# thresholds / +inf thresholds) at config 2 and at the headline shape.
set -e
export TMPDIR=/tmp
O=gpurun_out/r05floor2
mkdir -p $O
timeout -k 10 300 python3 -u tools/scan_floor.py --users 1000000 --items 1000000 --dim 64 > $O/floor_cfg2.json 2> $O/floor_cfg2.err
timeout -k 10 500 python3 -u tools/scan_floor.py --users 1000000 --items 10000000 --dim 128 > $O/floor_10m.json 2> $O/floor_10m.err
