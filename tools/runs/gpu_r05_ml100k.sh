#!/bin/bash
# Round-5: where config 1's evaluation step spends its time.
set -e
export TMPDIR=/tmp
O=gpurun_out/r05ml100k
mkdir -p $O
timeout -k 10 300 python3 -u tools/ml100k_profile.py > $O/profile.txt 2> $O/profile.err
