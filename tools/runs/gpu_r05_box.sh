#!/bin/bash
# Round-5: the final build's headline and config-2 lines on one more box
# (box-to-box spread of the same binary). Output dir from $1.
set -e
export TMPDIR=/tmp
O=gpurun_out/$1
mkdir -p $O
timeout -k 10 300 python3 bench.py --no-cpu-baseline > $O/bench.jsonl 2> $O/bench.err
timeout -k 10 300 python3 bench.py --workload score1m --steps 3 --warmup 1 --no-cpu-baseline > $O/score1m.jsonl 2> $O/score1m.err
