#!/bin/bash
# Round 5: the headline bench line (cold + hot MFMA probes) and config 2's.
set -e
export TMPDIR=/tmp
O=gpurun_out/r05bench
mkdir -p $O
timeout -k 10 400 python3 -u bench.py > $O/bench.jsonl 2> $O/bench.err
timeout -k 10 300 python3 -u bench.py --workload score1m --steps 3 --warmup 1 >> $O/workloads.jsonl 2>> $O/workloads.err
