#!/bin/bash
# Secondary workload lines (configs 2, 3, 5 and the gather roofline) with the
# current product build.
set -e
mkdir -p gpurun_out
for w in score1m gather bpr mmr; do
  timeout -k 10 300 python bench.py --workload $w > gpurun_out/s39_$w.json 2>> gpurun_out/s39.err
done
