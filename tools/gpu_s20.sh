#!/bin/bash
set -e
mkdir -p gpurun_out
timeout -k 10 200 python -u tools/ild_ab.py --libs product,ild1 > gpurun_out/s20_ild_ab.json 2> gpurun_out/s20.err
timeout -k 10 200 python -u tools/ild_ab.py --libs product,ild1 --k 10 > gpurun_out/s20_ild_ab_k10.json 2>> gpurun_out/s20.err
