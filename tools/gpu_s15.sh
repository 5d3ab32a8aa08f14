#!/bin/bash
set -e
mkdir -p gpurun_out
timeout -k 10 300 python -u tools/mmr_ab.py --libs product,mmrA,mmrNP,mmrNPP > gpurun_out/s15_mmr_ab.json 2> gpurun_out/s15.err
timeout -k 10 300 python -u tools/mmr_ab.py --libs product,mmrA,mmrNP,mmrNPP --users 1000000 --rounds 2 > gpurun_out/s15_mmr_ab_1m.json 2>> gpurun_out/s15.err
