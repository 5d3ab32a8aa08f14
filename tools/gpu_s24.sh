#!/bin/bash
set -e
mkdir -p gpurun_out
timeout -k 10 200 python -u tools/ild_ab.py --libs product,ildA > gpurun_out/s24_ild_k100.json 2> gpurun_out/s24.err
timeout -k 10 200 python -u tools/ild_ab.py --libs product,ildA --k 10 > gpurun_out/s24_ild_k10.json 2>> gpurun_out/s24.err
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q -k "ild" --timeout 120 --timeout-method thread > gpurun_out/s24_tests.log 2>&1
