set -e
mkdir -p gpurun_out/diagk
timeout -k 10 200 python tools/diag_topk.py --users 262144 --items 10000000 --dim 128 --k 100 > gpurun_out/diagk/k100.json 2> gpurun_out/diagk/k100.err
timeout -k 10 200 python tools/diag_topk.py --users 262144 --items 10000000 --dim 128 --k 1000 > gpurun_out/diagk/k1000.json 2> gpurun_out/diagk/k1000.err
timeout -k 10 200 python tools/diag_topk.py --users 1000000 --items 1000000 --dim 64 --k 100 > gpurun_out/diagk/c2.json 2> gpurun_out/diagk/c2.err
