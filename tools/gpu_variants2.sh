set -e
mkdir -p gpurun_out
export TMPDIR=/tmp
LIBS=product,m16n3,n3,nut2,base
timeout -k 10 300 python -u tools/variant_bench.py --libs $LIBS --users 131072 --items 10000000 --dim 128 --rounds 3 > gpurun_out/v2_bench128.json 2> gpurun_out/v2_bench128.err
timeout -k 10 300 python -u tools/variant_bench.py --libs $LIBS --users 262144 --items 1000000 --dim 64 --rounds 3 > gpurun_out/v2_bench64.json 2> gpurun_out/v2_bench64.err
bash tools/gpu_pmc.sh
