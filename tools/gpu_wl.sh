# Secondary bench lines given as arguments (with their CPU baselines).
set -e
mkdir -p gpurun_out
for w in "$@"; do
  timeout -k 10 300 python bench.py --workload $w > gpurun_out/wl_$w.json 2> gpurun_out/wl_$w.err
done
