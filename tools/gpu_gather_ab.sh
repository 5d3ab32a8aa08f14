set -e
mkdir -p gpurun_out
L=$GRAFT_REPO_ROOT/diversity-recommendations_amd/divrec/_lib
timeout -k 10 300 python bench.py --workload gather --no-cpu-baseline > gpurun_out/gab_prod.json 2> gpurun_out/gab_prod.err
DIVREC_HIP_LIB=$L/libdivrec_hip_guw16.so timeout -k 10 300 python bench.py --workload gather --no-cpu-baseline > gpurun_out/gab_uw16.json 2> gpurun_out/gab_uw16.err
timeout -k 10 300 python bench.py --workload gather --no-cpu-baseline > gpurun_out/gab_prod2.json 2> gpurun_out/gab_prod2.err
