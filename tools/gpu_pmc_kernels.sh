#!/bin/bash
# rocprof evidence for the HBM-bound kernels: for each bench workload, one
# kernel-trace --stats pass (per-kernel average durations) and two PMC passes
# (FETCH_SIZE, WRITE_SIZE: separate runs, MI355X_MICROARCH.md HBM section),
# reduced by tools/pmc_kernels.py to per-dispatch bytes. bench.py reads the
# resulting profiles/pmc_<workload>.json into roofline.traffic.
#   usage: bash tools/gpu_pmc_kernels.sh [workload ...]   (default: gather bpr mmr catalog;
#   also score1m fp32)
# Every GPU step has its own time limit; the first failure ends the script.
set -e
mkdir -p gpurun_out/pmck
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
WL=${@:-gather bpr mmr catalog}
for w in $WL; do
  case $w in
    gather) args="--workload gather --steps 1 --warmup 1"; cfg=gather; lim=240 ;;
    bpr) args="--workload bpr --steps 1 --warmup 1"; cfg=bpr; lim=240 ;;
    mmr) args="--workload mmr --steps 1 --warmup 0"; cfg=mmr_U1000000_I10000000_d128_C1000_k100; lim=300 ;;
    catalog) args="--steps 1 --warmup 0"; cfg=U1000000_I10000000_d128_k100_G1; lim=240 ;;
    score1m) args="--workload score1m --steps 1 --warmup 0"; cfg=U1000000_I1000000_d64_k100_G1; lim=240 ;;
    fp32) args="--workload fp32 --steps 1 --warmup 0"; cfg=fp32_U262144_I1000000_d100_k100; lim=240 ;;
    *) echo "unknown workload $w"; exit 1 ;;
  esac
  reps=$(python3 -c "import re,sys; a=sys.argv[1]; print(int(re.search(r'--steps (\d+)',a).group(1))+int(re.search(r'--warmup (\d+)',a).group(1)))" "$args")
  cd /tmp
  timeout -k 10 $lim rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/pmck/$w/trace -o trace -- python3 $R/bench.py $args --no-cpu-baseline > $R/gpurun_out/pmck/$w.trace.log 2>&1
  timeout -s KILL $lim rocprofv3 --pmc FETCH_SIZE --output-format csv -d $R/gpurun_out/pmck/$w/fetch -o fetch -- python3 $R/bench.py $args --no-cpu-baseline > $R/gpurun_out/pmck/$w.fetch.log 2>&1
  timeout -s KILL $lim rocprofv3 --pmc WRITE_SIZE --output-format csv -d $R/gpurun_out/pmck/$w/write -o write -- python3 $R/bench.py $args --no-cpu-baseline > $R/gpurun_out/pmck/$w.write.log 2>&1
  cd $R
  python3 tools/pmc_kernels.py gpurun_out/pmck/$w/fetch/fetch_counter_collection.csv gpurun_out/pmck/$w/write/write_counter_collection.csv --workload $w --reps $reps --config $cfg --logs gpurun_out/pmck/$w.fetch.log gpurun_out/pmck/$w.write.log gpurun_out/pmck/$w.trace.log --out gpurun_out/pmck/pmc_$w.json > gpurun_out/pmck/$w.summary.txt
done
