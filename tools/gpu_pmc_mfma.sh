#!/bin/bash
# MFMA utilisation evidence for the score scans (north_star: "rocprof showing
# ... MFMA utilisation on the score GEMM"): per workload one kernel-trace
# --stats pass (kernel durations, for the effective clock) and ONE counter
# pass with SQ_VALU_MFMA_BUSY_CYCLES, SQ_BUSY_CYCLES and GRBM_GUI_ACTIVE
# (2 SQ + 1 GRBM counters: within one pass's slots), reduced by
# tools/pmc_mfma.py to profiles/pmc_mfma_<workload>.json (bench.py reads it
# into roofline.mfma_counters).
#   usage: bash tools/gpu_pmc_mfma.sh [catalog] [score1m]
set -e
mkdir -p gpurun_out/pmcm
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
WL=${@:-catalog score1m}
for w in $WL; do
  case $w in
    catalog) args="--steps 1 --warmup 0"; cfg=U1000000_I10000000_d128_k100_G1; flops=2.56e15; lim=240 ;;
    score1m) args="--workload score1m --steps 1 --warmup 0"; cfg=U1000000_I1000000_d64_k100_G1; flops=1.28e14; lim=240 ;;
    *) echo "unknown workload $w"; exit 1 ;;
  esac
  cd /tmp
  timeout -k 10 $lim rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/pmcm/$w/trace -o trace -- python3 $R/bench.py $args --no-cpu-baseline > $R/gpurun_out/pmcm/$w.trace.log 2>&1
  timeout -s KILL $lim rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE --output-format csv -d $R/gpurun_out/pmcm/$w/mfma -o mfma -- python3 $R/bench.py $args --no-cpu-baseline > $R/gpurun_out/pmcm/$w.mfma.log 2>&1
  cd $R
  kms=$(python3 - "$R/gpurun_out/pmcm/$w/trace/trace_kernel_stats.csv" <<'PY'
import csv, sys
tot = 0.0
for r in csv.DictReader(open(sys.argv[1])):
    if "score_scan_kernel" in r["Name"]:  # every scan dispatch of the one call
        tot += float(r["TotalDurationNs"]) / 1e6
print(tot)
PY
)
  python3 tools/pmc_mfma.py gpurun_out/pmcm/$w/mfma/mfma_counter_collection.csv --workload $w --reps 1 --config $cfg --flops $flops --kernel-ms $kms --logs gpurun_out/pmcm/$w.mfma.log gpurun_out/pmcm/$w.trace.log --out gpurun_out/pmcm/pmc_mfma_$w.json > gpurun_out/pmcm/$w.summary.txt
done
