# rocprofv3 kernel-trace summaries of config 2 (score1m) and config 5 (mmr pipeline)
set -e
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/prof_c25
mkdir -p $O
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/score1m -o trace -- python3 $R/bench.py --workload score1m --steps 3 --warmup 1 --no-cpu-baseline > $O/score1m.log 2>&1
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/mmr -o trace -- python3 $R/bench.py --workload mmr --steps 2 --warmup 1 --no-cpu-baseline > $O/mmr.log 2>&1
