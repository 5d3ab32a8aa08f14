#!/bin/bash
# Round 5 (final build): where the score scans' wave cycles go: one rocprofv3 pass of 8 SQ counters
# (the SQ block's 8 slots) per workload, config 2 and the headline, reduced by
# tools/sq_breakdown.py. Each pass under its own kill timeout.
set -e
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r05sq
mkdir -p $O
CTR="SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_VALU_MFMA_BUSY_CYCLES"
cd /tmp
timeout -s KILL 120 rocprofv3 --pmc $CTR --output-format csv -d $O/score1m -o sq -- python3 $R/bench.py --workload score1m --steps 1 --warmup 0 --no-cpu-baseline > $O/score1m.log 2>&1
timeout -s KILL 180 rocprofv3 --pmc $CTR --output-format csv -d $O/catalog -o sq -- python3 $R/bench.py --steps 1 --warmup 0 --no-cpu-baseline > $O/catalog.log 2>&1
cd $R
python3 tools/sq_breakdown.py $O/score1m/sq_counter_collection.csv --out $O/sq_score1m.json > /dev/null
python3 tools/sq_breakdown.py $O/catalog/sq_counter_collection.csv --out $O/sq_catalog.json > /dev/null
