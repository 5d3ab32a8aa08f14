#!/bin/bash
# Round-4 first GPU pass: the new GPU tests first (config-5 full-size plan +
# MMR, the 8-rank product exchange at full configs[3] size, short-list MMR
# prefetch, device-batch range checks, padded-table cache), then the whole
# GPU suite and smoke, then bench.py --gpus 4 launching its own ranks (gloo,
# all on cuda:0) with the multi-rank list check. Each GPU step has its own
# time limit; the first failure ends the script.
set -e
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r04c
mkdir -p $O
cd $R
timeout -k 10 600 python3 -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu \
  tests/test_real_plans.py::test_configs3_eight_way_item_shards_full_size \
  tests/test_real_plans.py::test_config5_plan_1m_x_10m_k1000_then_mmr \
  "tests/test_hip_kernels.py::test_mmr_rerank_persistent_prefetch_short_lists" \
  tests/test_hip_kernels.py::test_padded_item_table_cached_per_version \
  "tests/test_api_gpu.py::test_pair_wise_train_loop_bad_device_batch_leaves_no_trace" > $O/new_tests.log 2>&1
timeout -k 10 900 python3 -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread > $O/gpu_tests.log 2>&1
timeout -k 10 120 python3 -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1
timeout -k 10 400 python3 bench.py --gpus 4 --backend gloo --same-device --check-users 1024 --steps 1 --warmup 0 --no-alt-grid > $O/launch4.jsonl 2> $O/launch4.err
