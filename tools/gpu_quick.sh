# Quick GPU check after a kernel change: the whole parity suite, then the
# secondary workload lines given as arguments (e.g. bpr gather).
set -e
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/q_tests.log 2>&1
for w in "$@"; do
  timeout -k 10 300 python bench.py --workload $w --no-cpu-baseline > gpurun_out/q_$w.json 2> gpurun_out/q_$w.err
done
