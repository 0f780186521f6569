#!/bin/bash
# GPU-box quick check: parity tests, a short bench, one kernel-trace pass.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests -x -q -m gpu --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1 || { echo "pytest failed"; tail -30 gpurun_out/pytest_gpu.log; exit 1; }
tail -2 gpurun_out/pytest_gpu.log
timeout -k 10 300 python bench.py --steps ${STEPS:-10} --warmup 2 ${BENCH_ARGS} > gpurun_out/bench.log 2>&1 || { echo "bench failed"; tail -30 gpurun_out/bench.log; exit 1; }
tail -1 gpurun_out/bench.log
rm -rf gpurun_out/trace
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/trace -o run --output-format csv -- python3 bench.py --steps 10 --warmup 2 --no-cpu-baseline > gpurun_out/trace.log 2>&1 || { echo "rocprof failed"; exit 1; }
cut -d, -f1-4 gpurun_out/trace/run_kernel_stats.csv | head -20
