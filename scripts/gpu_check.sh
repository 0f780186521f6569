#!/bin/bash
# GPU-box check: parity tests, then a short bench.  Each GPU step has its own
# time limit; the script stops at the first failure.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 600 python -m pytest tests -x -q -m gpu > gpurun_out/pytest_gpu.log 2>&1
rc=$?
echo "pytest rc=$rc" >> gpurun_out/pytest_gpu.log
[ $rc -ne 0 ] && exit $rc
timeout -k 10 400 python bench.py --steps ${STEPS:-10} --warmup 2 ${BENCH_ARGS} > gpurun_out/bench.log 2>&1
rc=$?
echo "bench rc=$rc" >> gpurun_out/bench.log
exit $rc
