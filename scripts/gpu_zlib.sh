#!/bin/bash
# GPU box: zlib-stage parity tests (one process, bounded time).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_zlib.py -x -v --timeout 150 --timeout-method thread ${PYTEST_ARGS} > gpurun_out/pytest_zlib.log 2>&1
rc=$?
tail -40 gpurun_out/pytest_zlib.log
exit $rc
