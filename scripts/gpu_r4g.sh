#!/bin/bash
# Round 4: encoder parity, then headline timing A/B (LIBS).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/r4g
timeout -k 10 400 python -u -m pytest tests/test_gpu_encode.py tests/test_gpu_fullsize.py -x -q --timeout 200 --timeout-method thread > gpurun_out/r4g/pytest.log 2>&1 || { echo "pytest failed"; tail -30 gpurun_out/r4g/pytest.log; exit 1; }
tail -1 gpurun_out/r4g/pytest.log
bash scripts/dev/ab_time.sh
