#!/bin/bash
# Round 4: streaming piece loads for independent chunks -- the whole GPU suite, smoke, headline timing A/B.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/pytest_nt.log 2>&1 || { echo "pytest failed"; tail -30 gpurun_out/pytest_nt.log; exit 1; }
tail -1 gpurun_out/pytest_nt.log
timeout -k 10 300 python -c 'import __graft_entry__ as g; g.smoke()' 2>&1 | grep -v amdgpu.ids | tail -1
REPS=3 LIBS="wanproxy_amd/libxcgpu.so scripts/dev/libxcgpu_prev.so" bash scripts/dev/ab_time.sh
