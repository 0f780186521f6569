#!/bin/bash
# Round 4, last session check: the whole GPU suite and smoke() on the committed build.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/pytest_last.log 2>&1 || { echo "pytest failed"; tail -30 gpurun_out/pytest_last.log; exit 1; }
tail -1 gpurun_out/pytest_last.log
timeout -k 10 300 python -c 'import __graft_entry__ as g; g.smoke()' 2>&1 | grep -v amdgpu.ids | tail -2
