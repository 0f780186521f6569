#!/bin/bash
# Round 4: the whole GPU suite, then C4 / C2-S2 kernel traces and headline timing under LIBS (A/B).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/r4i
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/r4i/pytest.log 2>&1 || { echo "pytest failed"; tail -30 gpurun_out/r4i/pytest.log; exit 1; }
tail -1 gpurun_out/r4i/pytest.log
for cfg in c4 c2s; do CFG=$cfg LIBS="$LIBS" bash scripts/dev/ab_trace.sh || exit 1; done
REPS=2 LIBS="$LIBS" bash scripts/dev/ab_time.sh
