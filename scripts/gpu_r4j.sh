#!/bin/bash
# Round 4: stream-kernel changes -- the whole GPU suite, then C4 / C2-S2 / C5-LRU traces under LIBS (A/B).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/r4j
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/r4j/pytest.log 2>&1 || { echo "pytest failed"; tail -30 gpurun_out/r4j/pytest.log; exit 1; }
tail -1 gpurun_out/r4j/pytest.log
for cfg in c4 c2s c5lru; do CFG=$cfg LIBS="$LIBS" bash scripts/dev/ab_trace.sh 2>&1 | grep "==\|encode_stream" || exit 1; done
