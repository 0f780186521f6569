#!/bin/bash
# Round 4: the whole GPU suite, then the default bench line (what the driver runs).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/pytest.log 2>&1 || { echo "pytest failed"; tail -30 gpurun_out/pytest.log; exit 1; }
tail -2 gpurun_out/pytest.log
timeout -k 10 600 python -u bench.py > gpurun_out/bench.json 2> gpurun_out/bench.err || { echo "bench failed"; tail -30 gpurun_out/bench.err; exit 1; }
python -c "import json; d=json.load(open('gpurun_out/bench.json')); print(json.dumps(d['summary']))"
