#!/bin/bash
# Round 4, first GPU call: the VMM probe, the GPU suite, C5-PAIR phases.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 60 ./scripts/dev/vmm_test > gpurun_out/vmm.txt 2>&1; echo "vmm rc=$?" >> gpurun_out/vmm.txt
cat gpurun_out/vmm.txt
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/pytest.log 2>&1 || { echo "pytest failed"; tail -30 gpurun_out/pytest.log; exit 1; }
tail -2 gpurun_out/pytest.log
XCG_PAIR_DEBUG=1 timeout -k 10 300 python -u scripts/configs_bench.py c5pair --reps 1 --no-decode > gpurun_out/c5pair.json 2> gpurun_out/c5pair_dbg.err || { echo "c5pair failed"; tail -20 gpurun_out/c5pair_dbg.err; exit 1; }
cat gpurun_out/c5pair.json | head -c 1500
