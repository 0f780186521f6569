#!/bin/bash
# Round 4: the VMM probe, the pair tests, the whole GPU suite, C5-PAIR phases.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 60 ./scripts/dev/vmm_test > gpurun_out/vmm.txt 2>&1; echo "vmm rc=$?" >> gpurun_out/vmm.txt
cat gpurun_out/vmm.txt
timeout -k 10 400 python -u -m pytest tests/test_gpu_pair.py tests/test_gpu_pair_decode.py -m gpu -x -v --timeout 200 --timeout-method thread > gpurun_out/pytest_pair.log 2>&1 || { echo "pair tests failed"; grep -E "PASS|FAIL|Error|error|assert" gpurun_out/pytest_pair.log | head -40; tail -40 gpurun_out/pytest_pair.log; exit 1; }
tail -3 gpurun_out/pytest_pair.log
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/pytest.log 2>&1 || { echo "pytest failed"; tail -40 gpurun_out/pytest.log; exit 1; }
tail -2 gpurun_out/pytest.log
XCG_PAIR_DEBUG=1 timeout -k 10 300 python -u scripts/configs_bench.py c5pair --reps 1 --no-decode > gpurun_out/c5pair.json 2> gpurun_out/c5pair_dbg.err || { echo "c5pair failed"; tail -20 gpurun_out/c5pair_dbg.err; exit 1; }
head -c 1500 gpurun_out/c5pair.json
timeout -k 10 60 ./scripts/dev/vmm_test host > gpurun_out/vmm_host.txt 2>&1; echo "vmm host rc=$?" >> gpurun_out/vmm_host.txt; cat gpurun_out/vmm_host.txt
head -c 1500 gpurun_out/c5pair.json
