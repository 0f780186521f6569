#!/bin/bash
# GPU-box: the -m gpu tests given as arguments (default: all), one pytest
# process, each test bounded; stops at the first failure.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
LOG=gpurun_out/${LOG:-pytest_gpu.log}
timeout -k 10 ${LIMIT:-900} python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu "${@:-tests}" > $LOG 2>&1
rc=$?
echo "pytest rc=$rc" >> $LOG
tail -5 $LOG
exit $rc
