#!/bin/bash
# indep_time.py under several library builds, alternating (diagnostics): LIBS, REPS.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
for i in $(seq ${REPS:-2}); do
  for L in ${LIBS}; do
    XCGPU_LIB=$PWD/$L timeout -k 10 120 python -u scripts/dev/indep_time.py 2>&1 | grep -v amdgpu.ids || exit 1
  done
done
