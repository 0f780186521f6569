#!/bin/bash
# Round 4: headline kernel diagnostics -- per-chunk phase split (setup, prefetch wait).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/r4f
PH_SLOT1=setup XCGPU_LIB=$PWD/scripts/dev/libxcgpu_ph_setup.so timeout -k 10 200 python -u scripts/dev/indep_phases.py 2>&1 | grep -v amdgpu.ids | tee gpurun_out/r4f/phases.txt
PH_SLOT1=prefetch-wait XCGPU_LIB=$PWD/scripts/dev/libxcgpu_ph_wait.so timeout -k 10 200 python -u scripts/dev/indep_phases.py 2>&1 | grep -v amdgpu.ids | tee -a gpurun_out/r4f/phases.txt
