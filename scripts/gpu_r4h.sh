#!/bin/bash
# Round 4: stream parse phase split on C4 (4 KiB packets) and C2-S2 (diagnostics).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
for cfg in "CH=4096 CHUNKS=65536 DUP=4 SEED=0xC4" "CH=65536 CHUNKS=4096 DUP=50 SEED=0xC2"; do
  echo "== $cfg"
  env $cfg timeout -k 10 120 python -u scripts/dev/stream_phases.py 2>&1 | grep -v amdgpu.ids || exit 1
  env $cfg XCGPU_LIB=$PWD/scripts/dev/lib_ph_ev.so timeout -k 10 120 python -u scripts/dev/stream_phases.py 2>&1 | grep -v amdgpu.ids || exit 1
  env $cfg SLOT1=1 XCGPU_LIB=$PWD/scripts/dev/lib_ph_setup.so timeout -k 10 120 python -u scripts/dev/stream_phases.py 2>&1 | grep -v amdgpu.ids || exit 1
done
