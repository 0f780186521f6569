#!/bin/bash
# C4 kernel traces of library variants (XCGPU_LIB): scripts/dev/c4var.sh v1 v2 ...
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
for v in "$@"; do
  lib=wanproxy_amd/libxcgpu.$v.so
  [ "$v" = base ] && lib=wanproxy_amd/libxcgpu.so
  mkdir -p gpurun_out/c4var/$v
  XCGPU_LIB=$PWD/$lib timeout -k 10 120 rocprofv3 --kernel-trace -d gpurun_out/c4var/$v -o run --output-format csv -- python3 scripts/configs_bench.py c4 --reps 2 --no-decode > gpurun_out/c4var/$v.log 2>&1 || exit 1
  echo "$v: $(python3 scripts/dev/trace_tail.py gpurun_out/c4var/$v/run_kernel_trace.csv cache_wipe 34 | grep -E 'screen_kernel|stream_kernel|finish' | awk '{printf "%s ", $2}')"
done
