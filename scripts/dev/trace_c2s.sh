#!/bin/bash
# Kernel trace of the C2-S2 step (configs_bench c2s: cache clear + stream encode), GPU box.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
rm -rf gpurun_out/c2s_trace; mkdir -p gpurun_out
timeout -k 10 240 rocprofv3 --kernel-trace --memory-copy-trace --stats -d gpurun_out/c2s_trace -o run --output-format csv -- python3 scripts/configs_bench.py c2s --reps 4 --no-decode > gpurun_out/c2s_trace.log 2>&1
