#!/bin/bash
# Round 4: non-temporal piece loads A/B -- C4 and C2-S2 stream traces, headline timing, parity of the variant.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
XCGPU_LIB=$PWD/scripts/dev/lib_nt.so timeout -k 10 400 python -u -m pytest tests/test_gpu_encode.py tests/test_gpu_stream.py tests/test_gpu_configs.py -x -q --timeout 200 --timeout-method thread 2>&1 | tail -1
for cfg in c4 c2s; do CFG=$cfg LIBS="wanproxy_amd/libxcgpu.so scripts/dev/lib_nt.so" bash scripts/dev/ab_trace.sh 2>&1 | grep "==\|encode_stream" || exit 1; done
REPS=2 LIBS="wanproxy_amd/libxcgpu.so scripts/dev/lib_nt.so" bash scripts/dev/ab_time.sh
