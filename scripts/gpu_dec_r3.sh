#!/bin/bash
# GPU box: decoder tests + the per-call drop-in decode timing and its kernel trace.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_decode.py tests/test_gpu_dropin.py -x -q --timeout 200 --timeout-method thread > gpurun_out/dec.log 2>&1 || { tail -30 gpurun_out/dec.log; exit 1; }
tail -3 gpurun_out/dec.log
timeout -k 10 200 python3 scripts/dev/decode_call_loop.py 512 || exit 1
rm -rf gpurun_out/dcl2
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d gpurun_out/dcl2 -o run --output-format csv -- python3 scripts/dev/decode_call_loop.py 512 > gpurun_out/dcl2.log 2>&1 || exit 1
f=$(find gpurun_out/dcl2 -name "*kernel_stats.csv" | head -1); cut -d, -f1-8 "$f" | head -5
