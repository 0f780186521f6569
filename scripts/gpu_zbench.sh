#!/bin/bash
# GPU box: zlib-stage throughput (both workloads) + kernel trace of one.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 240 python -u scripts/zlib_bench.py --kind xcodec ${ZB_ARGS} > gpurun_out/zb_xcodec.json 2> gpurun_out/zb_xcodec.err || { echo "xcodec bench failed"; tail -20 gpurun_out/zb_xcodec.err; exit 1; }
cat gpurun_out/zb_xcodec.json
timeout -k 10 240 python -u scripts/zlib_bench.py --kind text ${ZB_ARGS} > gpurun_out/zb_text.json 2> gpurun_out/zb_text.err || { echo "text bench failed"; tail -20 gpurun_out/zb_text.err; exit 1; }
cat gpurun_out/zb_text.json
rm -rf gpurun_out/ztrace
timeout -k 10 240 rocprofv3 --kernel-trace --stats -d gpurun_out/ztrace -o run --output-format csv -- python3 scripts/zlib_bench.py --kind text --check 0.05 ${ZB_ARGS} > gpurun_out/ztrace.log 2>&1 || { echo "rocprof failed"; tail -5 gpurun_out/ztrace.log; exit 1; }
f=$(find gpurun_out/ztrace -name '*kernel_stats.csv' | head -1); cut -d, -f1-8 "$f" | head -14
