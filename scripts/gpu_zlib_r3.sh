#!/bin/bash
# GPU box: zlib-stage tests, level-1 and level-6 throughput, per-call drop-in figures.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_zlib.py -x -v --timeout 150 --timeout-method thread > gpurun_out/pytest_zlib.log 2>&1 || { tail -30 gpurun_out/pytest_zlib.log; exit 1; }
tail -3 gpurun_out/pytest_zlib.log
timeout -k 10 240 python -u scripts/zlib_bench.py --kind text --level 1 --streams 2048 --steps 3 --check 0.25 > gpurun_out/zb_text_l1.json 2> gpurun_out/zb_text_l1.err || { tail -20 gpurun_out/zb_text_l1.err; exit 1; }
cat gpurun_out/zb_text_l1.json
timeout -k 10 240 python -u scripts/zlib_bench.py --kind xcodec --streams 2048 --steps 3 --check 0.25 > gpurun_out/zb_xcodec.json 2> gpurun_out/zb_xcodec.err || { tail -20 gpurun_out/zb_xcodec.err; exit 1; }
cat gpurun_out/zb_xcodec.json
timeout -k 10 240 python -u scripts/zlib_bench.py --kind text --per-call > gpurun_out/zb_percall_text.json 2> gpurun_out/zb_percall.err || { tail -20 gpurun_out/zb_percall.err; exit 1; }
cat gpurun_out/zb_percall_text.json
timeout -k 10 240 python -u scripts/zlib_bench.py --kind xcodec --per-call > gpurun_out/zb_percall_xcodec.json 2>> gpurun_out/zb_percall.err || { tail -20 gpurun_out/zb_percall.err; exit 1; }
cat gpurun_out/zb_percall_xcodec.json
