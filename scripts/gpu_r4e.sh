#!/bin/bash
# Round 4: headline kernel A/B (direct-mapped NX2 keys + SGPR any-mask) -- parity first, then
# alternating bench lines of the previous and the new library on the same box, then a rocprof trace.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/r4e
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_encode.py tests/test_gpu_fullsize.py -x -q --timeout 200 --timeout-method thread > gpurun_out/r4e/pytest.log 2>&1 || { echo "pytest failed"; tail -30 gpurun_out/r4e/pytest.log; exit 1; }
tail -2 gpurun_out/r4e/pytest.log
for i in 1 2; do
  for L in scripts/dev/libxcgpu_prev.so wanproxy_amd/libxcgpu.so; do
    XCGPU_LIB=$PWD/$L timeout -k 10 200 python -u bench.py --no-extras --no-configs --no-zlib --no-cpu-baseline > gpurun_out/r4e/b_$(basename $L)_$i.json 2> gpurun_out/r4e/b_err.txt || { echo "bench failed"; tail -20 gpurun_out/r4e/b_err.txt; exit 1; }
    python -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[2], d['value'], d['roofline']['kernel_ms'])" gpurun_out/r4e/b_$(basename $L)_$i.json $L
  done
done
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d gpurun_out/r4e/prof -o run --output-format csv -- python3 bench.py --no-extras --no-configs --no-zlib --no-cpu-baseline > gpurun_out/r4e/prof.log 2>&1 || { echo "rocprof failed"; tail -20 gpurun_out/r4e/prof.log; exit 1; }
f=$(find gpurun_out/r4e/prof -name 'run_kernel_stats.csv' | head -1)
head -4 "$f" | cut -c1-160
