#!/bin/bash
# Headline bench lines of several library builds on one box, alternating (diagnostics): LIBS, REPS.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
mkdir -p gpurun_out/ab
for i in $(seq ${REPS:-2}); do
  for L in ${LIBS}; do
    XCGPU_LIB=$PWD/$L timeout -k 10 200 python -u bench.py --no-extras --no-configs --no-zlib --no-cpu-baseline > gpurun_out/ab/b.json 2> gpurun_out/ab/b_err.txt || { echo "bench failed $L"; tail -20 gpurun_out/ab/b_err.txt; exit 1; }
    python -c "import json,sys; d=json.load(open(sys.argv[1])); print('%-40s %9.1f GiB/s  kernel %.4f ms' % (sys.argv[2], d['value'], d['roofline']['kernel_ms']))" gpurun_out/ab/b.json $L
  done
done
