set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/zi_prof -o run --output-format csv -- python3 scripts/zlib_bench.py --per-call --kind text > gpurun_out/zi_prof.log 2>&1 || exit $?
find gpurun_out/zi_prof -name '*kernel_stats.csv' | head -3
