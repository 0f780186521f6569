set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/c4dbg
export TMPDIR=/tmp
XCG_STREAM_DEBUG=1 timeout -k 10 200 python3 scripts/configs_bench.py c4 --reps 2 --no-decode > gpurun_out/c4dbg/debug.log 2>&1 || exit 1
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d gpurun_out/c4dbg/trace -o run --output-format csv -- python3 scripts/configs_bench.py c4 --reps 2 --no-decode > gpurun_out/c4dbg/trace.log 2>&1 || exit 1
grep -v amdgpu.ids gpurun_out/c4dbg/debug.log | tail -25
