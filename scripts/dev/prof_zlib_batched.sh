#!/bin/bash
# rocprofv3 over the batched zlib stage (2048 streams x 64 KiB, text): kernel trace + stats, then one PMC pass
# each for FETCH_SIZE and WRITE_SIZE (one run holds 4 TCC counters) -- the workgroup inflate's time and HBM bytes.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
CMD="python3 scripts/zlib_bench.py --kind ${KIND:-text} --streams 2048 --steps 3 --check 0.02"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/zb_trace -o run --output-format csv -- $CMD \
	> gpurun_out/zb_trace.log 2>&1 || exit $?
for c in FETCH_SIZE WRITE_SIZE; do
	timeout -s KILL 300 rocprofv3 --pmc $c -d gpurun_out/zb_pmc_$c -o run --output-format csv -- $CMD \
		> gpurun_out/zb_pmc_$c.log 2>&1 || exit $?
done
find gpurun_out/zb_trace gpurun_out/zb_pmc_* -name '*.csv' | head
