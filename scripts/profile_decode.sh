#!/bin/bash
# rocprofv3 over the bench's C2-S2 batch decode (scripts/decode_step.py, GPU
# box): kernel trace + stats, then FETCH_SIZE, WRITE_SIZE and L2 passes, one
# per run (MI355X_MICROARCH.md "rocprofv3 PMC slots").
# Summarise with scripts/prof_decode_summary.py gpurun_out/profd OUT.json.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/profd
rm -rf $OUT; mkdir -p $OUT
CMD="python3 scripts/decode_step.py --calls ${CALLS:-5}"
timeout -k 10 240 rocprofv3 --kernel-trace --stats -d $OUT/trace -o run --output-format csv -- $CMD > $OUT/trace.log 2>&1 || exit $?
timeout -s KILL 240 rocprofv3 --pmc FETCH_SIZE -d $OUT/fetch -o run --output-format csv -- $CMD > $OUT/fetch.log 2>&1 || exit $?
timeout -s KILL 240 rocprofv3 --pmc WRITE_SIZE -d $OUT/write -o run --output-format csv -- $CMD > $OUT/write.log 2>&1 || exit $?
timeout -s KILL 240 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum TCC_READ_sum TCC_EA0_RDREQ_sum -d $OUT/l2 -o run --output-format csv -- $CMD > $OUT/l2.log 2>&1 || exit $?
echo decode profiled
