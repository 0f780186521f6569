#!/bin/bash
# rocprofv3 over the stream-semantics configurations (GPU box): kernel trace +
# stats, then one PMC pass per counter group (FETCH_SIZE and WRITE_SIZE do not
# share a pass on gfx950, MI355X_MICROARCH.md "rocprofv3 PMC slots").
# CFGS: configs_bench.py configurations to run (default c2s c4 c5).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/profs
rm -rf $OUT; mkdir -p $OUT
CMD="python3 scripts/configs_bench.py ${CFGS:-c2s c4 c5} --reps ${REPS:-2} --no-decode"
timeout -k 10 240 rocprofv3 --kernel-trace --stats -d $OUT/trace -o run --output-format csv -- $CMD > $OUT/trace.log 2>&1 || exit $?
timeout -k 10 240 rocprofv3 --pmc FETCH_SIZE -d $OUT/fetch -o run --output-format csv -- $CMD > $OUT/fetch.log 2>&1 || exit $?
timeout -k 10 240 rocprofv3 --pmc WRITE_SIZE -d $OUT/write -o run --output-format csv -- $CMD > $OUT/write.log 2>&1 || exit $?
timeout -k 10 240 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VMEM SQ_INSTS_SMEM -d $OUT/sq -o run --output-format csv -- $CMD > $OUT/sq.log 2>&1 || exit $?
timeout -k 10 240 rocprofv3 --pmc SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_LDS GRBM_GUI_ACTIVE -d $OUT/sq2 -o run --output-format csv -- $CMD > $OUT/sq2.log 2>&1 || exit $?
echo profile done
