#!/bin/bash
# rocprofv3 passes over the bench (GPU box).  Kernel trace + stats first, then
# one PMC pass per TCC counter group (FETCH_SIZE and WRITE_SIZE do not fit one
# pass on gfx950, MI355X_MICROARCH.md "rocprofv3 PMC slots").
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/prof
mkdir -p $OUT
ARGS="--steps ${STEPS:-20} --warmup 2 --no-cpu-baseline ${BENCH_ARGS}"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/trace -o run --output-format csv -- python3 bench.py $ARGS > $OUT/trace.log 2>&1 || exit $?
PARGS="--steps ${STEPS:-20} --warmup 2 --no-cpu-baseline --no-extras"
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE -d $OUT/fetch -o run --output-format csv -- python3 bench.py $PARGS > $OUT/fetch.log 2>&1 || exit $?
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE -d $OUT/write -o run --output-format csv -- python3 bench.py $PARGS > $OUT/write.log 2>&1 || exit $?
timeout -k 10 300 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE -d $OUT/sq -o run --output-format csv -- python3 bench.py $PARGS > $OUT/sq.log 2>&1 || exit $?
timeout -k 10 300 rocprofv3 --pmc SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VMEM SQ_INSTS_SMEM SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_LDS -d $OUT/sq2 -o run --output-format csv -- python3 bench.py $PARGS > $OUT/sq2.log 2>&1 || exit $?
find $OUT -name "*.csv" | head -50
