#!/bin/bash
# rocprofv3 over the stream-semantics configurations (GPU box), one
# configuration per run so every dispatch belongs to one configuration:
# kernel trace + stats, then one PMC pass per counter group (FETCH_SIZE and
# WRITE_SIZE do not share a pass on gfx950, MI355X_MICROARCH.md "rocprofv3
# PMC slots").  CFGS: configs_bench.py configurations (default c2s c4 c5 c5lru c5pair).
# Summarise with scripts/prof_stream_summary.py gpurun_out/profs OUT.json.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/profs
rm -rf $OUT; mkdir -p $OUT
for cfg in ${CFGS:-c2s c4 c5 c5lru c5pair}; do
	D=$OUT/$cfg
	CMD="python3 scripts/configs_bench.py $cfg --reps ${REPS:-1} --no-decode"
	timeout -k 10 240 rocprofv3 --kernel-trace --stats -d $D/trace -o run --output-format csv -- $CMD > $D.trace.log 2>&1 || exit $?
	timeout -k 10 240 rocprofv3 --pmc FETCH_SIZE -d $D/fetch -o run --output-format csv -- $CMD > $D.fetch.log 2>&1 || exit $?
	timeout -k 10 240 rocprofv3 --pmc WRITE_SIZE -d $D/write -o run --output-format csv -- $CMD > $D.write.log 2>&1 || exit $?
	timeout -k 10 240 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VMEM SQ_INSTS_SMEM -d $D/sq -o run --output-format csv -- $CMD > $D.sq.log 2>&1 || exit $?
	timeout -k 10 240 rocprofv3 --pmc SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_LDS GRBM_GUI_ACTIVE -d $D/sq2 -o run --output-format csv -- $CMD > $D.sq2.log 2>&1 || exit $?
	echo "$cfg profiled"
done
echo profile done
