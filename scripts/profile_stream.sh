#!/bin/bash
# rocprofv3 over the stream-semantics configurations (GPU box), one
# configuration per run so every dispatch belongs to one configuration:
# kernel trace + stats, then one PMC pass per counter group (FETCH_SIZE and
# WRITE_SIZE do not share a pass on gfx950, MI355X_MICROARCH.md "rocprofv3
# PMC slots").  CFGS: configs_bench.py configurations (default c2s c4 c5 c5lru c5pair).
# PASSES: which passes (default trace fetch write sq sq2; l2 = L2 hit / miss /
# read requests, MI355X_MICROARCH.md "L2 per XCD"; tcp = the L1 side).
# Summarise with scripts/prof_stream_summary.py gpurun_out/profs OUT.json.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=${PROF_OUT:-gpurun_out/profs}
rm -rf $OUT; mkdir -p $OUT
declare -A PMC=(
	[fetch]="FETCH_SIZE"
	[write]="WRITE_SIZE"
	[sq]="SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VMEM SQ_INSTS_SMEM"
	[sq2]="SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_LDS GRBM_GUI_ACTIVE"
	[l2]="TCC_HIT_sum TCC_MISS_sum TCC_READ_sum TCC_EA0_RDREQ_sum"
	[tcp]="TCP_TOTAL_CACHE_ACCESSES_sum TCP_TCC_READ_REQ_sum GRBM_GUI_ACTIVE"
)
for cfg in ${CFGS:-c2s c4 c5 c5lru c5pair}; do
	D=$OUT/$cfg
	CMD="python3 scripts/configs_bench.py $cfg --reps ${REPS:-1} --no-decode ${CFG_ARGS}"
	for pass in ${PASSES:-trace fetch write sq sq2}; do
		if [ $pass = trace ]; then
			timeout -k 10 240 rocprofv3 --kernel-trace --stats -d $D/trace -o run --output-format csv -- $CMD > $D.trace.log 2>&1 || exit $?
		else
			timeout -s KILL 240 rocprofv3 --pmc ${PMC[$pass]} -d $D/$pass -o run --output-format csv -- $CMD > $D.$pass.log 2>&1 || exit $?
		fi
	done
	echo "$cfg profiled"
done
echo profile done
