#!/bin/bash
# PMC passes over C4 (stream_screen_kernel and encode_stream_kernel): one pass
# per counter group, each under its own limit.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
OUT=gpurun_out/pmc_scr
rm -rf $OUT; mkdir -p $OUT
CMD="python3 scripts/configs_bench.py c4 --reps 1 --no-decode"
timeout -k 10 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_INSTS_VMEM -d $OUT/p1 -o run --output-format csv -- $CMD > $OUT/p1.log 2>&1 || exit 1
timeout -k 10 120 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS SQ_INSTS_SMEM SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS SQ_ACTIVE_INST_SCA SQ_INSTS_FLAT -d $OUT/p2 -o run --output-format csv -- $CMD > $OUT/p2.log 2>&1 || exit 1
timeout -k 10 120 rocprofv3 --pmc FETCH_SIZE -d $OUT/p3 -o run --output-format csv -- $CMD > $OUT/p3.log 2>&1 || exit 1
python3 - <<'PY'
import csv, glob, collections
agg = collections.defaultdict(lambda: collections.defaultdict(float))
for f in glob.glob('gpurun_out/pmc_scr/p*/**/*counter_collection.csv', recursive=True):
    for r in csv.DictReader(open(f)):
        k = r['Kernel_Name'][:40]
        agg[k][r['Counter_Name']] += float(r['Counter_Value'])
        agg[k]['_n_' + r['Counter_Name']] += 1
for k, d in agg.items():
    if 'screen' in k or 'encode_stream' in k:
        print(k, {c: int(v) for c, v in sorted(d.items()) if not c.startswith('_')})
PY
