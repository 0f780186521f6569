#!/bin/bash
# Headline-kernel PMC counters under two builds (diagnostics): SQ issue / wait split, instruction mix, clock.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
mkdir -p gpurun_out/pmc
for L in ${LIBS:-scripts/dev/libxcgpu_prev.so wanproxy_amd/libxcgpu.so}; do
  O=gpurun_out/pmc/$(basename $L); rm -rf $O; mkdir -p $O
  XCGPU_LIB=$PWD/$L timeout -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS GRBM_GUI_ACTIVE -d $O -o run --output-format csv -- python3 bench.py --no-extras --no-configs --no-zlib --no-cpu-baseline --steps 5 --warmup 1 > $O/log.txt 2>&1 || { echo "pmc failed $L"; tail -5 $O/log.txt; exit 1; }
  f=$(find $O -name 'run_counter_collection.csv' | head -1)
  python3 - "$f" "$L" <<'PY'
import csv, sys, collections
acc = collections.defaultdict(list)
for r in csv.DictReader(open(sys.argv[1])):
    if 'encode_independent' not in r['Kernel_Name']:
        continue
    acc[(r['Dispatch_Id'], r['Counter_Name'])].append(float(r['Counter_Value']))
per = collections.defaultdict(list)
for (d, c), v in acc.items():
    per[c].append(sum(v))
print('==', sys.argv[2], {c: round(sum(v) / len(v) / 1e6, 3) for c, v in sorted(per.items())}, '(M, per dispatch)')
PY
done
