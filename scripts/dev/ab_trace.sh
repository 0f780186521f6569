#!/bin/bash
# Kernel stats of one config under two builds of the library (diagnostics): CFG, LIBS.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
for L in ${LIBS:-scripts/dev/libxcgpu_prev.so wanproxy_amd/libxcgpu.so}; do
  O=gpurun_out/abt/$(basename $L); rm -rf $O; mkdir -p $O
  XCGPU_LIB=$PWD/$L timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O -o run --output-format csv -- python3 scripts/configs_bench.py ${CFG:-c4} --reps 2 --no-decode > $O/log.txt 2>&1 || exit 1
  f=$(find $O -name 'run_kernel_stats.csv' | head -1)
  echo "== $L: $(grep -o '"encode_GiBps": [0-9.]*' $O/log.txt)"
  python3 -c "
import csv
for r in list(csv.DictReader(open('$f')))[:14]:
    print('   %-50s %6s %9.1f %9.1f' % (r['Name'][:50], r['Calls'], float(r['AverageNs'])/1e3, float(r['TotalDurationNs'])/1e6))
"
done
