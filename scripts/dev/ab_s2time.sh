#!/bin/bash
# C2-S2 stream-parse kernel time under several library builds, no parity check (diagnostics: timing
# experiments whose output is wrong): LIBS.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
for L in ${LIBS}; do
  O=gpurun_out/s2t/$(basename $L); rm -rf $O; mkdir -p $O
  XCGPU_LIB=$PWD/$L timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $O -o run --output-format csv -- python3 scripts/dev/stream_phases.py > $O/log.txt 2>&1 || { tail -5 $O/log.txt; exit 1; }
  f=$(find $O -name 'run_kernel_stats.csv' | head -1)
  python3 -c "
import csv
for r in csv.DictReader(open('$f')):
    if 'encode_stream' in r['Name']: print('%-36s %s calls avg %.1f us' % ('$(basename $L)', r['Calls'], float(r['AverageNs'])/1e3))
"
done
