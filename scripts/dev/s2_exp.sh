#!/bin/bash
# Kernel times of C2-S2 steps per XCG_EXP setting (diagnostics).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
for e in ${EXPS:-0}; do
  O=gpurun_out/s2exp/$e; rm -rf $O; mkdir -p $O
  XCG_EXP=$e timeout -k 10 120 rocprofv3 --kernel-trace --stats -d $O -o run --output-format csv -- python3 scripts/dev/s2_exp.py > $O/log.txt 2>&1 || exit 1
  f=$(find $O -name 'run_kernel_stats.csv' | head -1)
  echo "== XCG_EXP=$e $(grep 'step 5' $O/log.txt) | $(grep back-to-back $O/log.txt)"
  python3 -c "
import csv,sys
for r in csv.DictReader(open('$f')):
    n=r['Name']
    if any(k in n for k in ('build_batch','commit_kernel','seed_tiling','encode_stream','round_prep','verify','cache_wipe')):
        print('   %-40s %5s %9.1f' % (n[:40], r['Calls'], float(r['AverageNs'])/1e3))
"
done
