#!/bin/bash
# C4 stream-parse kernel PMC (diagnostics): SQ issue / wait split and instruction mix, then HBM reads.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
O=gpurun_out/pmc_c4; rm -rf $O; mkdir -p $O
timeout -s KILL 200 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS GRBM_GUI_ACTIVE -d $O/sq -o run --output-format csv -- python3 scripts/configs_bench.py c4 --reps 1 --no-decode > $O/sq.txt 2>&1 || { tail -5 $O/sq.txt; exit 1; }
timeout -s KILL 200 rocprofv3 --pmc FETCH_SIZE -d $O/fetch -o run --output-format csv -- python3 scripts/configs_bench.py c4 --reps 1 --no-decode > $O/fetch.txt 2>&1 || { tail -5 $O/fetch.txt; exit 1; }
python3 - <<'PY'
import csv, glob, collections
for grp in ('sq', 'fetch'):
    f = glob.glob(f'gpurun_out/pmc_c4/{grp}/**/run_counter_collection.csv', recursive=True)[0]
    acc = collections.defaultdict(float); disp = set()
    for r in csv.DictReader(open(f)):
        if 'encode_stream' not in r['Kernel_Name']:
            continue
        acc[r['Counter_Name']] += float(r['Counter_Value']); disp.add(r['Dispatch_Id'])
    n = max(1, len(disp))
    print(grp, 'dispatches', n, {k: round(v / n / 1e6, 3) for k, v in sorted(acc.items())}, '(M per dispatch)')
PY
