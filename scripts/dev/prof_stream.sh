#!/bin/bash
# Per-dispatch kernel times + SQ counters of the stream encoder on C2-S2 (diagnostics).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
O=gpurun_out/ps; rm -rf $O; mkdir -p $O
CMD="python3 scripts/configs_bench.py ${CFG:-c2s} --reps 2"
timeout -k 10 200 rocprofv3 --kernel-trace -d $O/t -o run --output-format csv -- $CMD > $O/t.log 2>&1 || exit 1
timeout -k 10 200 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY -d $O/p1 -o run --output-format csv -- $CMD > $O/p1.log 2>&1 || exit 1
timeout -k 10 200 rocprofv3 --pmc SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_SCA SQ_WAIT_ANY SQ_INSTS_SMEM SQ_ACTIVE_INST_ANY -d $O/p2 -o run --output-format csv -- $CMD > $O/p2.log 2>&1 || exit 1
python3 - <<'PY'
import csv, glob, collections
O='gpurun_out/ps'
tr = list(csv.DictReader(open(glob.glob(O+'/t/**/run_kernel_trace.csv', recursive=True)[0])))
for r in tr:
    n = r['Kernel_Name']
    if 'encode_stream' in n or 'commit' in n or 'build_batch' in n:
        print(f"{n[:40]:40s} {(int(r['End_Timestamp'])-int(r['Start_Timestamp']))/1e3:9.1f} us")
for p in ('p1','p2'):
    f = glob.glob(O+f'/{p}/**/run_counter_collection.csv', recursive=True)[0]
    agg = collections.defaultdict(dict)
    for r in csv.DictReader(open(f)):
        if 'encode_stream' in r['Kernel_Name']:
            agg[int(r['Dispatch_Id'])][r['Counter_Name']] = float(r['Counter_Value'])
    for d in sorted(agg)[:8]:
        print(d, {k: f"{v:.3g}" for k, v in agg[d].items()})
PY
