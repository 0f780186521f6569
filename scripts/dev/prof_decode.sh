#!/bin/bash
# Per-dispatch timeline of the decoder on a config (diagnostics).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
O=gpurun_out/pd; rm -rf $O; mkdir -p $O
timeout -k 10 200 rocprofv3 --kernel-trace -d $O/t -o run --output-format csv -- python3 scripts/configs_bench.py ${CFG:-c3} --reps 1 > $O/t.log 2>&1 || exit 1
python3 - <<'PY'
import csv, glob
tr = list(csv.DictReader(open(glob.glob('gpurun_out/pd/t/**/run_kernel_trace.csv', recursive=True)[0])))
tr.sort(key=lambda r: int(r['Start_Timestamp']))
idx = [i for i, r in enumerate(tr) if 'decode_kernel<false>' in r['Kernel_Name']]
start = idx[-2]
t0 = int(tr[start]['Start_Timestamp']); prev = t0
for r in tr[start - 8:start + 16]:
    s, e = int(r['Start_Timestamp']), int(r['End_Timestamp'])
    print(f"{(s-t0)/1e3:9.1f} {(e-s)/1e3:8.1f} gap {(s-prev)/1e3:7.1f}  {r['Kernel_Name'][:70]}")
    prev = e
PY
