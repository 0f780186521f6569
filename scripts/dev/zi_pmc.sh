#!/bin/bash
# GPU box: instruction counters of the inflate kernel (text workload, 1024 streams)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
rm -rf gpurun_out/zipmc
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_SMEM SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_INSTS_BRANCH -d gpurun_out/zipmc -o run --output-format csv -- python3 scripts/zlib_bench.py --kind text --streams 1024 --steps 2 --check 0.01 > gpurun_out/zipmc.log 2>&1 || { tail -5 gpurun_out/zipmc.log; exit 1; }
f=$(find gpurun_out/zipmc -name '*counter_collection.csv' | head -1)
python3 - "$f" <<'PY'
import csv, sys, collections
rows = list(csv.DictReader(open(sys.argv[1])))
agg = collections.defaultdict(lambda: collections.defaultdict(float))
for r in rows:
    k = r['Kernel_Name'][:40]
    agg[k][r['Counter_Name']] += float(r['Counter_Value'])
for k, v in agg.items():
    print(k, {c: f'{x:.3g}' for c, x in v.items()})
PY
