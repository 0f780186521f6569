#!/bin/bash
# Sweep the LDS-filter key threshold over C2-S2 / C4 / C5 (diagnostics).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
mkdir -p gpurun_out
for k in ${KS:-100000 160000 220000 300000}; do
  XCG_LDS_FILTER_KEYS=$k timeout -k 10 300 python -u scripts/configs_bench.py ${CFGS:-c2s c4 c5} > gpurun_out/sweep_$k.log 2>&1 || exit 1
  echo "== $k"; grep -o '"config": "[^"]*".*"encode_GiBps": [0-9.]*' gpurun_out/sweep_$k.log | sed 's/, "batch_chunks": [0-9]*//'
done
