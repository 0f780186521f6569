#!/bin/bash
# Region shape sweep of the workgroup inflate (XCG_ZI_WARM warm-up bits, XCG_ZI_THREADS per region):
# per-call text inflate via scripts/dev/zi_percall.py (mode 2 lines only).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
for th in 1024 512; do
	for w in 0 64 128 256; do
		r=$(XCG_ZI_WARM=$w XCG_ZI_THREADS=$th timeout -k 10 120 python3 scripts/dev/zi_percall.py 24 2>&1 | grep '^mode 2:' | tail -1) || exit 1
		echo "threads $th warm $w: $r"
	done
done
