#!/bin/bash
# Round 4: kernel trace of C5-PAIR (2 reps) and the lapping variant's phases.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/prof_pair
mkdir -p $OUT
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/trace -o run --output-format csv -- python3 scripts/configs_bench.py c5pair --reps 2 --no-decode > $OUT/trace.log 2>&1 || { tail -20 $OUT/trace.log; exit 1; }
tail -1 $OUT/trace.log | head -c 600; echo
XCG_PAIR_DEBUG=1 timeout -k 10 300 python3 -u scripts/configs_bench.py c5pair --reps 2 --no-decode > $OUT/c5pair.json 2> $OUT/c5pair.err || { tail -20 $OUT/c5pair.err; exit 1; }
head -c 600 $OUT/c5pair.json; echo
XCG_PAIR_DEBUG=1 timeout -k 10 300 python3 -u scripts/configs_bench.py c5pair --reps 2 --no-decode --disk-laps 3 > $OUT/laps.json 2> $OUT/laps.err || { tail -20 $OUT/laps.err; exit 1; }
head -c 800 $OUT/laps.json; echo
