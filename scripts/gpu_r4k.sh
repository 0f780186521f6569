#!/bin/bash
# Round 4: C2-S2 A/B (LIBS) and the stream PMC summary of the current library.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_stream.py tests/test_gpu_chain.py -x -q --timeout 200 --timeout-method thread 2>&1 | tail -1
for cfg in c2s c2s; do CFG=$cfg LIBS="$LIBS" bash scripts/dev/ab_trace.sh 2>&1 | grep "==\|encode_stream" || exit 1; done
CFGS="c2s" REPS=2 bash scripts/profile_stream.sh > gpurun_out/prof_stream.log 2>&1 || { tail -20 gpurun_out/prof_stream.log; exit 1; }
python3 scripts/prof_stream_summary.py gpurun_out/profs gpurun_out/stream_summary.json c2s_round0=1 c2s_round1=1 c2s_seeded=1 > /dev/null || exit 1
python3 -c "import json; g=json.load(open('gpurun_out/stream_summary.json'))['c2s_seeded']; print('seeded hbm', g['hbm_bytes'], 'fetch', g['FETCH_SIZE_sum'], 'write', g['WRITE_SIZE_sum'], 'us', g['us_sum'])"
