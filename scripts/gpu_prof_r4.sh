#!/bin/bash
# GPU box: rocprofv3 passes for the round-4 profiles: the headline kernel
# (scripts/profile.sh) and the stream configurations (scripts/profile_stream.sh).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
STEPS=20 bash scripts/profile.sh > gpurun_out/prof_main.log 2>&1 || { tail -20 gpurun_out/prof_main.log; exit 1; }
python3 scripts/prof_summary.py gpurun_out/prof encode_independent > gpurun_out/c2_summary.json || exit 1
cat gpurun_out/c2_summary.json
CFGS="c2s" REPS=2 bash scripts/profile_stream.sh > gpurun_out/prof_stream.log 2>&1 || { tail -20 gpurun_out/prof_stream.log; exit 1; }
python3 scripts/prof_stream_summary.py gpurun_out/profs gpurun_out/stream_summary.json c2s_round0=1 c2s_round1=1 c2s_seeded=1 > /dev/null || exit 1
cat gpurun_out/stream_summary.json | head -c 2000
