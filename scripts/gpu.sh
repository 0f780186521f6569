#!/bin/bash
# The GPU-box lease script: one step per invocation, chained with && in the
# gpurun command, e.g.
#   gpurun -- 'bash scripts/gpu.sh tests && bash scripts/gpu.sh bench'
# Steps (each under its own time limit; output under gpurun_out/):
#   tests [pytest args]   the -m gpu tests (default: all of tests/), one process
#   smoke                 __graft_entry__.smoke()
#   bench [bench args]    bench.py -> gpurun_out/bench.json (+ .err)
#   dist N [bench args]   bench.py --gpus N --dist-backend gloo (N ranks sharing the GPU)
#   prof                  rocprofv3 trace + PMC passes of the headline (scripts/profile.sh)
#   prof-stream           the same over configs_bench.py configurations (CFGS, REPS)
# LIMIT overrides the step's time limit (seconds); LOG the log's name.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
step=$1
shift
case "$step" in
tests)
	LOG=gpurun_out/${LOG:-pytest_gpu.log}
	timeout -k 10 ${LIMIT:-900} python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu \
		"${@:-tests}" > $LOG 2>&1
	rc=$?
	echo "pytest rc=$rc" >> $LOG
	tail -3 $LOG
	exit $rc ;;
smoke)
	timeout -k 10 ${LIMIT:-300} python -c 'import __graft_entry__ as g; g.smoke()' 2>&1 | grep -v amdgpu.ids | tail -2 ;;
bench)
	OUT=gpurun_out/${LOG:-bench}
	timeout -k 10 ${LIMIT:-600} python -u bench.py "$@" > $OUT.json 2> $OUT.err
	rc=$?
	[ $rc -ne 0 ] && tail -20 $OUT.err
	python3 -c "import json,sys; d=json.load(open('$OUT.json')); print(json.dumps({k: d.get(k) for k in ('value','n_gpus','ms_per_step','summary')})[:3000])" || exit 1
	exit $rc ;;
dist)
	N=$1
	shift
	OUT=gpurun_out/${LOG:-bench_dist$N}
	timeout -k 10 ${LIMIT:-900} python -u bench.py --gpus $N --dist-backend gloo "$@" > $OUT.json 2> $OUT.err
	rc=$?
	[ $rc -ne 0 ] && tail -20 $OUT.err
	head -c 1500 $OUT.json
	exit $rc ;;
prof)
	bash scripts/profile.sh ;;
prof-stream)
	bash scripts/profile_stream.sh ;;
*)
	echo "usage: scripts/gpu.sh tests|smoke|bench|dist N|prof|prof-stream [args]" >&2
	exit 2 ;;
esac
