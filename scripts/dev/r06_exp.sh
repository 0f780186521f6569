#!/bin/bash
# Round-6 experiments (GPU box), one step per argument:
#   segs     C2-S2 at three cache capacities (the probe tables scale with them)
#   pairdbg  C5-PAIR with XCG_PAIR_DEBUG (per sub-batch phase ms; syncs added)
#   trace    rocprofv3 kernel trace of c5pair and c2s (CFGS overrides)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
for step in "$@"; do
	case "$step" in
	segs)
		for s in 131072 262144 524288; do
			timeout -k 10 200 python3 scripts/configs_bench.py c2s --reps 5 --no-decode --c2s-segs $s \
				> gpurun_out/segs_$s.json 2> gpurun_out/segs_$s.err || exit $?
			echo "segs $s $(head -c 400 gpurun_out/segs_$s.json)"
		done ;;
	pairdbg)
		XCG_PAIR_DEBUG=1 timeout -k 10 200 python3 scripts/configs_bench.py c5pair --reps 2 --no-decode \
			> gpurun_out/pairdbg.json 2> gpurun_out/pairdbg.err || exit $?
		grep -E '^pair' gpurun_out/pairdbg.err | tail -12 ;;
	trace)
		for cfg in ${CFGS:-c5pair c2s}; do
			timeout -k 10 240 rocprofv3 --kernel-trace --stats -d gpurun_out/tr_$cfg -o run --output-format csv -- \
				python3 scripts/configs_bench.py $cfg --reps 2 --no-decode > gpurun_out/tr_$cfg.log 2>&1 || exit $?
			echo "traced $cfg"
		done ;;
	ab)
		# A/B of the main library against wanproxy_amd/libxcgpu.$VAR.so (CFGS, two alternations)
		for rep in 1 2; do
			for lib in libxcgpu.so libxcgpu.${VAR:-nodefer}.so; do
				XCGPU_LIB=$PWD/wanproxy_amd/$lib timeout -k 10 300 python3 scripts/configs_bench.py ${CFGS:-c5lru c5pair} \
					--reps 3 --no-decode $ARGS > gpurun_out/ab_${lib}_$rep.json 2> gpurun_out/ab_${lib}_$rep.err || exit $?
				python3 -c "import json,sys; [print(sys.argv[1], json.loads(l)['config'][:18], json.loads(l)['encode_GiBps'], json.loads(l).get('rounds')) for l in open(sys.argv[2]) if l.startswith('{')]" $lib gpurun_out/ab_${lib}_$rep.json
			done
		done ;;
	big)
		timeout -k 10 300 python3 scripts/configs_bench.py c5pair --reps 3 --no-decode --batch-mib 1024 \
			> gpurun_out/big.json 2> gpurun_out/big.err || exit $?
		head -c 600 gpurun_out/big.json ;;
	pairs)
		# the pair configurations as the bench runs them (1 GiB calls; LAPS in 512 MiB; DENSE)
		timeout -k 10 300 python3 scripts/configs_bench.py c5pair --reps 3 --no-decode --batch-mib 1024 \
			> gpurun_out/pairs.json 2> gpurun_out/pairs.err || exit $?
		timeout -k 10 300 python3 scripts/configs_bench.py c5pair --reps 2 --no-decode --disk-laps 3 \
			>> gpurun_out/pairs.json 2>> gpurun_out/pairs.err || exit $?
		timeout -k 10 300 python3 scripts/configs_bench.py c5dense --reps 2 --no-decode --dense-pool 16 --lru-check 0.1 \
			>> gpurun_out/pairs.json 2>> gpurun_out/pairs.err || exit $?
		python3 -c "import json,sys; [print(json.loads(l)['config'][:60], json.loads(l)['encode_GiBps'], json.loads(l).get('rounds'), json.loads(l).get('kernel')) for l in open(sys.argv[1]) if l.startswith('{')]" gpurun_out/pairs.json ;;
	sizes)
		# call sizes: C5 in 512 vs 1024 MiB calls, C4 in 65536 vs 131072 packets
		for a in "c5 --batch-mib 512" "c5 --batch-mib 1024" "c4 --c4-batch 65536" "c4 --c4-batch 131072"; do
			timeout -k 10 300 python3 scripts/configs_bench.py $a --reps 3 --no-decode > gpurun_out/sizes.json 2> gpurun_out/sizes.err || exit $?
			python3 -c "import json,sys; [print(sys.argv[1], json.loads(l)['encode_GiBps'], json.loads(l).get('rounds')) for l in open(sys.argv[2]) if l.startswith('{')]" "$a" gpurun_out/sizes.json
		done ;;
	lfk)
		# the LDS-alone threshold (XCG_LDS_FILTER_KEYS) on the big-cache configurations
		for k in 150000 40000 0; do
			for a in "c5pair --batch-mib 1024" "c5 --batch-mib 512" "c5lru --batch-mib 1024" "c2s"; do
				XCG_LDS_FILTER_KEYS=$k timeout -k 10 300 python3 scripts/configs_bench.py $a --reps 3 --no-decode > gpurun_out/lfk.json 2> gpurun_out/lfk.err || exit $?
				python3 -c "import json,sys; [print(sys.argv[1], json.loads(l)['encode_GiBps'], json.loads(l).get('rounds'), json.loads(l).get('kernel',{}).get('stream_kernel_ms')) for l in open(sys.argv[2]) if l.startswith('{')]" "lfk=$k $a" gpurun_out/lfk.json
			done
		done ;;
	auto)
		# the automatic LDS-alone threshold against the old fixed 150000, alternating
		for rep in 1 2; do
			for k in auto 150000; do
				for a in "c4 --c4-batch 65536" "c4 --c4-batch 131072" "c5 --batch-mib 512" "c3"; do
					if [ $k = auto ]; then unset XCG_LDS_FILTER_KEYS; else export XCG_LDS_FILTER_KEYS=$k; fi
					timeout -k 10 300 python3 scripts/configs_bench.py $a --reps 3 --no-decode > gpurun_out/auto.json 2> gpurun_out/auto.err || exit $?
					python3 -c "import json,sys; [print(sys.argv[1], json.loads(l)['encode_GiBps'], json.loads(l).get('rounds')) for l in open(sys.argv[2]) if l.startswith('{')]" "$k $a" gpurun_out/auto.json
				done
			done
		done
		unset XCG_LDS_FILTER_KEYS ;;
	*) echo "unknown step $step"; exit 2 ;;
	esac
done
