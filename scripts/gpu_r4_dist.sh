#!/bin/bash
# Round 4: rehearse bench.py's N > 1 path on one GPU (two ranks share it, gloo for the barriers / reductions).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/dist
timeout -k 10 900 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29517 bench.py --gpus 2 --dist-backend gloo --steps 5 --warmup 2 > gpurun_out/dist/bench2.json 2> gpurun_out/dist/bench2.err || { echo "dist bench failed"; tail -30 gpurun_out/dist/bench2.err; exit 1; }
python3 -c "
import json; d=json.load(open('gpurun_out/dist/bench2.json'))
print('value', d['value'], 'n_gpus', d['n_gpus'], 'ms_per_step', d['ms_per_step'])
print(json.dumps(d.get('sharded_configs'))[:1500])"
