import sys, time, os
sys.path.insert(0, os.environ.get('GRAFT_REPO_ROOT', '.'))
import numpy as np, torch
sys.argv = ['x']
import importlib.util
spec = importlib.util.spec_from_file_location('cb', 'scripts/configs_bench.py'); cb = importlib.util.module_from_spec(spec); spec.loader.exec_module(cb)
from wanproxy_amd import synth
from wanproxy_amd.xcgpu import Context
n = 131072
data = np.frombuffer(synth.stream(0xC4, n * 4096, 4, 0), np.uint8).copy()
offs, lens = synth.chunks_of(data.tobytes(), 4096)
ctx = Context(0, cache_segments=300000)
B = cb.Batches(ctx, data, offs, lens, per=16384)
B.encode_all(); got = B.outputs()
dctx = Context(0, cache_segments=300000)
for per in (16384, 65536, 131072):
    dctx.cache_clear()
    t = time.perf_counter(); dec, secs = cb.decode_device(dctx, got, per=per, chunk=4096); t = time.perf_counter() - t
    print(per, 'decode GiB/s', round(data.size / 2**30 / secs, 1), 'wall incl rehearsal+copies', round(t, 2), dec == data.tobytes())
