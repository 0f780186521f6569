"""Diagnostics: C2-S2 stream steps (bench.py's stream_semantics shape, no
parity check) for kernel-time experiments under rocprofv3 --kernel-trace."""
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(__file__), '..', '..'))
import numpy as np
import torch

from wanproxy_amd import synth
from wanproxy_amd.xcgpu import XCG_SEM_STREAM, Context

CH, N = 65536, 4096
dev = torch.device('cuda', 0)
data = np.frombuffer(synth.stream(0xC2, N * CH, 50, 0), dtype=np.uint8)
d_in = torch.from_numpy(data.copy()).to(dev)
d_len = torch.full((N,), CH, dtype=torch.int32, device=dev)
d_off = torch.arange(N, dtype=torch.int64, device=dev) * CH
bound = 2 * CH + 16
d_oo = torch.arange(N, dtype=torch.int64, device=dev) * bound
d_out = torch.empty(N * bound, dtype=torch.uint8, device=dev)
d_ol = torch.zeros(N, dtype=torch.int64, device=dev)
d_st = torch.zeros(4 * N, dtype=torch.int32, device=dev)
ctx = Context(0, cache_segments=1 << 18)
import time
for rep in range(int(os.environ.get('REPS', 6))):
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    ctx.cache_clear()
    ctx.encode_batch_device(d_in, d_off, d_len, N, CH, d_out, d_oo, d_ol, d_st, semantics=XCG_SEM_STREAM)
    torch.cuda.synchronize()
    print(f'step {rep}: {(time.perf_counter() - t0) * 1e3:.3f} ms rounds {ctx.last_rounds()}', flush=True)
torch.cuda.synchronize()
t0 = time.perf_counter()
for rep in range(5):
    ctx.cache_clear()
    ctx.encode_batch_device(d_in, d_off, d_len, N, CH, d_out, d_oo, d_ol, d_st, semantics=XCG_SEM_STREAM)
torch.cuda.synchronize()
dt = (time.perf_counter() - t0) / 5
print(f'back-to-back: {dt * 1e3:.3f} ms per step = {N * CH / 2**30 / dt:.1f} GiB/s', flush=True)
ctx.close()
