"""Kernel time of the C2 independent (headline) encode under XCGPU_LIB, no
parity check (diagnostics: timing-experiment builds whose output is wrong)."""
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(__file__), '..', '..'))
import numpy as np
import torch

from wanproxy_amd import synth
from wanproxy_amd.xcgpu import Context

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
ctx = Context(0)
s = torch.cuda.current_stream(dev)
for _ in range(3):
    ctx.encode_batch_device(d_in, d_off, d_len, N, CH, d_out, d_oo, d_ol, d_st, stream=s)
torch.cuda.synchronize()
best = []
for rep in range(3):
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record(s)
    for _ in range(20):
        ctx.encode_batch_device(d_in, d_off, d_len, N, CH, d_out, d_oo, d_ol, d_st, stream=s)
    e1.record(s)
    torch.cuda.synchronize()
    best.append(e0.elapsed_time(e1) / 20 * 1e3)
print('%-36s per launch %6.1f us (reps %s)' % (os.path.basename(os.environ.get('XCGPU_LIB', 'libxcgpu.so')), min(best),
                                             ' '.join('%.1f' % b for b in best)))
