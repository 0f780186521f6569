"""Per-chunk parse time of a bounded-cache stream batch (diagnostics, GPU box;
XCG_TIMING build via XCGPU_LIB, see wave_timing.py).  Each chunk's stats hold
the start/end stamps of its LAST parse."""
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(__file__), '..', '..'))
import numpy as np
import torch

from wanproxy_amd import synth
from wanproxy_amd.xcgpu import XCG_SEM_STREAM, Context

CH = 131072
N = int(os.environ.get('CHUNKS', 4096))
LIMIT = int(os.environ.get('LIMIT_MIB', 128)) << 20
dev = torch.device('cuda', 0)
data = np.frombuffer(synth.stream(0xC5, 2 * N * CH, 20, 0), dtype=np.uint8)
d_in = torch.from_numpy(data.copy()).to(dev)
d_len = torch.full((N,), CH, dtype=torch.int32, device=dev)
bound = 2 * CH + 16
d_oo = torch.arange(N, dtype=torch.int64, device=dev) * bound
d_out = torch.empty(N * bound, dtype=torch.uint8, device=dev)
d_ol = torch.zeros(N, dtype=torch.int64, device=dev)
d_st = torch.zeros(4 * N, dtype=torch.int32, device=dev)
for name, kw in (('unbounded', dict(cache_segments=1 << 20)), ('bounded', dict(memory_cache_limit=LIMIT))):
    ctx = Context(0, **kw)
    for half in range(2):        # the second batch runs on a full cache
        d_off = (torch.arange(N, dtype=torch.int64, device=dev) + half * N) * CH
        ctx.encode_batch_device(d_in, d_off, d_len, N, CH, d_out, d_oo, d_ol, d_st, semantics=XCG_SEM_STREAM)
    torch.cuda.synchronize()
    st = d_st.cpu().numpy().view(np.uint32).reshape(N, 4).astype(np.int64)
    dur = (st[:, 1] - st[:, 0]) * 10.0 / 1000.0
    print(name, 'rounds', ctx.last_rounds(), 'dur us pct 0/10/50/90/99/100:',
          ' '.join(f'{v:.0f}' for v in np.percentile(dur, [0, 10, 50, 90, 99, 100])))
    top = np.argsort(-dur)[:8]
    print('  slowest chunks', [(int(i), round(float(dur[i]))) for i in top])
    ctx.close()
