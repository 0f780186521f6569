"""Per-chunk phase times of the C2 independent (headline) encode (diagnostics,
GPU box; XCG_PHASES build via XCGPU_LIB)."""
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
for _ in range(3):
    ctx.encode_batch_device(d_in, d_off, d_len, N, CH, d_out, d_oo, d_ol, d_st)
torch.cuda.synchronize()
st = d_st.cpu().numpy().view(np.uint32).reshape(N, 4).astype(np.float64)
w3 = st[:, 3].astype(np.int64)
vec, evt, tot, pcs, nev = st[:, 0] / 100, st[:, 1] / 100, st[:, 2] / 100, w3 & 0xFFFF, w3 >> 16
rest = tot - vec - evt
slot1 = os.environ.get('PH_SLOT1', 'exact events')   # what the build's XCG_PHASES_SLOT1 put in word 1
if slot1 == 'exact events':
    print(f'independent: per chunk (us, median) total {np.median(tot):.0f} vector {np.median(vec):.0f} exact events '
          f'{np.median(evt):.0f} ({np.median(nev):.0f} events, {np.median(evt / np.maximum(nev, 1)):.1f} us each) '
          f'rest {np.median(rest):.0f}; pieces {np.median(pcs):.0f}')
else:
    print(f'independent: per chunk (us, median) total {np.median(tot):.1f} vector {np.median(vec):.1f} '
          f'{slot1} {np.median(evt):.1f}; pieces {np.median(pcs):.0f}')
