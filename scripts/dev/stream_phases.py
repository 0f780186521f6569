"""Per-chunk phase times of the C2-S2 stream parse (diagnostics, GPU box;
XCG_PHASES build via XCGPU_LIB)."""
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(__file__), '..', '..'))
import numpy as np
import torch

from wanproxy_amd import synth
from wanproxy_amd.xcgpu import XCG_SEM_STREAM, Context, lib

CH = int(os.environ.get('CH', 65536))
N = int(os.environ.get('CHUNKS', 4096))
DUP = int(os.environ.get('DUP', 50))
dev = torch.device('cuda', 0)
data = np.frombuffer(synth.stream(0xC2, N * CH, DUP, 0), dtype=np.uint8)
d_in = torch.from_numpy(data.copy()).to(dev)
d_len = torch.full((N,), CH, dtype=torch.int32, device=dev)
d_off = torch.arange(N, dtype=torch.int64, device=dev) * CH
bound = 2 * CH + 16
d_oo = torch.arange(N, dtype=torch.int64, device=dev) * bound
d_out = torch.empty(N * bound, dtype=torch.uint8, device=dev)
d_ol = torch.zeros(N, dtype=torch.int64, device=dev)
d_st = torch.zeros(4 * N, dtype=torch.int32, device=dev)
for seed in (0, 1):
    lib().xcg_debug_set_stream_seed(seed)
    ctx = Context(0, cache_segments=1 << 18)
    ctx.encode_batch_device(d_in, d_off, d_len, N, CH, d_out, d_oo, d_ol, d_st, semantics=XCG_SEM_STREAM)
    torch.cuda.synchronize()
    st = d_st.cpu().numpy().view(np.uint32).reshape(N, 4).astype(np.float64)
    w3 = st[:, 3].astype(np.int64)
    vec, evt, tot, pcs, nev = st[:, 0] / 100, st[:, 1] / 100, st[:, 2] / 100, w3 & 0xFFFF, w3 >> 16
    rest = tot - vec - evt
    print(f'seed {seed} rounds {ctx.last_rounds()}: per chunk (us, median) total {np.median(tot):.0f} '
          f'vector {np.median(vec):.0f} exact events {np.median(evt):.0f} ({np.median(nev):.0f} events, '
          f'{np.median(evt / np.maximum(nev, 1)):.1f} us each) rest {np.median(rest):.0f}; pieces {np.median(pcs):.0f}')
    ctx.close()
