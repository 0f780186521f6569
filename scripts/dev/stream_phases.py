"""Per-chunk phase times of the C2-S2 stream parse (diagnostics, GPU box;
XCG_PHASES build via XCGPU_LIB; without it: the op counts per chunk)."""
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
SEED = int(os.environ.get('SEED', '0xC2'), 0)
phases = bool(os.environ.get('XCGPU_LIB'))
dev = torch.device('cuda', 0)
DENSE = int(os.environ.get('DENSE', 0))            # synth.dense pool size instead of the C2 generator
data = np.frombuffer(synth.dense(SEED, N * CH, DENSE) if DENSE else synth.stream(SEED, N * CH, DUP, 0),
                     dtype=np.uint8)
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
    for rep in range(2):
        ctx.cache_clear()
        d_st.zero_()
        ctx.encode_batch_device(d_in, d_off, d_len, N, CH, d_out, d_oo, d_ol, d_st, semantics=XCG_SEM_STREAM)
    torch.cuda.synchronize()
    st = d_st.cpu().numpy().view(np.uint32).reshape(N, 4).astype(np.float64)
    if not phases:
        print(f'seed {seed} rounds {ctx.last_rounds()}: per chunk (median / mean) extracts {np.median(st[:, 0]):.0f}/'
              f'{st[:, 0].mean():.1f} refs {np.median(st[:, 1]):.0f}/{st[:, 1].mean():.1f} collisions '
              f'{st[:, 2].mean():.2f} pieces {np.median(st[:, 3]):.0f}/{st[:, 3].mean():.1f}')
    else:
        w3 = st[:, 3].astype(np.int64)
        vec, evt, tot, pcs, nev = st[:, 0] / 100, st[:, 1] / 100, st[:, 2] / 100, w3 & 0xFFFF, w3 >> 16
        rest = tot - vec - evt
        slot1 = 'setup' if os.environ.get('SLOT1') else 'exact events'
        print(f'seed {seed} rounds {ctx.last_rounds()}: per chunk (us, median) total {np.median(tot):.0f} '
              f'vector {np.median(vec):.0f} {slot1} {np.median(evt):.0f} ({np.median(nev):.0f} events, '
              f'{np.median(evt / np.maximum(nev, 1)):.1f} us each) rest {np.median(rest):.0f}; pieces {np.median(pcs):.0f} '
              f'(mean {pcs.mean():.1f}, events mean {nev.mean():.1f})')
        top = np.argsort(-tot)[:6]
        print('  slowest chunks (us total / vector / events / pieces / events n):',
              [(int(c), round(tot[c]), round(vec[c]), round(evt[c]), int(pcs[c]), int(nev[c])) for c in top],
              'p99 %.0f max %.0f' % (np.percentile(tot, 99), tot.max()))
    ctx.close()
