"""Per-wave timing of the C2 encode launch (diagnostics, GPU box).

Run with the XCG_TIMING build of the library:
    python -c "from wanproxy_amd.build import build_lib; \
        build_lib(force=True, out='wanproxy_amd/libxcgpu_timing.so', defines=['XCG_TIMING'])"
    XCGPU_LIB=wanproxy_amd/libxcgpu_timing.so python scripts/dev/wave_timing.py
Each wave stamps s_memrealtime (100 MHz) at start/end plus HW_ID / XCC_ID into
the stats words; this prints the start spread, the duration distribution and
how the slowest waves are placed.
"""
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(__file__), '..', '..'))
import numpy as np
import torch

from wanproxy_amd import synth
from wanproxy_amd.xcgpu import Context

N = int(os.environ.get('CHUNKS', 4096))
CH = 65536
dev = torch.device('cuda', 0)
data = np.frombuffer(synth.stream(0xC2, N * CH, 50, 0), dtype=np.uint8)
d_in = torch.from_numpy(data.copy()).to(dev)
# REVERSE=1: wave w parses data chunk N-1-w (separates data/address effects
# from dispatch-order effects)
REV = os.environ.get('REVERSE') == '1'
d_off = torch.arange(N, dtype=torch.int64, device=dev) * CH
if REV:
    d_off = d_off.flip(0).contiguous()
d_len = torch.full((N,), CH, dtype=torch.int32, device=dev)
bound = 2 * CH + 16
d_oo = torch.arange(N, dtype=torch.int64, device=dev) * bound
d_out = torch.empty(N * bound, dtype=torch.uint8, device=dev)
d_ol = torch.zeros(N, dtype=torch.int64, device=dev)
d_st = torch.zeros(4 * N, dtype=torch.int32, device=dev)
ctx = Context(0)
for _ in range(5):
    ctx.encode_batch_device(d_in, d_off, d_len, N, CH, d_out, d_oo, d_ol, d_st)
torch.cuda.synchronize()
ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
ev0.record()
ctx.encode_batch_device(d_in, d_off, d_len, N, CH, d_out, d_oo, d_ol, d_st)
ev1.record()
torch.cuda.synchronize()
st = d_st.cpu().numpy().view(np.uint32).reshape(N, 4).astype(np.int64)
t0 = st[:, 0].min()
start = (st[:, 0] - t0) * 10.0 / 1000.0          # us
end = (st[:, 1] - t0) * 10.0 / 1000.0
dur = end - start
hw = st[:, 2]
xcc = st[:, 3] & 0xF
cu = (hw >> 8) & 0xF
sh = (hw >> 12) & 0x1
se = (hw >> 13) & 0x7
simd = (hw >> 4) & 0x3
q = lambda a: ' '.join(f'{v:7.1f}' for v in np.percentile(a, [0, 10, 50, 90, 99, 100]))
print(f'event time {ev0.elapsed_time(ev1) * 1000:.1f} us; chunks {N}')
print('pct            0     10     50     90     99    100')
print('start  ', q(start))
print('end    ', q(end))
print('dur    ', q(dur))
slot = (xcc * 8 + se) * 64 + sh * 16 + cu
ncu = len(np.unique(slot))
print(f'distinct CUs {ncu}; waves per CU: min {np.bincount(np.unique(slot, return_inverse=True)[1]).min()} '
      f'max {np.bincount(np.unique(slot, return_inverse=True)[1]).max()}')
late = start > np.percentile(start, 50) + 20
print(f'waves starting >20us after the median start: {late.sum()}')
for x in range(8):
    m = xcc == x
    print(f'xcc {x}: waves {m.sum():5d} start max {start[m].max():7.1f} end max {end[m].max():7.1f} '
          f'dur mean {dur[m].mean():6.1f}')
o = np.argsort(-end)[:8]
print('latest-ending waves: chunk start dur xcc se cu simd')
for i in o:
    print(f'  {i:5d} {start[i]:7.1f} {dur[i]:7.1f} {xcc[i]} {se[i]} {cu[i]} {simd[i]}')
os.makedirs('gpurun_out', exist_ok=True)
np.savez('gpurun_out/wave_timing%s.npz' % ('_rev' if REV else ''), start=start, end=end, hw=hw, xcc=xcc)
