"""Inflate kernel phase cycles (diagnostics build with -DXCG_ZI_TIMING)."""
import ctypes as C, os, sys, time
sys.path.insert(0, os.getcwd())
os.environ['XCGPU_LIB'] = os.path.join(os.getcwd(), 'wanproxy_amd', 'libxcgpu.zitime.so')
import numpy as np, torch, zlib
from tests.zlib_cases import wan_stream
from wanproxy_amd import zpipe
S = 1024
calls = [wan_stream(5000 + s, 2, 65536) for s in range(S)]
zs = []
for s in range(S):
    c = zlib.compressobj(6, zlib.DEFLATED, 15, 8)
    zs.append([c.compress(calls[s][k]) + c.flush(zlib.Z_SYNC_FLUSH) for k in range(2)])
ctx = zpipe.InflatePipes(S)
L = zpipe._lib()
L.xcg_debug_zi_times.argtypes = [C.c_void_p]
t = np.zeros(16, np.uint64)
for k in range(2):
    L.xcg_debug_zi_times(t.ctypes.data)
    t0 = time.perf_counter()
    out = ctx.consume_many([(s, zs[s][k]) for s in range(S)])
    dt = time.perf_counter() - t0
    L.xcg_debug_zi_times(t.ctypes.data)
    assert all(o == calls[s][k] for s, (o, st) in enumerate(out))
    names = ['setup', 'fastlit', 'fastmatch', 'careful', 'flush', 'stored', 'tail']
    tot = t[:7].sum()
    print(f'step {k}: wall {dt*1e3:.1f} ms; per call cycles:', {n: int(t[i]) // S for i, n in enumerate(names)}, 'share', {n: round(float(t[i]) / tot, 3) for i, n in enumerate(names)})
