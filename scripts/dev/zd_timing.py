"""Deflate trees / emit phase cycles (diagnostics build with -DXCG_ZD_TIMING):
build with wanproxy_amd.build.build_lib(out=.../libxcgpu.zdtime.so,
defines=('XCG_ZD_TIMING',)), run on the GPU."""
import ctypes as C, os, sys, time
sys.path.insert(0, os.getcwd())
os.environ['XCGPU_LIB'] = os.path.join(os.getcwd(), 'wanproxy_amd', 'libxcgpu.zdtime.so')
import numpy as np, torch
from tests.zlib_cases import wan_stream
from wanproxy_amd import zpipe
S = 2048
calls = [wan_stream(5000 + s, 2, 65536) for s in range(S)]
ctx = zpipe.DeflatePipes(6, S)
L = zpipe._lib()
L.xcg_debug_zd_times.argtypes = [C.c_void_p]
t = np.zeros(16, np.uint64)
names = {0: 'tr_hist', 1: 'tr_ltree', 2: 'tr_dtree_bl', 3: 'tr_bits', 4: 'tr_tabs', 8: 'em_head', 9: 'em_size', 10: 'em_pack'}
for k in range(2):
    L.xcg_debug_zd_times(t.ctypes.data)
    t0 = time.perf_counter()
    ctx.consume_many([(s, calls[s][k]) for s in range(S)])
    dt = time.perf_counter() - t0
    L.xcg_debug_zd_times(t.ctypes.data)
    nb, nw = max(1, int(t[15])), max(1, int(t[14]))
    print(f'step {k}: wall {dt*1e3:.1f} ms, {nb} blocks, {nw} tree waves; cycles per tree wave / emit block:',
          {n: int(t[i]) // (nw if n.startswith('tr') else nb) for i, n in names.items()})
    nc = max(1, int(t[12]))
    print(f'  scan per call: slow iterations {int(t[5]) // nc}, fast runs {int(t[6]) // nc} covering {int(t[7]) // nc} positions, cycles {int(t[11]) // nc}')
