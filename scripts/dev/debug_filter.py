import sys, os, ctypes as C
sys.path.insert(0, os.path.join(os.path.dirname(__file__), '..', '..'))
import numpy as np
from oracle.lib import Oracle
from wanproxy_amd.xcgpu import Context, XCG_SEM_STREAM, lib
o = Oracle()
rng = np.random.default_rng(1)
A = rng.integers(0, 256, 2048, dtype=np.uint8); B = rng.integers(0, 256, 2048, dtype=np.uint8)
ctx = Context(0, cache_segments=4096)
d0 = np.concatenate([A, B]).tobytes()
ctx.encode_chunks(d0, np.array([0]), np.array([len(d0)]), semantics=XCG_SEM_STREAM)
L = lib()
L.xcg_debug_cache_dump.argtypes = [C.c_void_p, C.c_void_p, C.c_void_p, C.c_uint64, C.c_void_p]
filt = np.zeros(1 << 14, np.uint32); fm = np.zeros(1, np.uint32)
ftab = np.zeros(4 * 65536, np.uint32)
rc = L.xcg_debug_cache_dump(ctx.h, filt.ctypes.data, ftab.ctypes.data, ftab.size, fm.ctypes.data)
print('rc', rc, 'fmask', fm[0], 'filt bits set', int(np.unpackbits(filt.view(np.uint8)).sum()), 'ftab nonzero', int((ftab != 0).sum()))
M=0xFFFFFFFF
for name, w in (('A', A), ('B', B)):
    h = o.hash(w.tobytes()); lo = h & M; hi = h >> 32; bh = (hi >> 4) & 0x0FFFFFFF; fp = lo | 1
    fb = (fp ^ ((bh << 3) & M) ^ (bh >> 13)) & ((1 << 19) - 1)
    b = ((fp >> 7) ^ ((bh * 0x9E37) & M) ^ ((fp << 9) & M)) & int(fm[0])
    print(name, hex(h), 'filt bit', fb, bool((filt[fb >> 5] >> (fb & 31)) & 1), 'bucket', b, [hex(v) for v in ftab[4*b:4*b+4]], 'fp', hex(fp))
    print('  nonzero filt words', np.nonzero(filt)[0][:8], 'nonzero ftab idx', np.nonzero(ftab)[0][:8])
