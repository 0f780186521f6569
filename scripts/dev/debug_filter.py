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
    h = o.hash(w.tobytes()); lo = h & M; k = (-lo) & M; fp = k | 1
    fb = k & ((1 << 19) - 1)
    def mix32(a, b):
        x = ((a * 0x9E3779B1) & M) ^ (((b + 0x7F4A7C15) & M) * 0x85EBCA77 & M)
        x ^= x >> 15; x = (x * 0x2C1B3C6D) & M; x ^= x >> 13; return x
    b = mix32(k, 0x5BD1E995) & int(fm[0])
    print(name, hex(h), 'filt bit', fb, bool((filt[fb >> 5] >> (fb & 31)) & 1), 'bucket', b, [hex(v) for v in ftab[4*b:4*b+4]], 'fp', hex(fp))
    print('  nonzero filt words', np.nonzero(filt)[0][:8], 'nonzero ftab idx', np.nonzero(ftab)[0][:8])
