"""Which encode sets the status word, and the declared keys' LDS buckets
(diagnostics, GPU box)."""
import ctypes as C
import os
import sys
from collections import Counter
sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), '..', '..'))
sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), '..', '..', 'tests'))
from test_gpu_pipe import payload  # noqa: E402
from wanproxy_amd.xcgpu import Context, XCG_SEM_STREAM, XCGError, lib  # noqa: E402
import numpy as np  # noqa: E402

msgs = [payload(40 + i % 7, 400_000 + 9_000 * i) for i in range(9)]
ctx = Context(0, memory_cache_limit=600 * 2048)
for i, m in enumerate(msgs):
    piece = m[:512 * 1024]
    err = None
    try:
        ctx.encode_chunks(piece, np.array([0], np.uint64), np.array([len(piece)], np.uint32), semantics=XCG_SEM_STREAM)
    except XCGError as e:
        err = e
    hs = (C.c_uint64 * 600)()
    ps = (C.c_uint32 * 600)()
    cnt = C.c_uint32()
    lib().xcg_last_declarations(ctx.h, 0, hs, ps, 600, C.byref(cnt))
    keys = [((-(h & 0xFFFFFFFF)) & 0xFFFFFFFF) for h in hs[:cnt.value]]
    b = Counter((k >> 3) & 1023 for k in keys)
    dupk = Counter(keys)
    print('msg', i, 'decls', cnt.value, 'max bucket', max(b.values()) if b else 0,
          'buckets>2', sum(1 for v in b.values() if v > 2), 'dup keys', sum(1 for v in dupk.values() if v > 1),
          'dup hashes', len(hs[:cnt.value]) - len(set(hs[:cnt.value])), 'err', err)
    if err:
        break
