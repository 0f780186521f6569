import sys, os
sys.path.insert(0, os.path.join(os.path.dirname(__file__), '..', '..'))
import numpy as np
from oracle.lib import Oracle
from wanproxy_amd.xcgpu import Context, XCG_SEM_STREAM
o = Oracle()
rng = np.random.default_rng(1)
A = rng.integers(0, 256, 2048, dtype=np.uint8)
B = rng.integers(0, 256, 2048, dtype=np.uint8)
C = rng.integers(0, 256, 2048, dtype=np.uint8)
cases = {
  'aligned': [np.concatenate([A, B]), np.concatenate([A, C])],
  'aligned_second': [np.concatenate([B, A]), np.concatenate([C, A, C])],
  'shifted': [np.concatenate([A, B]), np.concatenate([C[:100], A, C])],
}
ctx = Context(0, cache_segments=4096)
for name, parts in cases.items():
    d = np.concatenate(parts).tobytes()
    lens = np.array([len(p) for p in parts], np.uint32)
    offs = np.zeros(len(parts), np.uint64); offs[1:] = np.cumsum(lens)[:-1]
    exp = o.encode_batch(d, offs, lens, mode=1)
    ctx.cache_clear()
    got, st = ctx.encode_chunks(d, offs, lens, semantics=XCG_SEM_STREAM, with_stats=True)
    print(name, 'rounds', ctx.last_rounds(), 'match', got == exp, [len(g) for g in got], [len(e) for e in exp], st.tolist())
# cache persistence: chunk 1 as a second call
ctx.cache_clear()
d0 = np.concatenate([A, B]).tobytes(); d1 = np.concatenate([A, C]).tobytes()
g0 = ctx.encode_chunks(d0, np.array([0]), np.array([len(d0)]), semantics=XCG_SEM_STREAM)
print('cache size after call 1:', ctx.cache_size())
g1, st = ctx.encode_chunks(d1, np.array([0]), np.array([len(d1)]), semantics=XCG_SEM_STREAM, with_stats=True)
print('second call len', len(g1[0]), 'stats', st.tolist(), 'starts with REF', g1[0][:2] == b'\xf1\x02')
