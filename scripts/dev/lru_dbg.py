"""Bounded-cache debugging on the GPU box: one golden case, pass log (XCG_LRU_DEBUG)."""
import os
import sys
sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), '..', '..'))
sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), '..', '..', 'tests'))
os.environ['XCG_LRU_DEBUG'] = '1'
from test_lru_oracle import mlg  # noqa: E402
from oracle.lib import Oracle, MODE_STREAM  # noqa: E402
from wanproxy_amd.synth import chunks_of  # noqa: E402
from wanproxy_amd.xcgpu import Context, XCG_SEM_STREAM, lib  # noqa: E402

name, chunk, limit = sys.argv[1], int(sys.argv[2]), int(sys.argv[3])
seed = int(sys.argv[4]) if len(sys.argv) > 4 else -1
lib().xcg_debug_set_stream_seed(seed)
d = mlg.inputs(name)
offs, lens = chunks_of(d, chunk)
o = Oracle()
c = o.cache_new(limit)
exp = o.encode_batch(d, offs, lens, mode=MODE_STREAM, cache=c)
ctx = Context(0, memory_cache_limit=limit)
try:
    got = ctx.encode_chunks(d, offs, lens, semantics=XCG_SEM_STREAM)
    bad = [i for i in range(len(exp)) if got[i] != exp[i]]
    print('mismatch chunks', bad[:20], 'of', len(exp), 'size', ctx.cache_size(), o.lib.xco_cache_size(c))
except Exception as e:
    print('error', e)
