"""The REF-dense pair decode case (tests/test_gpu_pair.py geom (3, 1, 200)):
frames from the oracle, decoded on a pair context in batches of 16; prints
the first failing batch's rc.  XCGPU_LIB picks the library variant."""
import importlib.util
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from oracle.lib import MODE_STREAM, Oracle  # noqa: E402
from wanproxy_amd import synth  # noqa: E402
from wanproxy_amd.xcgpu import Context  # noqa: E402

spec = importlib.util.spec_from_file_location('mpg', 'tests/golden/make_pair_golden.py')
mpg = importlib.util.module_from_spec(spec)
spec.loader.exec_module(mpg)
lim, nb, distinct = [int(x) for x in (sys.argv[1:4] if len(sys.argv) > 3 else (3, 1, 200))]
per = int(sys.argv[4]) if len(sys.argv) > 4 else 16
d = synth.dense(0xDE0 + distinct, 8 << 20, distinct)
offs, lens = synth.chunks_of(d, 65536)
o = Oracle()
c = o.cache_new_pair(lim * 2048, mpg.disk_bytes(nb))
exp = o.encode_batch(d, offs, lens, mode=MODE_STREAM, cache=c)
o.cache_free(c)
ctx = Context(0, memory_cache_limit=lim * 2048, disk_bytes=mpg.disk_bytes(nb))
outs = []
for a in range(0, len(exp), per):
    try:
        out, st, _, unk = ctx.decode_chunks(exp[a:a + per])
    except Exception as e:
        print('batch', a, 'error', e)
        break
    if (st != 0).any() or unk:
        print('batch', a, 'status', st, len(unk))
        break
    outs += out
print('decoded', len(outs), 'of', len(exp), 'ok' if b''.join(outs) == d[:sum(map(len, outs))] else 'MISMATCH')
