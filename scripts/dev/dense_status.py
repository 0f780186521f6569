"""REF-dense stream encode on an unbounded context (diagnostics): synth.dense
data (`pool` segments, `nbytes`) in 128 KiB chunks, batches of 4096 chunks on
one context; on a status error, bisect the shortest failing prefix (each on a
fresh context) and print that chunk's parse facts next to the oracle's."""
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(__file__), '..', '..'))
from oracle.lib import Oracle  # noqa: E402
from wanproxy_amd import synth  # noqa: E402
from wanproxy_amd.xcgpu import XCG_SEM_STREAM, Context, XCGError  # noqa: E402

pool = int(sys.argv[1]) if len(sys.argv) > 1 else 16
nbytes = int(sys.argv[2]) if len(sys.argv) > 2 else 1 << 30
per = int(sys.argv[3]) if len(sys.argv) > 3 else 4096
d = synth.dense(0xC5D, nbytes, pool)
offs, lens = synth.chunks_of(d, 131072)


def run(m):
    ctx = Context(0, cache_segments=1 << 20)
    try:
        for a in range(0, m, per):
            b = min(m, a + per)
            ctx.encode_chunks(d, offs[a:b], lens[a:b], semantics=XCG_SEM_STREAM)
        ctx.status()
        return True
    except XCGError as e:
        print('  prefix', m, 'error', e, flush=True)
        return False
    finally:
        ctx.close()


n = offs.size
if len(sys.argv) > 4:                              # just this prefix (e.g. under a diagnostics build)
    print('prefix', sys.argv[4], 'ok' if run(int(sys.argv[4])) else 'failed')
    sys.exit(0)
if run(n):
    print('all', n, 'chunks ok')
    sys.exit(0)
lo, hi = 0, n
while hi - lo > 1:
    mid = (lo + hi) // 2
    if run(mid):
        lo = mid
    else:
        hi = mid
print('first failing prefix', hi, '(chunk', hi - 1, ', batch position', (hi - 1) % per, ')')
o = Oracle()
c = o.cache_new()
exp = o.encode_batch(d, offs[:hi], lens[:hi], mode=1, cache=c)
e = exp[-1]
print('oracle chunk', hi - 1, 'out', len(e), 'extracts', e.count(b'\xf1\x01'), 'refs', e.count(b'\xf1\x02'))
