import sys
sys.path.insert(0, '.')
from wanproxy_amd import synth
from wanproxy_amd.xcgpu import XCG_SEM_STREAM, Context
d = synth.stream(0x5E1, 2 << 20, 25, 0)
offs, lens = synth.chunks_of(d, 65536)
for segs in (40, 1 << 14, 1 << 16, 1 << 18, 1 << 19):
    try:
        c = Context(0, memory_cache_limit=segs * 2048, disk_bytes=(18 + 3 * 205) * 2048)
        out = c.encode_chunks(d, offs, lens, semantics=XCG_SEM_STREAM)
        print(segs, 'ok', sum(map(len, out)), flush=True)
        c.close()
    except Exception as e:
        print(segs, 'FAIL', e, flush=True)
