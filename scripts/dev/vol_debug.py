"""Diagnostics: the reopened-volume case of tests/test_gpu_disk.py, step by
step -- live entries after the reload on both sides, then the first chunk
whose encoding differs."""
import os
import sys
import tempfile

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))), 'tests'))
import test_gpu_disk as T  # noqa: E402
from oracle.lib import MODE_STREAM, Oracle  # noqa: E402
from wanproxy_amd.xcgpu import XCG_SEM_STREAM, Context, Disk  # noqa: E402

nb = int(sys.argv[1]) if len(sys.argv) > 1 else 3
ro = Oracle(ref=True)
limit, disk = 40 * 2048, T.mpg.disk_bytes(nb)
local, peer = T._uuid(0x100 + nb), T._uuid(0x200 + nb)
d, parts = T._vol_case(0x7E1 + nb, 3)
e, eparts = T._vol_case(0x8E1 + nb, 2)
tmp = tempfile.mkdtemp()
vref, vgpu = os.path.join(tmp, 'ref.vol'), os.path.join(tmp, 'gpu.vol')
pa = ro.cache_open_pair(limit, disk, vref, local)
pb = ro.cache_pair_front(pa, peer, limit)
ro.encode_batch(e, *eparts[0], mode=MODE_STREAM, cache=pb)
for o, l in parts[:2]:
    ro.encode_batch(d, o, l, mode=MODE_STREAM, cache=pa)
print('ref before save: local', ro.pair_stats(pa, disk_live=True), 'peer', ro.pair_stats(pb, disk_live=True))
ro.disk_save(pa, vref)
pa2 = ro.cache_open_pair(limit, disk, vref, T._uuid(0x999))
pb2 = ro.cache_pair_front(pa2, peer, limit)
print('ref after reload: local', ro.pair_stats(pa2, disk_live=True), 'peer', ro.pair_stats(pb2, disk_live=True))
K = Disk(disk, path=vgpu)
ca = Context(0, memory_cache_limit=limit, disk=K, uuid=local)
cb = Context(0, memory_cache_limit=limit, disk=K, uuid=peer)
cb.encode_chunks(e, *eparts[0], semantics=XCG_SEM_STREAM)
for o, l in parts[:2]:
    ca.encode_chunks(d, o, l, semantics=XCG_SEM_STREAM)
print('gpu before save: local', ca.pair_stats(), 'peer', cb.pair_stats(), 'disk', K.stats())
K.save(vgpu)
ca.close(); cb.close(); K.close()
print('volumes equal:', open(vref, 'rb').read() == open(vgpu, 'rb').read())
K2 = Disk(disk, path=vgpu)
ca2 = Context(0, memory_cache_limit=limit, disk=K2, uuid=local)
cb2 = Context(0, memory_cache_limit=limit, disk=K2, uuid=peer)
print('gpu after reload: local', ca2.pair_stats(), 'peer', cb2.pair_stats(), 'disk', K2.stats())
import struct
vol = open(vgpu, 'rb').read()
cands = []
for b in range(nb):
    blk = vol[(18 + b) * 2048:(19 + b) * 2048]
    ctr = struct.unpack_from('<Q', blk, 0)[0]
    ents = [struct.unpack_from('<HQ', blk, 8 + 10 * j) for j in range(204)]
    print('index block', b, 'counter', ctr, 'xuid0 entries', sum(1 for x, h in ents if x == 0 and h))
    cands += [(b, j, h) for j, (x, h) in enumerate(ents) if x == 0 and h]
found = 0
for b, j, h in (cands[-30:] if len(sys.argv) > 2 else []):
    seg = ca2.cache_lookup(h)
    found += seg is not None
print('engine lookups of 30 local entries: found', found)
o, l = parts[1]
for k in range(len(o)):
    x = ro.encode_batch(d, o[k:k + 1], l[k:k + 1], mode=MODE_STREAM, cache=pa2)[0]
    y = ca2.encode_chunks(d, o[k:k + 1], l[k:k + 1], semantics=XCG_SEM_STREAM)[0]
    if x != y:
        print('chunk', k, 'differs: ref len', len(x), 'gpu len', len(y))
        print('ref stats', ro.pair_stats(pa2, disk_live=True), 'gpu stats', ca2.pair_stats())
        break
else:
    print('all chunks equal')
