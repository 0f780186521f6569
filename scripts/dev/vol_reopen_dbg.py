"""Debug: reopen of a single-front volume (tests/test_gpu_disk.py
test_volume_saved_after_its_fronts_are_gone) -- first differing chunk and op."""
import os, sys, tempfile
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from oracle.lib import Oracle, MODE_STREAM
from wanproxy_amd import synth
from wanproxy_amd.xcgpu import XCG_SEM_STREAM, Context, Disk

SEG = 2048
def ops(b):
    i, pos, out = 0, 0, []
    while i < len(b):
        if b[i] != 0xF1:
            j = b.find(b'\xf1', i)
            j = len(b) if j < 0 else j
            pos += j - i; i = j; continue
        op = b[i + 1]
        if op == 0: i += 2; pos += 1
        elif op == 1: out.append(('X', pos)); i += 2 + SEG; pos += SEG
        else: out.append(('R', pos, b[i+2:i+10].hex())); i += 10; pos += SEG
    return out

ref = Oracle(ref=True)
nb = int(sys.argv[1]) if len(sys.argv) > 1 else 4
limit, disk = 40 * SEG, (18 + nb * 205) * SEG
local = '%08x-0000-4000-8000-%012x' % (0xD15C, 0x5A7E)
d = synth.stream(0x5A7, 6 << 20, 25, 0)
offs, lens = synth.chunks_of(d, 65536)
k = len(offs) // 2
parts = [(offs[:k], lens[:k]), (offs[k:], lens[k:])]
tmp = tempfile.mkdtemp()
vref = os.path.join(tmp, 'ref.vol')
pa = ref.cache_open_pair(limit, disk, vref, local)
e1 = ref.encode_batch(d, *parts[0], mode=MODE_STREAM, cache=pa)
ref.disk_save(pa, vref)
print('ref run1 stats', ref.pair_stats(pa, disk_live=True))
K = Disk(disk)
ca = Context(0, memory_cache_limit=limit, disk=K, uuid=local)
g1 = ca.encode_chunks(d, *parts[0], semantics=XCG_SEM_STREAM)
print('run1 equal', g1 == e1, 'gpu stats', ca.pair_stats(), K.stats(), 'head', K.head())
vg = os.path.join(tmp, 'gpu.vol')
K.save(vg)
ca.close(); K.close()
print('files equal', open(vg, 'rb').read() == open(vref, 'rb').read())
K2 = Disk(disk, path=vg)
print('reloaded head', K2.head(), 'stats', K2.stats())
c2 = Context(0, memory_cache_limit=limit, disk=K2, uuid=local)
print('reloaded pair stats', c2.pair_stats(), 'xuid', c2.xuid())
pa2 = ref.cache_open_pair(limit, disk, vref, '%08x-0000-4000-8000-%012x' % (0xD15C, 0x999))
print('ref reloaded stats', ref.pair_stats(pa2, disk_live=True))
B = int(sys.argv[2]) if len(sys.argv) > 2 else 8
for step in range(0, k, B):
    sl = (parts[0][0][step:step + B], parts[0][1][step:step + B])
    g = c2.encode_chunks(d, *sl, semantics=XCG_SEM_STREAM)
    e = ref.encode_batch(d, *sl, mode=MODE_STREAM, cache=pa2)
    if g != e:
        for i, (a, b) in enumerate(zip(g, e)):
            if a != b:
                oa, ob = ops(a), ops(b)
                j = next((t for t in range(min(len(oa), len(ob))) if oa[t] != ob[t]), min(len(oa), len(ob)))
                print('chunk', step + i, 'differs at op', j, 'gpu', oa[j:j+3], 'ref', ob[j:j+3], 'nops', len(oa), len(ob))
                break
        print('gpu stats', c2.pair_stats(), 'ref', ref.pair_stats(pa2, disk_live=True))
        break
else:
    print('all equal', c2.pair_stats(), ref.pair_stats(pa2, disk_live=True))
