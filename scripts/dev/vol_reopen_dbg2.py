"""Debug: the exact sequence of tests/test_gpu_disk.py
test_volume_saved_after_its_fronts_are_gone, with variants (argv[1]):
  a  save open + close + save closed, reopen from closed (the test)
  b  save open, close, reopen from open
  c  close, save closed only, reopen from closed"""
import os, sys, tempfile
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))), 'tests'))
from oracle.lib import Oracle, MODE_STREAM
from wanproxy_amd import synth
from wanproxy_amd.xcgpu import XCG_SEM_STREAM, Context, Disk
from test_gpu_disk import _first_diff, _vol_case, _uuid, mpg, SEG
v = sys.argv[1]
ref = Oracle(ref=True)
limit, disk = 40 * SEG, mpg.disk_bytes(4)
local = _uuid(0x5A7E)
d, parts = _vol_case(0x5A7, 2)
tmp = tempfile.mkdtemp()
vref = os.path.join(tmp, 'ref.vol')
pa = ref.cache_open_pair(limit, disk, vref, local)
for o, l in parts[:1]:
    ref.encode_batch(d, o, l, mode=MODE_STREAM, cache=pa)
ref.disk_save(pa, vref)
K = Disk(disk)
ca = Context(0, memory_cache_limit=limit, disk=K, uuid=local)
for o, l in parts[:1]:
    ca.encode_chunks(d, o, l, semantics=XCG_SEM_STREAM)
open_ = os.path.join(tmp, 'open.vol')
closed = os.path.join(tmp, 'closed.vol')
if v in 'ab':
    K.save(open_)
ca.close()
if v in 'ac':
    K.save(closed)
K.close()
src = open_ if v == 'b' else closed
print(v, 'file equal', open(src, 'rb').read() == open(vref, 'rb').read())
K2 = Disk(disk, path=src)
c2 = Context(0, memory_cache_limit=limit, disk=K2, uuid=local)
got = [c2.encode_chunks(d, o, l, semantics=XCG_SEM_STREAM) for o, l in parts[:1]]
st = c2.pair_stats()
c2.close()
K2.close()
pa2 = ref.cache_open_pair(limit, disk, vref, _uuid(0x999))
exp = [ref.encode_batch(d, o, l, mode=MODE_STREAM, cache=pa2) for o, l in parts[:1]]
print(v, 'equal', got == exp, _first_diff(got[0], exp[0]), st, ref.pair_stats(pa2, disk_live=True))
