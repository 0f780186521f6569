"""The oracle's XCodecCachePair (xcodec/xcodec_cache.h:140-237) of a bounded
XCodecMemoryCache primary and a disk FIFO secondary (XCodecDisk,
xcodec/xcodec_cache_disk.cc:694-823) pinned against the reference: fixtures
made by tests/golden/make_pair_golden.py from the real pair, encoder and
decoder over a restated disk level (oracle/ref_driver.cc RefDiskCache; the
reference's XCodecDisk needs libuuid's header, absent here), and a direct
comparison with oracle/_ref when it is built."""
import hashlib
import importlib.util
import json
import os

import pytest

from oracle.lib import MODE_STREAM

HERE = os.path.dirname(os.path.abspath(__file__))
_spec = importlib.util.spec_from_file_location('make_pair_golden', os.path.join(HERE, 'golden/make_pair_golden.py'))
mpg = importlib.util.module_from_spec(_spec)
_spec.loader.exec_module(mpg)


def sha(b):
    return hashlib.sha256(b).hexdigest()


@pytest.fixture(scope='module')
def pair_golden():
    with open(os.path.join(HERE, 'golden/pair.json')) as f:
        return json.load(f)


def pair_inputs(name, _memo={}):
    if name not in _memo:
        _memo[name] = mpg.inputs(name)
    return _memo[name]


def test_pair_inputs_pinned(pair_golden):
    for name, meta in pair_golden['inputs'].items():
        d = pair_inputs(name)
        assert (len(d), sha(d)) == (meta['len'], meta['sha256']), name


def test_pair_geometry():
    # XCodecDisk(fd, size): (size / 2048 - 18) / 205 index blocks of 204 entries
    assert mpg.disk_bytes(1) == (18 + 205) * 2048
    from oracle.lib import Oracle
    o = Oracle()
    with pytest.raises(ValueError):
        o.cache_new_pair(1 << 20, 222 * 2048)            # one block short of an index block
    c = o.cache_new_pair(1 << 20, mpg.disk_bytes(3))
    o.cache_free(c)


def test_pair_encode_golden(pair_golden, oracle):
    from wanproxy_amd.synth import chunks_of
    for case in pair_golden['cases']:
        d = pair_inputs(case['input'])
        offs, lens = chunks_of(d, case['chunk'])
        c = oracle.cache_new_pair(case['limit'], case['disk'])
        outs = oracle.encode_batch(d, offs, lens, mode=MODE_STREAM, cache=c)
        entries, written = oracle.pair_stats(c)
        oracle.cache_free(c)
        key = (case['input'], case['chunk'], case['limit'], case['disk'])
        assert [len(o) for o in outs] == case['lens'], key
        assert [sha(o)[:32] for o in outs] == case['chunk_sha256'], key
        assert (entries, written) == (case['disk_entries'], case['disk_written']), key


def test_pair_decode_golden(pair_golden, oracle):
    from wanproxy_amd.synth import chunks_of
    for case in pair_golden['cases']:
        d = pair_inputs(case['input'])
        offs, lens = chunks_of(d, case['chunk'])
        c = oracle.cache_new_pair(case['limit'], case['disk'])
        encs = oracle.encode_batch(d, offs, lens, mode=MODE_STREAM, cache=c)
        oracle.cache_free(c)
        dc = oracle.cache_new_pair(case['limit'], case['disk'])
        dec = oracle.decoder_new(dc)
        for e, want in zip(encs, case['dec']):
            ok, out, cons, unk = oracle.decode(e, dc, decoder=dec)
            got = {'ok': ok, 'consumed': cons, 'nunknown': len(unk), 'out_len': len(out), 'out_sha256': sha(out)}
            assert got == want, (case['input'], case['chunk'], case['limit'])
        oracle.decoder_free(dec)
        oracle.cache_free(dc)


def test_pair_vs_reference_live(ref_oracle, oracle):
    """Random geometries, both libraries on the same stream."""
    import numpy as np
    from wanproxy_amd import synth
    rng = np.random.default_rng(7)
    for t in range(6):
        d = synth.stream(int(rng.integers(1 << 30)), int(rng.integers(1, 5)) << 20, int(rng.integers(10, 70)), 0)
        chunk = int(rng.choice([4096, 16384, 65536, 131072]))
        limit = int(rng.integers(1, 600)) * 2048
        disk = mpg.disk_bytes(int(rng.integers(1, 8)))
        offs, lens = synth.chunks_of(d, chunk)
        res = []
        for lib in (oracle, ref_oracle):
            c = lib.cache_new_pair(limit, disk)
            res.append((lib.encode_batch(d, offs, lens, mode=MODE_STREAM, cache=c), lib.pair_stats(c)))
            lib.cache_free(c)
        assert res[0] == res[1], (t, chunk, limit, disk)


def test_ref_shared_disk_fronts(ref_oracle):
    """The restated XCodecDisk of the reference harness (oracle/ref_driver.cc
    RefDisk): a pair XCodecCache::connect makes for a peer (xcodec_cache.h:158-161)
    is a second front on the SAME disk (XCodecDisk::connect,
    xcodec_cache_disk.cc:640-690).  Its writes lap the ring and take the local
    front's entries with them (index_invalidate_entries walks every front,
    :327-382); the connect registry returns the same cache for a uuid."""
    from wanproxy_amd import synth
    limit, disk = 50 * 2048, mpg.disk_bytes(1)          # 204 data blocks
    pa = ref_oracle.cache_new_pair(limit, disk)
    pb = ref_oracle.cache_connect(pa, '11111111-2222-4333-8444-555555555555')
    assert ref_oracle.cache_connect(pa, '11111111-2222-4333-8444-555555555555') == pb
    a = synth.stream(0xA, 300 * 2048, 0, 0)             # 300 unique segments
    offs, lens = synth.chunks_of(a, 65536)
    ref_oracle.encode_batch(a, offs, lens, mode=MODE_STREAM, cache=pa)
    ea, wa, la = ref_oracle.pair_stats(pa, disk_live=True)
    assert wa == 300 and 0 < ea <= 204 and la == ea
    b = synth.stream(0xB, 250 * 2048, 0, 0)
    offs, lens = synth.chunks_of(b, 65536)
    ref_oracle.encode_batch(b, offs, lens, mode=MODE_STREAM, cache=pb)
    ea2, wa2, la2 = ref_oracle.pair_stats(pa, disk_live=True)
    eb2, wb2, _ = ref_oracle.pair_stats(pb, disk_live=True)
    assert wa2 == wb2 == 550                             # one write head
    assert ea2 == 0 and la2 == eb2 > 0                  # the peer front's lap took every local entry


_NAME_REUSE_CHILD = r'''
import hashlib, json, sys
sys.path[:0] = [sys.argv[1], sys.argv[2]]
import test_gpu_pair_decode as t
from oracle.lib import Oracle
o = Oracle(ref=True)
x, y, calls = t.name_reuse_calls(o.hash)
res = t.name_reuse_run(o, calls)
print(json.dumps([[r[0], hashlib.sha256(r[1]).hexdigest(), r[2], r[3]] for r in res[:-1]] + [list(res[-1])]))
'''


def test_name_reuse_port_vs_reference():
    """The name-reuse calls of tests/test_gpu_pair_decode.py (pair replace at
    both levels, xcodec_decoder.cc:110-133) on the restatement and on the
    reference.  The reference runs in a child process: its replace keeps a
    segment it holds no reference to (xcodec_cache.h:333-336) and a later window
    collision unrefs it after eviction freed it (xcodec_window.h:77-80), which
    may crash; only a clean exit is compared."""
    import subprocess
    import sys
    if not os.path.exists(os.path.join(HERE, '..', 'oracle/_ref/libxcref.so')):
        pytest.skip('oracle/_ref/libxcref.so not built (needs /root/reference)')
    from oracle.lib import Oracle
    sys.path.insert(0, HERE)
    import test_gpu_pair_decode as t
    port = Oracle()
    x, y, calls = t.name_reuse_calls(port.hash)
    res = t.name_reuse_run(port, calls)
    exp = [[r[0], sha(r[1]), r[2], r[3]] for r in res[:-1]] + [list(res[-1])]
    assert res[1][1] == x + y + y + b'\xf1'
    p = subprocess.run([sys.executable, '-c', _NAME_REUSE_CHILD, HERE, os.path.dirname(HERE)],
                       capture_output=True, text=True, timeout=120)
    if p.returncode < 0:
        pytest.xfail('reference crashed (signal %d): its replace/window use-after-free' % -p.returncode)
    assert p.returncode == 0, p.stderr[-2000:]
    assert json.loads(p.stdout.strip().splitlines()[-1]) == exp


def test_ref_volume_save_reopen(ref_oracle, tmp_path):
    """The restated disk's volume file (oracle/ref_driver.cc RefDisk::save /
    load, restating xcodec_cache_disk.cc:72-101 and :107-237): a reopened
    volume indexes exactly the entries of its written index blocks other than
    the write head's (the last entry of a hash wins), and saving it again
    without new writes gives the same file."""
    import struct
    from wanproxy_amd import synth
    spec = importlib.util.spec_from_file_location('make_pair_golden', os.path.join(HERE, 'golden/make_pair_golden.py'))
    mpg = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mpg)
    nb, limit = 5, 30 * 2048
    disk = mpg.disk_bytes(nb)
    local = '0000aaaa-0000-4000-8000-000000000001'
    d = synth.stream(0xF11E, 3 << 20, 25, 0)
    offs, lens = synth.chunks_of(d, 65536)
    v1, v2 = str(tmp_path / 'a.vol'), str(tmp_path / 'b.vol')
    pa = ref_oracle.cache_open_pair(limit, disk, v1, local)
    ref_oracle.encode_batch(d, offs, lens, mode=MODE_STREAM, cache=pa)
    ref_oracle.disk_save(pa, v1)
    vol = open(v1, 'rb').read()
    ctr = [struct.unpack_from('<Q', vol, (18 + b) * 2048)[0] for b in range(nb)]
    head = min(range(nb), key=lambda b: ctr[b]) if 0 not in ctr else ctr.index(0)
    want = {}
    for b in sorted((b for b in range(nb) if ctr[b] and b != head), key=lambda b: ctr[b]):
        for j in range(204):
            x, h = struct.unpack_from('<HQ', vol, (18 + b) * 2048 + 8 + 10 * j)
            if h and x == 0:
                want[h] = b * 204 + j
    pb = ref_oracle.cache_open_pair(limit, disk, v1, '0000aaaa-0000-4000-8000-0000000000ff')
    assert ref_oracle.pair_stats(pb)[0] == len(want) > 0
    ref_oracle.disk_save(pb, v2)
    assert open(v2, 'rb').read() == vol
