"""The decoding side of wanproxy on the engine: XCodecDecoder on an
XCodecCachePair (xcodec/xcodec_cache.h:140-237; decode: xcodec/xcodec_decoder.cc:
66-272), caches made by XCodecCache::connect (xcodec/xcodec_cache.h:101-111, as
XCodecPipePair makes its decoder's cache on <HELLO>, xcodec/xcodec_pipe_pair.cc:
203), and one XCodecDisk shared by the local pair and the connected ones
(xcodec/xcodec_cache_disk.h:33-69).  Checked call by call against the real
reference classes (oracle/_ref/libxcref.so; the disk level is the restated
RefDisk of oracle/ref_driver.cc: XCodecDisk itself needs libuuid's header)."""
import importlib.util
import os
import random

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
_spec = importlib.util.spec_from_file_location('make_pair_golden', os.path.join(HERE, 'golden/make_pair_golden.py'))
mpg = importlib.util.module_from_spec(_spec)
_spec.loader.exec_module(mpg)
SEG = 2048


@pytest.fixture(scope='module')
def dropin():
    p = os.path.join(ROOT, 'oracle/_ref/libxcdropin.so')
    if not os.path.exists(p):
        pytest.skip('drop-in harness not built (needs the reference sources at build time)')
    from oracle.lib import Oracle
    return Oracle(dropin=True)


_uuid_n = [0]


def uuid():
    """A fresh 36-character UUID string per connect (the registry is process-wide)."""
    _uuid_n[0] += 1
    return '%08x-0000-4000-8000-%012x' % (os.getpid() & 0xFFFFFFFF, _uuid_n[0])


def frames_of(ref_oracle, d, chunk, make_cache):
    """The reference encoder's frames of d in `chunk`-byte encode() calls on a
    cache make_cache(ref_oracle) (one persistent encoder)."""
    c = make_cache(ref_oracle)
    e = ref_oracle.encoder_new(c)
    fr = [ref_oracle.encode_refmap(e, d[a:a + chunk])[0] for a in range(0, len(d), chunk)]
    ref_oracle.encoder_free(e)
    ref_oracle.cache_free(c)
    return fr


def decode_calls(o, cache, frames):
    dec = o.decoder_new(cache)
    res = [o.decode(f, cache, decoder=dec) for f in frames]
    o.decoder_free(dec)
    return res


@pytest.mark.parametrize('geom', [(120, 2), (40, 1), (300, 6)])
def test_pair_decoder_call_by_call(dropin, ref_oracle, geom):
    """One persistent decoder on a pair, frame by frame: output, consumed bytes,
    ASK sets and the disk counters equal the reference's.  The encoder side ran
    on a larger pair, so the decoder's smaller pair evicts and promotes."""
    limit, nb = geom[0] * SEG, geom[1]
    d = mpg.inputs('pair_far') + mpg.inputs('pair_hot')[:1 << 20]
    frames = frames_of(ref_oracle, d, 65536, lambda o: o.cache_new_pair(400 * SEG, mpg.disk_bytes(12)))
    res, stats = [], []
    for o in (ref_oracle, dropin):
        c = o.cache_new_pair(limit, mpg.disk_bytes(nb))
        res.append(decode_calls(o, c, frames))
        stats.append(o.pair_stats(c))
        o.cache_free(c)
    for k, (a, b) in enumerate(zip(*res)):
        assert a == b, (geom, k, a[0], b[0], a[2], b[2], len(a[3]), len(b[3]))
    assert stats[0] == stats[1]
    if geom[0] < 200:
        assert any(r[3] for r in res[0]), 'the small pair never asked: the case tests nothing'


@pytest.mark.parametrize('geom', [(8, 1, 16), (3, 1, 200), (40, 2, 64)])
def test_pair_decoder_ref_dense(dropin, ref_oracle, geom):
    """REF-dense frames (synth.dense: 2 KiB blocks from a small pool) decoded
    frame by frame on a pair of the encoder's geometry: hundreds of REFs per
    entity in one frame, a disk of one or two index blocks that dies and is
    touched again.  Output, consumed bytes, ASK sets and the disk counters
    equal the reference decoder's (the drop-in cuts what one batch declines)."""
    from wanproxy_amd import synth
    lim, nb, distinct = geom
    d = synth.dense(0xDE1 + distinct, 4 << 20, distinct)

    def mk(o):
        return o.cache_new_pair(lim * SEG, mpg.disk_bytes(nb))
    frames = frames_of(ref_oracle, d, 65536, mk)
    assert sum(map(len, frames)) < len(d)
    res, stats = [], []
    for o in (ref_oracle, dropin):
        c = mk(o)
        res.append(decode_calls(o, c, frames))
        stats.append(o.pair_stats(c))
        o.cache_free(c)
    for k, (a, b) in enumerate(zip(*res)):
        assert a == b, (geom, k, a[0], b[0], a[2], b[2], len(a[3]), len(b[3]))
    assert stats[0] == stats[1]


def test_pair_decode_batch_vs_reference(ref_oracle):
    """The engine's batch decode (many frames, one launch chain) on a pair
    context equals the reference decoder run over the same frames one call at
    a time, up to the first ASK, with the same disk counters."""
    from wanproxy_amd.xcgpu import Context
    d = mpg.inputs('pair_far')
    frames = frames_of(ref_oracle, d, 65536, lambda o: o.cache_new_pair(200 * SEG, mpg.disk_bytes(6)))
    limit, disk = 200 * SEG, mpg.disk_bytes(6)
    c = ref_oracle.cache_new_pair(limit, disk)
    exp = decode_calls(ref_oracle, c, frames)
    est = ref_oracle.pair_stats(c)
    ref_oracle.cache_free(c)
    assert all(r[0] and not r[3] for r in exp)
    ctx = Context(0, memory_cache_limit=limit, disk_bytes=disk)
    for a in range(0, len(frames), 7):         # batches of 7 frames
        outs, st, cons, unk = ctx.decode_chunks(frames[a:a + 7])
        assert not (st != 0).any() and not unk, a
        assert outs == [r[1] for r in exp[a:a + 7]], a
    st = ctx.pair_stats()
    ctx.close()
    assert (st[1], st[2]) == est
    assert b''.join(r[1] for r in exp) == d


@pytest.mark.parametrize('kind', ['bounded', 'pair'])
def test_dropin_connected_caches_like_reference(dropin, ref_oracle, kind):
    """wanproxy's receiving proxy: the codec's own cache encodes one direction
    while the cache XCodecCache::connect made for the peer decodes the other.
    The connected cache is bounded with the parent's limit
    (xcodec_cache.h:297-301) or a pair of connected levels on the SAME disk
    (:158-161, XCodecDisk::connect): the two interleave in one FIFO ring.  Every
    call's output (and refmap / ASK set) and the disk counters equal the
    reference's."""
    from wanproxy_amd import synth
    limit, disk = 150 * SEG, mpg.disk_bytes(3)
    mk = (lambda o: o.cache_new(limit)) if kind == 'bounded' else (lambda o: o.cache_new_pair(limit, disk))
    peer = synth.stream(0xC0DE, 3 << 20, 40, 0)
    frames = frames_of(ref_oracle, peer, 65536, mk)        # what the peer sends (its own cache of that geometry)
    local = synth.stream(0x10CA1, 3 << 20, 40, 0)
    u = uuid()
    res = []
    for o in (ref_oracle, dropin):
        parent = mk(o)
        conn = o.cache_connect(parent, u)
        assert o.cache_connect(parent, u) == conn         # the registry returns the same cache
        enc = o.encoder_new(parent)
        dec = o.decoder_new(conn)
        calls = []
        for k, f in enumerate(frames):
            calls.append(o.encode_refmap(enc, local[k * 65536:(k + 1) * 65536]))
            calls.append(o.decode(f, conn, decoder=dec))
        if kind == 'pair':
            calls.append((o.pair_stats(parent, disk_live=True), o.pair_stats(conn, disk_live=True)))
        o.encoder_free(enc)
        o.decoder_free(dec)
        res.append(calls)
    for k, (a, b) in enumerate(zip(*res)):
        assert a == b, (kind, k)
    if kind == 'pair':
        assert res[0][-1][0][1] > 2 * 204 * 3, 'the shared disk never lapped'


def test_dropin_pair_ask_learn(dropin, ref_oracle):
    """A pair decoder that lacks what the frames name blocks with the
    reference's ASK set; <LEARN>ing the segments into the host cache (the pipe
    pair's lookup + enter, xcodec_pipe_pair.cc:296-327) lets it continue, as
    the reference does."""
    d = mpg.inputs('pair_far')[:2 << 20]
    frames = frames_of(ref_oracle, d, 65536, lambda o: o.cache_new(0))
    segs = {}
    for a in range(0, len(d) - SEG + 1, SEG):
        segs[ref_oracle.hash(d[a:a + SEG])] = d[a:a + SEG]
    res = []
    for o in (ref_oracle, dropin):
        c = o.cache_new_pair(60 * SEG, mpg.disk_bytes(1))
        dec = o.decoder_new(c)
        calls = []
        for f in frames[::2] + frames[1::2]:              # frames out of order: unknown REFs
            buf = f
            for _ in range(8):
                ok, out, cons, unk = o.decode(buf, c, decoder=dec)
                calls.append((ok, out, cons, unk))
                buf = buf[cons:]
                if not unk or not buf:
                    break
                for h in unk:
                    if h in segs:
                        o.cache_learn(c, segs[h])
        calls.append(o.pair_stats(c))
        o.decoder_free(dec)
        res.append(calls)
    assert res[0] == res[1]
    assert sum(1 for r in res[0][:-1] if r[3]) > 3


def _collision_pair():
    """X, Y with XCodecHash(X) == XCodecHash(Y), X != Y."""
    r = random.Random(42)
    x = bytearray(min(201, max(7, r.getrandbits(8) | 1)) for _ in range(SEG))
    y = bytearray(x)
    y[100] += 2
    y[101] -= 4
    y[102] += 2
    return bytes(x), bytes(y)


def _extract(seg):
    return b'\xf1\x01' + seg


def _ref(h):
    return b'\xf1\x02' + h.to_bytes(8, 'big')


def name_reuse_calls(hash_fn):
    """Decode calls exercising name reuse on a 3-slot pair (see below)."""
    x, y = _collision_pair()
    h = hash_fn(x)
    assert h == hash_fn(y) and x != y
    r = random.Random(5)
    fill = [bytes(r.getrandbits(8) | 1 for _ in range(SEG)) for _ in range(6)]
    return x, y, [
        _extract(x) + b'lit',
        _ref(h) + _extract(y) + _ref(h) + b'\xf1\x00',
        b''.join(_extract(s) for s in fill[:4]),         # push h out of a 3-slot primary (disk only)
        _extract(x) + _ref(h),                           # disk hit, promoted, then replaced back to x
        _ref(h) + b''.join(_extract(s) for s in fill[4:]) + _ref(h),
    ]


def name_reuse_run(o, calls):
    c = o.cache_new_pair(3 * SEG, mpg.disk_bytes(1))
    res = decode_calls(o, c, calls) + [o.pair_stats(c)]
    o.cache_free(c)
    return res


def test_pair_decode_name_reuse(dropin):
    """<EXTRACT> of cached bytes under a hash the cache holds with other bytes
    (name reuse, xcodec_decoder.cc:110-133): the pair replaces at both levels
    (primary replace + disk remove / enter), and later REFs get the new bytes
    -- on a primary hit and on a disk-only hit (promoted first).

    Checked against the oracle restatement, not the reference in-process: the
    reference's XCodecMemoryCache::replace stores the new segment without a
    reference (xcodec_cache.h:333-336), so when the replaced entry is evicted
    its window's pointer dangles and the next window collision unrefs freed
    memory (xcodec_window.h:77-80) -- a crash that comes and goes with the
    heap.  tests/test_pair_oracle.py pins the restatement to the reference on
    these calls in a child process."""
    from oracle.lib import Oracle
    port = Oracle()
    x, y, calls = name_reuse_calls(port.hash)
    exp = name_reuse_run(port, calls)
    assert name_reuse_run(dropin, calls) == exp
    assert exp[1][1] == x + y + y + b'\xf1'


def test_shared_disk_contexts_vs_reference(ref_oracle):
    """Two pair contexts on one engine disk (xcg_ctx_create_pair_on) encoding
    in alternation equal the reference's local pair and a connected pair on one
    XCodecDisk: every chunk, and every front's disk counters."""
    from oracle.lib import MODE_STREAM
    from wanproxy_amd import synth
    from wanproxy_amd.xcgpu import XCG_SEM_STREAM, Context, Disk
    limit, disk = 100 * SEG, mpg.disk_bytes(2)
    da = synth.stream(0xA11, 2 << 20, 30, 0)
    db = synth.stream(0xB22, 2 << 20, 30, 0)
    oa, la = synth.chunks_of(da, 65536)
    ob, lb = synth.chunks_of(db, 65536)
    pa = ref_oracle.cache_new_pair(limit, disk)
    pb = ref_oracle.cache_connect(pa, uuid())
    exp, est = [], []
    for k in range(0, len(oa), 4):
        exp.append(ref_oracle.encode_batch(da, oa[k:k + 4], la[k:k + 4], mode=MODE_STREAM, cache=pa))
        exp.append(ref_oracle.encode_batch(db, ob[k:k + 4], lb[k:k + 4], mode=MODE_STREAM, cache=pb))
    est = [ref_oracle.pair_stats(pa, disk_live=True), ref_oracle.pair_stats(pb, disk_live=True)]
    K = Disk(disk)
    ca = Context(0, memory_cache_limit=limit, disk=K)
    cb = Context(0, memory_cache_limit=limit, disk=K)
    got = []
    for k in range(0, len(oa), 4):
        got.append(ca.encode_chunks(da, oa[k:k + 4], la[k:k + 4], semantics=XCG_SEM_STREAM))
        got.append(cb.encode_chunks(db, ob[k:k + 4], lb[k:k + 4], semantics=XCG_SEM_STREAM))
    sa, sb, ks = ca.pair_stats(), cb.pair_stats(), K.stats()
    ca.close()
    cb.close()
    K.close()
    for k, (a, b) in enumerate(zip(exp, got)):
        assert a == b, k
    assert (sa[1], sa[2], ks[0]) == est[0]
    assert (sb[1], sb[2], ks[0]) == est[1]
    assert ks[1] > 3 * 2 * 204, 'the shared disk never lapped'


def test_pair_host_lookup_enter(ref_oracle):
    """Single-segment host calls on a pair context (XCodecPipePair's <LEARN>
    path): enter puts a segment in both levels, lookups find it (and promote a
    disk-only one), a wrong hash is refused."""
    from wanproxy_amd.xcgpu import XCGError, Context
    r = random.Random(9)
    segs = [bytes(r.getrandbits(8) for _ in range(SEG)) for _ in range(6)]
    hs = [ref_oracle.hash(s) for s in segs]
    ctx = Context(0, memory_cache_limit=2 * SEG, disk_bytes=mpg.disk_bytes(1))
    for h, s in zip(hs, segs):
        ctx.cache_enter(h, s)
    st = ctx.pair_stats()
    assert st[0] == 2 and st[1] == 6
    for h, s in zip(hs, segs):                      # disk-only ones promote on lookup
        assert ctx.cache_lookup(h) == s
    assert ctx.cache_lookup(hs[0] ^ (1 << 40)) is None
    with pytest.raises(XCGError):
        ctx.cache_enter(hs[0], segs[1])
    ctx.close()
