"""Drop-in conformance: the reference's own driver code and Buffer / cache
classes, with XCodecEncoder / XCodecDecoder provided by integration/ on the
GPU engine (oracle/_ref/libxcdropin.so), against the reference goldens.
This is the class boundary tack and XCodecPipePair call
(xcodec/xcodec_encoder.h:40-43, xcodec/xcodec_decoder.h:41-45)."""
import os

import pytest

from golden_cases import MODES, chunks, data, sha

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.fixture(scope='module')
def dropin():
    p = os.path.join(ROOT, 'oracle/_ref/libxcdropin.so')
    if not os.path.exists(p):
        pytest.skip('drop-in harness not built (needs the reference sources at build time)')
    from oracle.lib import Oracle
    return Oracle(dropin=True)


def test_dropin_golden_stream_and_null(dropin, golden):
    n = 0
    for case in golden['cases']:
        if case['mode'] not in ('stream', 'null'):
            continue
        d, (offs, lens) = chunks(case)
        outs = dropin.encode_batch(d, offs, lens, mode=MODES[case['mode']], oob=case['mode'] == 'null')
        assert [sha(o)[:32] for o in outs] == case['chunk_sha256'], (case['input'], case['chunk'], case['mode'])
        n += 1
    assert n >= 15


def test_dropin_baseline_tack_shas(dropin, golden):
    for name, b in golden['baseline'].items():
        enc = dropin.encode_stream(data(name))
        assert (len(enc), sha(enc)) == (b['xc_len'], b['xc']), name


def test_dropin_decode_round_trip(dropin, ref_oracle):
    for name in ('kat_a', 'kat_b', 'kat_z', 'kat_col', 'magic_heavy', 'all_f1'):
        d = data(name)
        enc = ref_oracle.encode_stream(d)
        c = dropin.cache_new()
        ok, out, consumed, unk = dropin.decode(enc, c)
        dropin.cache_free(c)
        assert ok and not unk and consumed == len(enc) and out == d, name


def test_dropin_decode_unknown_like_reference(dropin, ref_oracle):
    d = data('kat_a')
    enc = ref_oracle.encode_stream(d)
    start = enc.index(b'\xf1\x02')
    res = []
    for o in (dropin, ref_oracle):
        c = o.cache_new()
        ok, out, consumed, unk = o.decode(enc[start:], c)
        o.cache_free(c)
        res.append((ok, out, consumed, sorted(unk)))
    assert res[0] == res[1]


def test_dropin_refmap_like_reference(dropin, ref_oracle):
    # encode(output, input, &refmap) as XCodecPipePair calls it
    # (xcodec/xcodec_pipe_pair.cc:610-618): the drop-in's output and refmap
    # (hash -> segment of every REF made) equal the reference's, call by call
    # on one persistent encoder + cache.
    from wanproxy_amd import synth
    d = synth.stream(0x7EF, 3 << 20, 60, 2)
    pieces = [d[a:a + 524288] for a in range(0, len(d), 524288)] + [d[:70000], d[100:2200], b'x' * 3000]
    encs = []
    for o in (ref_oracle, dropin):
        c = o.cache_new()
        e = o.encoder_new(c)
        encs.append([o.encode_refmap(e, p) for p in pieces])
        o.encoder_free(e)
        o.cache_free(c)
    for k, (r, g) in enumerate(zip(*encs)):
        assert r[0] == g[0], k
        assert r[1] == g[1], (k, len(r[1]), len(g[1]))
    assert sum(len(r[1]) for r in encs[0]) > 100


@pytest.mark.parametrize('kind', ['bounded', 'pair'])
def test_dropin_refmap_bounded_and_pair_like_reference(dropin, ref_oracle, kind):
    """The same calls on a bounded XCodecMemoryCache and on wanproxy.conf's
    XCodecCachePair: output and refmap call by call equal the reference's, and
    the host cache the adapter keeps in step (by replaying the engine's cache
    references in stream order, xcg_last_references) keeps agreeing with the
    engine -- later calls depend on its LRU order and disk contents."""
    import importlib.util
    from wanproxy_amd import synth
    spec = importlib.util.spec_from_file_location('mpg', os.path.join(ROOT, 'tests/golden/make_pair_golden.py'))
    mpg = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mpg)
    d = mpg.inputs('pair_far') + mpg.inputs('pair_hot')[:1 << 20]
    pieces = [d[a:a + 65536] for a in range(0, len(d), 65536)] + [d[:70000], d[100:2200], b'x' * 3000]
    res = []
    for o in (ref_oracle, dropin):
        c = o.cache_new(120 * 2048) if kind == 'bounded' else o.cache_new_pair(120 * 2048, mpg.disk_bytes(2))
        e = o.encoder_new(c)
        res.append([o.encode_refmap(e, p) for p in pieces])
        o.encoder_free(e)
        o.cache_free(c)
    for k, (a, b) in enumerate(zip(*res)):
        assert a == b, (kind, k)


def _uuid(k):
    return '%08x-0000-4000-8000-%012x' % (os.getpid() & 0xFFFFFFFF, k)


@pytest.mark.parametrize('limit_segs', [40, 0], ids=['bounded', 'unbounded'])
@pytest.mark.parametrize('nb', [3, 10])
def test_dropin_pair_reopened_volume_like_reference(dropin, ref_oracle, tmp_path, nb, limit_segs):
    """(limit_segs 0: the pair's primary is an unbounded XCodecMemoryCache,
    which never evicts -- the engine still runs it as a pair, so a primary
    miss finds the reopened volume's entries and the peer's front, loaded from
    the volume, serves the new pair over it: REFs where a plain memory cache
    would EXTRACT, xcodec/xcodec_cache.h:208-230.)
    wanproxy restarted on its cache volume (XCodecDisk::open,
    xcodec_cache_disk.cc:826-871): the first process encodes through the
    drop-in on a pair over the volume (the local front and a peer's), the
    volume is written and the caches go away; a second process opens the same
    file -- the host XCodecDisk reloads it (:107-237) and the engine's disk is
    read from the same file with the same reload -- and encodes on through the
    local front and the peer's front, found again by UUID.  Every call's output
    and refmap, the disk counters and the volume written by each process equal
    the reference's.  A fresh engine disk would not do: the second process REFs
    segments only the first declared."""
    from wanproxy_amd import synth
    limit, disk = limit_segs * 2048, (18 + nb * 205) * 2048
    local, peer = _uuid(0x300 + nb + 0x20 * (limit_segs == 0)), _uuid(0x400 + nb + 0x20 * (limit_segs == 0))
    d = synth.stream(0x5E1 + nb, 9 << 20, 25, 0)
    e = synth.stream(0x6E1 + nb, 6 << 20, 25, 0)
    calls = lambda x, a, b: [x[k:k + 65536] for k in range(a << 20, b << 20, 65536)]

    def run(o, tag):
        vol = str(tmp_path / f'{tag}.vol')
        out = []
        pa = o.cache_open_pair(limit, disk, vol, local)
        pb = o.cache_pair_front(pa, peer, limit)
        ea, eb = o.encoder_new(pa), o.encoder_new(pb)
        out += [o.encode_refmap(eb, p) for p in calls(e, 0, 3)]
        out += [o.encode_refmap(ea, p) for p in calls(d, 0, 6)]
        out.append(o.pair_stats(pa, disk_live=True))
        o.disk_save(pa, vol)
        first = open(vol, 'rb').read()
        o.encoder_free(ea)
        o.encoder_free(eb)
        o.cache_free(pb)
        o.cache_free(pa)
        # the restart: a new process's XCodecDisk on the same file
        pa2 = o.cache_open_pair(limit, disk, vol, _uuid(0x999))
        pb2 = o.cache_pair_front(pa2, peer, limit)
        ea2, eb2 = o.encoder_new(pa2), o.encoder_new(pb2)
        second = [o.encode_refmap(ea2, p) for p in calls(d, 5, 9)]
        second += [o.encode_refmap(eb2, p) for p in calls(e, 3, 6)]
        second += [(o.pair_stats(pa2, disk_live=True), o.pair_stats(pb2, disk_live=True))]
        o.disk_save(pa2, vol)
        o.encoder_free(ea2)
        o.encoder_free(eb2)
        return out, first, second, open(vol, 'rb').read()

    ref, gpu = run(ref_oracle, 'ref'), run(dropin, 'gpu')
    for k, (a, b) in enumerate(zip(ref[0], gpu[0])):
        assert a == b, ('first process', k)
    assert ref[1] == gpu[1], 'the first process left a different volume'
    for k, (a, b) in enumerate(zip(ref[2], gpu[2])):
        assert a == b, ('after the reopen', k)
    assert ref[3] == gpu[3], 'the second process left a different volume'
    # the reload made a difference: on a fresh volume the same calls declare more
    pf = ref_oracle.cache_new_pair(limit, disk)
    ef = ref_oracle.encoder_new(pf)
    fresh = [ref_oracle.encode_refmap(ef, p)[0] for p in calls(d, 5, 6)]
    ref_oracle.encoder_free(ef)
    assert sum(map(len, fresh)) > sum(len(r[0]) for r in ref[2][:len(fresh)]) + 100 * 2040


def test_dropin_decode_bounded_like_reference(dropin, ref_oracle):
    """One persistent decoder on a bounded cache, frame by frame (the REF
    lookups refresh its LRU: the adapter replays them into the host cache)."""
    from oracle.lib import MODE_STREAM
    from wanproxy_amd import synth
    d = synth.stream(0xDEC, 3 << 20, 60, 0)
    offs, lens = synth.chunks_of(d, 65536)
    c = ref_oracle.cache_new(300 * 2048)
    encs = ref_oracle.encode_batch(d, offs, lens, mode=MODE_STREAM, cache=c)
    ref_oracle.cache_free(c)
    res = []
    for o in (ref_oracle, dropin):
        dc = o.cache_new(300 * 2048)
        dec = o.decoder_new(dc)
        res.append([o.decode(e, dc, decoder=dec) for e in encs])
        o.decoder_free(dec)
        o.cache_free(dc)
    assert res[0] == res[1]


@pytest.mark.parametrize('shift', [0, -1, 1, -2050, 8])
def test_dropin_decode_op_at_the_piece_cut(dropin, ref_oracle, shift):
    """A decode() of more than 1 MiB on a bounded cache is cut into pieces of
    whole ops (integration/xcodec_decoder_xcgpu.cc cut_pieces).  An EXTRACT
    whose payload ends in 0xF1 placed to end exactly at the 1 MiB cut (and
    around it): the cut must not take the payload's last 0xF1 for an op start.
    Output, consumed bytes and ASK set equal the reference decoder's."""
    import random
    r = random.Random(0xC07 + shift)
    seg = bytearray(r.getrandbits(8) for _ in range(2048))
    for k in range(0, 2048, 97):
        seg[k] = 0xF1
    seg[-1] = 0xF1
    seg = bytes(seg)
    h = ref_oracle.hash(seg)
    lit = lambda n: bytes(r.randrange(0xF1) for _ in range(n))
    ext = b'\xf1\x01' + seg
    pre = (1 << 20) + shift - len(ext)
    stream = lit(pre) + ext + b'\xf1\x02' + h.to_bytes(8, 'big') + lit(3000) + b'\xf1\x00' + lit(7) + ext + lit(100)
    res = []
    for o in (ref_oracle, dropin):
        c = o.cache_new(300 * 2048)
        dec = o.decoder_new(c)
        res.append(o.decode(stream, c, decoder=dec))
        o.decoder_free(dec)
        o.cache_free(c)
    assert res[0] == res[1]
    assert res[0][0] and res[0][2] == len(stream) and res[0][1].count(seg) == 3


def _crafted_streams(ref_oracle):
    """Frames that stress the per-call decode's op walk (decode_small_kernel,
    parallel pointer-jumping walk): escapes next to ops, 0xF1 bytes inside
    EXTRACT payloads and REF hashes, a lone 0xF1 at the end, EXTRACT / REF cut
    short, an unknown opcode, a BACKREF (the batch path), no 0xF1 at all, an
    empty call, and payloads full of 0xF1 (more candidate op starts than the
    parallel walk holds: the sequential walk)."""
    import random
    r = random.Random(0x5A1C)
    lit = lambda n: bytes(r.randrange(0xF1) for _ in range(n))
    seg = lambda f1: bytes(0xF1 if r.random() < f1 else r.randrange(256) for _ in range(2048))
    s1, s2, s3 = seg(0.01), seg(0.3), seg(1.0)
    h = lambda s: ref_oracle.hash(s).to_bytes(8, 'big')
    ext = lambda s: b'\xf1\x01' + s
    ref = lambda s: b'\xf1\x02' + h(s)
    esc = b'\xf1\x00'
    out = [
        lit(100) + ext(s1) + esc + ref(s1) + esc + esc + lit(3) + ext(s2) + ref(s2) + ref(s1) + lit(50) + esc,
        esc + ext(s1) + ref(s1) * 40 + lit(7) + b'\xf1',
        lit(9) + ext(s2) + ext(s1)[:1000],
        lit(9) + ext(s1) + ref(s1)[:6],
        lit(20) + ext(s1) + b'\xf1\x07' + lit(30),
        lit(20) + ext(s1) + b'\xf1\x03\x05' + lit(30),
        lit(5000),
        b'',
        ext(s3) + ext(seg(0.99)) + ref(s3) + lit(11),
        (ext(s2) + ref(s2) + esc + lit(1)) * 30,
    ]
    return out


def test_dropin_decode_call_walk_edges(dropin, ref_oracle):
    """Each crafted frame decoded by one decode() call on a fresh unbounded
    cache: output, consumed bytes and ASK set equal the reference decoder's."""
    for k, stream in enumerate(_crafted_streams(ref_oracle)):
        res = []
        for o in (ref_oracle, dropin):
            c = o.cache_new()
            res.append(o.decode(stream, c))
            o.cache_free(c)
        assert res[0][:3] == res[1][:3] and sorted(res[0][3]) == sorted(res[1][3]), k
