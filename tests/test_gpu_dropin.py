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
