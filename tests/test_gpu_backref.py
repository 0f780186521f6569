"""GPU decode of streams with <BACKREF> ops (XCodecWindow semantics,
xcodec/xcodec_decoder.cc:137,160,165-181, xcodec/xcodec_window.h) against the
reference decoder's results (tests/golden/backref.json) and the C oracle."""
import hashlib
import json
import os

import pytest

from wanproxy_amd import synth
from backref_streams import stream_with_backrefs

pytestmark = pytest.mark.gpu

GOLDEN = json.load(open(os.path.join(os.path.dirname(__file__), 'golden', 'backref.json')))


def sha(b: bytes) -> str:
    return hashlib.sha256(b).hexdigest()


def streams(oracle, c):
    data = synth.stream(c['seed'], c['nbytes'], c['dup'], 0)
    encs = stream_with_backrefs(oracle, data, c['chunk'], c['seed'], c['rate'], c['bad'])
    assert sha(b''.join(encs)) == c['stream_sha256']
    return encs


def check_against_golden(c, outs, st, cons):
    calls = c['calls']
    for k, want in enumerate(calls):
        if want['ok']:
            assert int(st[k]) == 0, (c['name'], k, int(st[k]))
        else:
            assert int(st[k]) == -1, (c['name'], k, int(st[k]))
        assert int(cons[k]) == want['consumed'], (c['name'], k)
        assert len(outs[k]) == want['out_len'] and sha(outs[k]) == want['out_sha256'], (c['name'], k)
    for k in range(len(calls), len(st)):          # after decode() returned false
        assert int(st[k]) == 2, (c['name'], k)


@pytest.mark.parametrize('case', GOLDEN['cases'], ids=[c['name'] for c in GOLDEN['cases']])
def test_backref_one_batch(oracle, case):
    from wanproxy_amd.xcgpu import Context
    encs = streams(oracle, case)
    ctx = Context(0)
    outs, st, cons, unk = ctx.decode_chunks(encs)
    assert unk == []
    check_against_golden(case, outs, st, cons)


@pytest.mark.parametrize('case', GOLDEN['cases'], ids=[c['name'] for c in GOLDEN['cases']])
def test_backref_window_across_batches(oracle, case):
    """The window lives in the decoder, across xcg_decode_batch calls."""
    from wanproxy_amd.xcgpu import Context, Window
    encs = streams(oracle, case)
    ctx = Context(0)
    win = Window(ctx)
    outs, st, cons = [], [], []
    cuts = sorted({0, len(encs) // 3, len(encs) // 3 + 1, (2 * len(encs)) // 3, len(encs)})
    for a, b in zip(cuts, cuts[1:]):
        o, s, cn, _ = ctx.decode_chunks(encs[a:b], window=win)
        outs += o
        st += [int(v) for v in s]
        cons += [int(v) for v in cn]
        if min(st) < 0:
            break
    calls = case['calls']
    for k, want in enumerate(calls):
        if k >= len(st):
            break
        assert (st[k] == 0) == want['ok'] and cons[k] == want['consumed'], (case['name'], k)
        assert sha(outs[k]) == want['out_sha256'], (case['name'], k)


def test_backref_decoder_mirror_matches_oracle(oracle):
    """XCodecDecoder mirror (one decode() per call, own window) vs the C
    oracle's persistent decoder on more seeds."""
    from wanproxy_amd.xcgpu import Context, XCodecDecoder
    for seed in (21, 22, 23):
        data = synth.stream(seed, 1 << 19, 70, 1)
        encs = stream_with_backrefs(oracle, data, 16384, seed, 0.4, 0.03 if seed == 23 else 0.0)
        ctx = Context(0)
        dec = XCodecDecoder(ctx)
        cache = oracle.cache_new()
        odec = oracle.decoder_new(cache)
        try:
            for k, e in enumerate(encs):
                ok, out, cons, unk = dec.decode(e)
                wok, wout, wcons, wunk = oracle.decode(e, cache, decoder=odec)
                assert (ok, cons, unk) == (wok, wcons, wunk), (seed, k)
                assert out == wout, (seed, k)
                if not ok:
                    break
        finally:
            oracle.decoder_free(odec)
            oracle.cache_free(cache)


def test_backref_empty_window_is_an_error():
    """A BACKREF before any declare names an empty slot: decode() is false."""
    from wanproxy_amd.xcgpu import Context
    ctx = Context(0)
    outs, st, cons, _ = ctx.decode_chunks([b'abc\xf1\x03\x07tail', b'next'])
    assert int(st[0]) == -1 and int(cons[0]) == 6 and outs[0] == b'abc'
    assert int(st[1]) == 2
