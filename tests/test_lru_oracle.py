"""The oracle's bounded XCodecMemoryCache (LRU eviction, xcodec/xcodec_cache.h:
303-364 + xcodec/xcodec_lru.h) pinned against the reference: fixtures made by
tests/golden/make_lru_golden.py from the real reference classes, and a direct
comparison with oracle/_ref when it is built."""
import hashlib
import importlib.util
import json
import os

import numpy as np
import pytest

from oracle.lib import MODE_STREAM

HERE = os.path.dirname(os.path.abspath(__file__))
_spec = importlib.util.spec_from_file_location('make_lru_golden', os.path.join(HERE, 'golden/make_lru_golden.py'))
mlg = importlib.util.module_from_spec(_spec)
_spec.loader.exec_module(mlg)


def sha(b):
    return hashlib.sha256(b).hexdigest()


@pytest.fixture(scope='module')
def lru_golden():
    with open(os.path.join(HERE, 'golden/lru.json')) as f:
        return json.load(f)


def lru_inputs(name, _memo={}):
    if name not in _memo:
        _memo[name] = mlg.inputs(name)
    return _memo[name]


def test_lru_inputs_pinned(lru_golden):
    for name, meta in lru_golden['inputs'].items():
        d = lru_inputs(name)
        assert (len(d), sha(d)) == (meta['len'], meta['sha256']), name


def test_lru_encode_golden(lru_golden, oracle):
    from wanproxy_amd.synth import chunks_of
    for case in lru_golden['cases']:
        d = lru_inputs(case['input'])
        offs, lens = chunks_of(d, case['chunk'])
        c = oracle.cache_new(case['limit'])
        outs = oracle.encode_batch(d, offs, lens, mode=MODE_STREAM, cache=c)
        size = oracle.lib.xco_cache_size(c)
        oracle.cache_free(c)
        key = (case['input'], case['chunk'], case['limit'])
        assert [len(o) for o in outs] == case['lens'], key
        assert [sha(o)[:32] for o in outs] == case['chunk_sha256'], key
        assert size <= max(1, case['limit'] // 2048), key


def test_lru_decode_golden(lru_golden, oracle):
    from wanproxy_amd.synth import chunks_of
    for case in lru_golden['cases']:
        d = lru_inputs(case['input'])
        offs, lens = chunks_of(d, case['chunk'])
        c = oracle.cache_new(case['limit'])
        encs = oracle.encode_batch(d, offs, lens, mode=MODE_STREAM, cache=c)
        oracle.cache_free(c)
        dc = oracle.cache_new(case['limit'])
        dec = oracle.decoder_new(dc)
        for i, exp in enumerate(case['dec']):
            ok, o, cons, unk = oracle.decode(encs[i], dc, decoder=dec)
            got = {'ok': ok, 'consumed': cons, 'nunknown': len(unk), 'out_len': len(o), 'out_sha256': sha(o)}
            assert got == exp, (case['input'], case['chunk'], case['limit'], i)
        oracle.decoder_free(dec)
        oracle.cache_free(dc)


def test_lru_export_order(oracle):
    # Export lists entries least recently used first; a lookup hit refreshes.
    import ctypes as C
    rng = np.random.default_rng(3)
    segs = [rng.integers(0, 256, 2048, dtype=np.uint8) for _ in range(5)]
    c = oracle.cache_new(4 * 2048)
    L = oracle.lib
    L.xco_cache_lookup.restype = C.c_void_p
    L.xco_cache_lookup.argtypes = [C.c_void_p, C.c_uint64]
    for i in range(4):
        assert L.xco_cache_enter(c, 100 + i, segs[i].ctypes.data_as(C.POINTER(C.c_uint8))) == 0
    assert L.xco_cache_lookup(c, 100) is not None          # 100 becomes most recent
    assert L.xco_cache_enter(c, 104, segs[4].ctypes.data_as(C.POINTER(C.c_uint8))) == 0   # evicts 101
    keys = np.zeros(8, dtype=np.uint64)
    n = L.xco_cache_export(c, keys.ctypes.data_as(C.POINTER(C.c_uint64)), None, 8)
    assert list(keys[:n]) == [102, 103, 100, 104]
    assert L.xco_cache_lookup(c, 101) is None
    oracle.cache_free(c)


@pytest.mark.parametrize('limit_segs', [1, 5, 64, 333])
def test_lru_vs_reference_random(oracle, ref_oracle, limit_segs):
    from wanproxy_amd.synth import chunks_of
    d = mlg.recency_stream(1000 + limit_segs, 1 << 20, 55, 400)
    for chunk in (8192, 65536):
        offs, lens = chunks_of(d, chunk)
        outs = []
        for o in (oracle, ref_oracle):
            c = o.cache_new(limit_segs * 2048)
            outs.append(o.encode_batch(d, offs, lens, mode=MODE_STREAM, cache=c))
            o.cache_free(c)
        assert outs[0] == outs[1], (limit_segs, chunk)
