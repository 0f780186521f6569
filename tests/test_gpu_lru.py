"""GPU parity for the bounded cache: XCodecMemoryCache(uuid, limit) with LRU
eviction (xcodec/xcodec_cache.h:277-364, xcodec/xcodec_lru.h), stream
semantics, against the reference-made fixtures of tests/golden/lru.json and
the oracle's LRU restatement (tests/test_lru_oracle.py pins it)."""
import hashlib

import numpy as np
import pytest

from oracle.lib import MODE_STREAM
from test_lru_oracle import lru_golden, lru_inputs, mlg  # noqa: F401  (fixture)

pytestmark = pytest.mark.gpu
SEG = 2048


def sha(b):
    return hashlib.sha256(b).hexdigest()


def gpu_stream(d, offs, lens, limit, steps=None):
    from wanproxy_amd.xcgpu import XCG_SEM_STREAM, Context
    ctx = Context(0, memory_cache_limit=limit)
    try:
        if steps is None:
            outs = ctx.encode_chunks(d, offs, lens, semantics=XCG_SEM_STREAM)
        else:
            outs, i, k = [], 0, 0
            while i < len(offs):
                m = steps[k % len(steps)]
                outs += ctx.encode_chunks(d, offs[i:i + m], lens[i:i + m], semantics=XCG_SEM_STREAM)
                i += m
                k += 1
        return outs, ctx.cache_size()
    finally:
        ctx.close()


def oracle_stream(oracle, d, offs, lens, limit):
    c = oracle.cache_new(limit)
    outs = oracle.encode_batch(d, offs, lens, mode=MODE_STREAM, cache=c)
    size = oracle.lib.xco_cache_size(c)
    oracle.cache_free(c)
    return outs, size


def test_lru_golden_gpu(lru_golden, stream_seed):  # noqa: F811
    from wanproxy_amd.synth import chunks_of
    from wanproxy_amd.xcgpu import XCGError
    ran = 0
    for case in lru_golden['cases']:
        d = lru_inputs(case['input'])
        offs, lens = chunks_of(d, case['chunk'])
        segs = max(1, case['limit'] // SEG)
        key = (case['input'], case['chunk'], case['limit'])
        try:
            outs, _ = gpu_stream(d, offs, lens, case['limit'])
        except XCGError:
            # refused loudly only where one chunk's own references can exceed the limit
            assert segs < 2 * (case['chunk'] // SEG + 1), key
            continue
        assert [len(o) for o in outs] == case['lens'], key
        assert [sha(o)[:32] for o in outs] == case['chunk_sha256'], key
        ran += 1
    assert ran >= 6


@pytest.mark.parametrize('limit_segs,chunk', [(100, 4096), (333, 65536), (1000, 65536), (300, 131072),
                                              (5000, 65536), (150, 32768)])
def test_lru_random_vs_oracle(oracle, stream_seed, limit_segs, chunk):
    from wanproxy_amd.synth import chunks_of
    d = mlg.recency_stream(7000 + limit_segs, 4 << 20, 55, 2 * limit_segs)
    offs, lens = chunks_of(d, chunk)
    exp, esize = oracle_stream(oracle, d, offs, lens, limit_segs * SEG)
    got, gsize = gpu_stream(d, offs, lens, limit_segs * SEG)
    bad = [i for i in range(len(exp)) if got[i] != exp[i]]
    assert not bad, (limit_segs, chunk, bad[:8])
    assert gsize == esize


def test_lru_split_batches(oracle):
    # The cache (and its LRU order) persists across calls.
    from wanproxy_amd.synth import chunks_of
    d = mlg.recency_stream(4242, 3 << 20, 60, 500)
    offs, lens = chunks_of(d, 65536)
    exp, _ = oracle_stream(oracle, d, offs, lens, 200 * SEG)
    got, _ = gpu_stream(d, offs, lens, 200 * SEG, steps=(1, 5, 2, 11, 3))
    assert got == exp


def test_lru_cache_clear_restarts(oracle):
    # Clearing the bounded cache starts a fresh LRU (the same stream encodes the same).
    from wanproxy_amd.synth import chunks_of
    from wanproxy_amd.xcgpu import XCG_SEM_STREAM, Context
    d = mlg.recency_stream(99, 2 << 20, 60, 300)
    offs, lens = chunks_of(d, 65536)
    exp, _ = oracle_stream(oracle, d, offs, lens, 150 * SEG)
    ctx = Context(0, memory_cache_limit=150 * SEG)
    for _ in range(3):
        ctx.cache_clear()
        assert ctx.encode_chunks(d, offs, lens, semantics=XCG_SEM_STREAM) == exp
    ctx.close()


def test_lru_uniform_and_magic(oracle, stream_seed):
    from wanproxy_amd import synth
    for seed, dup, magic, limit in ((11, 50, 0, 128), (12, 70, 3, 257), (13, 90, 0, 700)):
        d = synth.stream(seed, 3 << 20, dup, magic)
        offs, lens = synth.chunks_of(d, 65536)
        exp, _ = oracle_stream(oracle, d, offs, lens, limit * SEG)
        got, _ = gpu_stream(d, offs, lens, limit * SEG)
        assert got == exp, (seed, limit)


def test_lru_no_eviction_equals_unbounded(oracle):
    # A limit the stream never reaches gives the unbounded encoding.
    from wanproxy_amd import synth
    d = synth.stream(0xC2, 2 << 20, 50, 0)
    offs, lens = synth.chunks_of(d, 65536)
    got, size = gpu_stream(d, offs, lens, 1 << 30)
    c = oracle.cache_new()
    assert got == oracle.encode_batch(d, offs, lens, mode=MODE_STREAM, cache=c)
    assert size == oracle.lib.xco_cache_size(c)
    oracle.cache_free(c)


def test_lru_unsupported_paths():
    from wanproxy_amd.xcgpu import Context, XCGError
    ctx = Context(0, memory_cache_limit=64 * SEG)
    with pytest.raises(XCGError):
        ctx.decode_chunks([b'\xf1\x00'])
    # independent chunks of more than limit * 2048 bytes could evict
    x = np.random.default_rng(1).integers(0, 256, 65 * SEG, dtype=np.uint8).tobytes()
    with pytest.raises(XCGError):
        ctx.encode_chunks(x, [0], [len(x)])
    ctx.close()
