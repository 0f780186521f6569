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
    # independent chunks of more than limit * 2048 bytes could evict
    x = np.random.default_rng(1).integers(0, 256, 65 * SEG, dtype=np.uint8).tobytes()
    with pytest.raises(XCGError):
        ctx.encode_chunks(x, [0], [len(x)])
    ctx.close()


def decode_calls(ctx, encs):
    """One decode() call per encoded chunk on ctx (a persistent decoder), as
    the reference harness made tests/golden/lru.json's 'dec' entries."""
    calls = []
    for e in encs:
        outs, st, cons, unk = ctx.decode_chunks([e])
        calls.append({'ok': int(st[0]) != -1, 'consumed': int(cons[0]), 'nunknown': len(unk),
                      'out_len': len(outs[0]), 'out_sha256': sha(outs[0])})
        if int(st[0]) == -1 or unk:
            break
    return calls


def test_lru_decode_golden_gpu(lru_golden, oracle):  # noqa: F811
    # The reference XCodecDecoder on a bounded cache, call by call (incl. the
    # collision case where the decoder's LRU falls out of step and blocks).
    from wanproxy_amd.synth import chunks_of
    from wanproxy_amd.xcgpu import Context, XCGError
    ran = 0
    for case in lru_golden['cases']:
        d = lru_inputs(case['input'])
        offs, lens = chunks_of(d, case['chunk'])
        encs, _ = oracle_stream(oracle, d, offs, lens, case['limit'])
        ctx = Context(0, memory_cache_limit=case['limit'])
        key = (case['input'], case['chunk'], case['limit'])
        try:
            got = decode_calls(ctx, encs)
        except XCGError:
            assert max(1, case['limit'] // SEG) < 2 * (case['chunk'] // SEG + 1), key
            continue
        finally:
            ctx.close()
        assert got == case['dec'], key
        ran += 1
    assert ran >= 6


def test_lru_decode_batch_vs_oracle(oracle):
    # A whole stream in one decode batch on a bounded cache, then more calls.
    from wanproxy_amd.synth import chunks_of
    from wanproxy_amd.xcgpu import Context
    d = mlg.recency_stream(515, 3 << 20, 60, 600)
    offs, lens = chunks_of(d, 65536)
    limit = 1500 * SEG
    encs, _ = oracle_stream(oracle, d, offs, lens, limit)
    ctx = Context(0, memory_cache_limit=limit)
    half = len(encs) // 2
    outs, st, cons, unk = ctx.decode_chunks(encs[:half])
    assert (st == 0).all() and not unk
    outs2, st2, _, unk2 = ctx.decode_chunks(encs[half:])
    assert (st2 == 0).all() and not unk2
    assert b''.join(outs + outs2) == d
    # cache state: the oracle decoder's cache after the same calls
    dc = oracle.cache_new(limit)
    dec = oracle.decoder_new(dc)
    for e in encs:
        oracle.decode(e, dc, decoder=dec)
    assert ctx.cache_size() == oracle.lib.xco_cache_size(dc)
    oracle.decoder_free(dec)
    oracle.cache_free(dc)
    ctx.close()


def test_lru_round_trip_gpu(oracle):
    # GPU bounded encode -> GPU bounded decode (same limit) gives the input back.
    from wanproxy_amd import synth
    from wanproxy_amd.xcgpu import Context
    d = synth.stream(0x1A9, 4 << 20, 40, 1)
    offs, lens = synth.chunks_of(d, 65536)
    got, _ = gpu_stream(d, offs, lens, 400 * SEG)
    ctx = Context(0, memory_cache_limit=400 * SEG)
    out = []
    for i in range(0, len(got), 8):
        o, st, _, unk = ctx.decode_chunks(got[i:i + 8])
        assert (st == 0).all() and not unk
        out += o
    ctx.close()
    assert b''.join(out) == d


@pytest.mark.parametrize('batch', [1, 4])
def test_lru_decode_blocks_like_reference(oracle, batch):
    # Frames from an UNBOUNDED encoder reference segments a bounded decoder has
    # evicted: decode() blocks there with the skim's unknown set (ASK), exactly
    # where the oracle's bounded XCodecDecoder does.
    from wanproxy_amd.synth import chunks_of
    from wanproxy_amd.xcgpu import Context
    d = mlg.recency_stream(808, 2 << 20, 60, 2000)
    offs, lens = chunks_of(d, 32768)
    c = oracle.cache_new()
    encs = oracle.encode_batch(d, offs, lens, mode=MODE_STREAM, cache=c)
    oracle.cache_free(c)
    limit = 120 * SEG
    dc = oracle.cache_new(limit)
    dec = oracle.decoder_new(dc)
    ctx = Context(0, memory_cache_limit=limit)
    blocked = False
    for i in range(0, len(encs), batch):
        part = encs[i:i + batch]
        outs, st, cons, unk = ctx.decode_chunks(part)
        exp_out, exp_unk = [], []
        for j, e in enumerate(part):
            ok, o, cn, u = oracle.decode(e, dc, decoder=dec)
            exp_out.append(o)
            if u:
                # (the batch decoder's skim also covers the frames after this one in its batch)
                exp_unk = u
                assert int(st[j]) == 1 and int(cons[j]) == cn, (i, j)
                assert outs[j] == o
                blocked = True
                break
            assert int(st[j]) == 0 and outs[j] == o and int(cons[j]) == cn, (i, j)
        if blocked:
            assert set(exp_unk) <= set(unk)
            break
    assert blocked
    oracle.decoder_free(dec)
    oracle.cache_free(dc)
    ctx.close()


def test_lru_host_ops_vs_oracle(oracle):
    # Single-segment lookups / enters (XCodecPipePair's <LEARN>: lookup, then
    # replace or enter) on a bounded cache, against the oracle's LRU.
    import ctypes as C
    from wanproxy_amd.xcgpu import Context
    rng = np.random.default_rng(21)
    L = oracle.lib
    L.xco_cache_lookup.restype = C.c_void_p
    L.xco_cache_lookup.argtypes = [C.c_void_p, C.c_uint64]
    L.xco_cache_replace.argtypes = [C.c_void_p, C.c_uint64, C.POINTER(C.c_uint8)]
    u8 = lambda b: (C.c_uint8 * 2048).from_buffer_copy(b)
    keys = [int(rng.integers(0, 1 << 62)) & ~(0xF << 32) for _ in range(40)]
    segs = {k: rng.integers(0, 256, 2048, dtype=np.uint8).tobytes() for k in keys}
    limit = 9
    oc = oracle.cache_new(limit * SEG)
    ctx = Context(0, memory_cache_limit=limit * SEG)

    def o_lookup(k):
        p = L.xco_cache_lookup(oc, k)
        return None if p is None else C.string_at(p, 2048)

    def o_learn(k, b):
        old = o_lookup(k)
        if old is None:
            assert L.xco_cache_enter(oc, k, u8(b)) == 0
        elif old != b:
            L.xco_cache_replace(oc, k, u8(b))

    for step in range(300):
        k = keys[int(rng.integers(0, 20 if step < 150 else 40))]
        if rng.random() < 0.5:
            b = segs[k] if rng.random() < 0.8 else rng.integers(0, 256, 2048, dtype=np.uint8).tobytes()
            o_learn(k, b)
            ctx.cache_enter(k, b)
        else:
            assert ctx.cache_lookup(k) == o_lookup(k), step
        assert ctx.cache_size() == L.xco_cache_size(oc), step
    for k in keys:                                   # final contents (lookups refresh both alike)
        assert ctx.cache_lookup(k) == o_lookup(k)
    ctx.close()
    oracle.cache_free(oc)


def test_lru_out_of_band(oracle):
    # Out-of-band declarations (F1 02 BE64, XCodecCache::out_of_band()) on a
    # bounded cache: the eviction order is the same, only the output form differs.
    from wanproxy_amd.synth import chunks_of
    from wanproxy_amd.xcgpu import XCG_SEM_STREAM, Context
    d = mlg.recency_stream(616, 2 << 20, 60, 400)
    offs, lens = chunks_of(d, 65536)
    limit = 180 * SEG
    c = oracle.cache_new(limit)
    exp = oracle.encode_batch(d, offs, lens, mode=MODE_STREAM, oob=True, cache=c)
    oracle.cache_free(c)
    ctx = Context(0, out_of_band=True, memory_cache_limit=limit)
    got = ctx.encode_chunks(d, offs, lens, semantics=XCG_SEM_STREAM)
    ctx.close()
    assert got == exp


def test_lru_fuzz(oracle):
    # Random limits, chunkings, data shapes and call splits against the oracle.
    from wanproxy_amd import synth
    from wanproxy_amd.xcgpu import XCG_SEM_STREAM, Context
    rng = np.random.default_rng(2024)
    for case in range(16):
        kind = case % 3
        nbytes = int(rng.integers(1 << 19, 3 << 20))
        if kind == 0:
            d = mlg.recency_stream(int(rng.integers(1 << 30)), nbytes, int(rng.integers(30, 90)),
                                   int(rng.integers(50, 3000)))
        elif kind == 1:
            d = synth.stream(int(rng.integers(1 << 30)), nbytes, int(rng.integers(10, 90)), int(rng.integers(0, 4)))
        else:   # runs and repeats of a short period: many collisions between nearby windows
            pat = rng.integers(0, 256, int(rng.integers(100, 5000)), dtype=np.uint8).tobytes()
            d = (pat * (nbytes // len(pat) + 1))[:nbytes]
            d = bytearray(d)
            for _ in range(200):
                d[int(rng.integers(0, nbytes))] = int(rng.integers(0, 256))
            d = bytes(d)
        chunk = int(rng.choice([4096, 20000, 65536, 131072]))
        offs, lens = synth.chunks_of(d, chunk)
        limit = int(rng.integers(2 * (chunk // SEG + 1) + 8, 3000)) * SEG
        exp, esize = oracle_stream(oracle, d, offs, lens, limit)
        ctx = Context(0, memory_cache_limit=limit)
        got, i = [], 0
        while i < len(offs):
            m = int(rng.integers(1, 40))
            got += ctx.encode_chunks(d, offs[i:i + m], lens[i:i + m], semantics=XCG_SEM_STREAM)
            i += m
        gsize = ctx.cache_size()
        ctx.close()
        bad = [k for k in range(len(exp)) if got[k] != exp[k]]
        assert not bad and gsize == esize, (case, kind, chunk, limit // SEG, bad[:5])


def test_lru_short_chunks_between_calls(oracle):
    # A chunk shorter than one segment makes no cache reference; its (scratch)
    # reference list must not keep an earlier call's entries.
    from wanproxy_amd.synth import chunks_of
    from wanproxy_amd.xcgpu import XCG_SEM_STREAM, Context
    d = mlg.recency_stream(77, 600_000, 50, 300)
    offs, lens = chunks_of(d, 4096)
    offs, lens = list(offs), list(lens)
    # splice in short chunks: every 5th chunk cut to 100 bytes + remainder
    o2, l2 = [], []
    for k, (a, n) in enumerate(zip(offs, lens)):
        if k % 5 == 3 and n > 100:
            o2 += [a, a + 100]
            l2 += [100, n - 100]
        else:
            o2.append(a)
            l2.append(n)
    o2, l2 = np.array(o2, np.uint64), np.array(l2, np.uint32)
    limit = 400 * SEG
    exp, esize = oracle_stream(oracle, d, o2, l2, limit)
    ctx = Context(0, memory_cache_limit=limit)
    got, i = [], 0
    for m in [7, 3, 11, 2, 9] * 200:
        if i >= len(o2):
            break
        got += ctx.encode_chunks(d, o2[i:i + m], l2[i:i + m], semantics=XCG_SEM_STREAM)
        i += m
    assert got == exp and ctx.cache_size() == esize
    ctx.close()


def test_lru_decode_fuzz(oracle):
    # Bounded decoders (GPU and oracle, same limit as the encoder) over random
    # call splits: same output, same cache size after every call.
    from wanproxy_amd import synth
    from wanproxy_amd.xcgpu import Context
    rng = np.random.default_rng(77)
    for case in range(8):
        nbytes = int(rng.integers(1 << 19, 2 << 20))
        if case % 2:
            d = mlg.recency_stream(int(rng.integers(1 << 30)), nbytes, int(rng.integers(30, 90)),
                                   int(rng.integers(50, 2000)))
        else:
            d = synth.stream(int(rng.integers(1 << 30)), nbytes, int(rng.integers(10, 90)), int(rng.integers(0, 3)))
        chunk = int(rng.choice([4096, 30000, 65536]))
        offs, lens = synth.chunks_of(d, chunk)
        limit = int(rng.integers(2 * (chunk // SEG + 1) + 8, 1500)) * SEG
        encs, _ = oracle_stream(oracle, d, offs, lens, limit)
        dc = oracle.cache_new(limit)
        dec = oracle.decoder_new(dc)
        ctx = Context(0, memory_cache_limit=limit)
        i = 0
        while i < len(encs):
            m = int(rng.integers(1, 12))
            part = encs[i:i + m]
            outs, st, _, unk = ctx.decode_chunks(part)
            exp = [oracle.decode(e, dc, decoder=dec)[1] for e in part]
            assert (st == 0).all() and not unk and outs == exp, (case, i)
            assert ctx.cache_size() == oracle.lib.xco_cache_size(dc), (case, i)
            i += m
        ctx.close()
        oracle.decoder_free(dec)
        oracle.cache_free(dc)
