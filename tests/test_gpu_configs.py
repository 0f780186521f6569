"""GPU parity on scaled-down versions of BASELINE.json's stream configurations
(SURVEY.md 8d C3, C4, C5), bit-exact against the CPU oracle run with the same
sequential XCodecEncoder semantics over the whole input, and decoded back.

Each runs with every lane-filter mode of the stream encoder forced (the 64 KiB
LDS filter; the LDS filter in front of the global L2-resident one, used above
~220 k keys; the global filter alone, above ~700 k), so the large-cache paths
are covered at sizes the oracle finishes in seconds.
"""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu

KiB, MiB = 1024, 1 << 20
# (LDS filter threshold, LDS-prefilter threshold) in keys
MODES = {'lds': (1 << 30, 1 << 30), 'prefilter': (0, 1 << 30), 'global': (0, 0)}


@pytest.fixture(params=sorted(MODES))
def filter_mode(request):
    from wanproxy_amd.xcgpu import lib
    old = lib().xcg_debug_set_lds_filter_keys(MODES[request.param][0])
    oldp = lib().xcg_debug_set_lds_prefilter_keys(MODES[request.param][1])
    yield request.param
    lib().xcg_debug_set_lds_filter_keys(old)
    lib().xcg_debug_set_lds_prefilter_keys(oldp)


def encode_in_batches(ctx, data, offs, lens, per):
    from wanproxy_amd.xcgpu import XCG_SEM_STREAM
    out = []
    for a in range(0, len(offs), per):
        out += ctx.encode_chunks(data, offs[a:a + per], lens[a:a + per], semantics=XCG_SEM_STREAM)
    return out


def first_diff(got, exp):
    return next((i for i in range(len(exp)) if got[i] != exp[i]), None)


def test_c3_warm_shared_cache(filter_mode, stream_seed, oracle):
    """C3: streams interleaved round-robin at 64 KiB, one shared cache; warm-up
    encode then the same data again against the warm cache (nearly all REF)."""
    from wanproxy_amd import synth
    from wanproxy_amd.xcgpu import Context
    nstreams, per_stream = 8, 1 * MiB
    streams = [np.frombuffer(synth.stream(100 + i, per_stream, 5, 0), np.uint8) for i in range(nstreams)]
    cps = per_stream // (64 * KiB)
    data = np.concatenate([streams[s][c * 64 * KiB:(c + 1) * 64 * KiB] for c in range(cps) for s in range(nstreams)])
    n = nstreams * cps
    offs = np.arange(n, dtype=np.uint64) * (64 * KiB)
    lens = np.full(n, 64 * KiB, np.uint32)
    cache = oracle.cache_new()
    try:
        exp_warm = oracle.encode_batch(data, offs, lens, mode=1, cache=cache)
        exp_hot = oracle.encode_batch(data, offs, lens, mode=1, cache=cache)
    finally:
        oracle.cache_free(cache)
    ctx = Context(0, cache_segments=1 << 16)
    warm = encode_in_batches(ctx, data, offs, lens, 32)
    assert first_diff(warm, exp_warm) is None, filter_mode
    hot = encode_in_batches(ctx, data, offs, lens, 32)
    assert first_diff(hot, exp_hot) is None, filter_mode
    assert sum(map(len, hot)) < data.size // 50          # warm: (almost) all REFs
    ctx.close()
    dctx = Context(0, cache_segments=1 << 16)
    outs, st, _, unk = dctx.decode_chunks(warm + hot)
    assert (st == 0).all() and not unk
    assert b''.join(outs) == data.tobytes() * 2
    dctx.close()


def test_c4_small_packets(filter_mode, stream_seed, oracle):
    """C4: 4 KiB packets, each one encode() call, one cache per shard."""
    from wanproxy_amd import synth
    from wanproxy_amd.xcgpu import Context
    n = 4096
    data = synth.stream(0xC4, n * 4 * KiB, 4, 0)
    offs, lens = synth.chunks_of(data, 4 * KiB)
    exp = oracle.encode_batch(data, offs, lens, mode=1)
    ctx = Context(0, cache_segments=1 << 14)
    got = encode_in_batches(ctx, data, offs, lens, 1024)
    assert first_diff(got, exp) is None, filter_mode
    ctx.close()


def test_c5_large_chunks_cold_cache(filter_mode, stream_seed, oracle):
    """C5: 128 KiB chunks, cold unbounded cache growing across batches."""
    from wanproxy_amd import synth
    from wanproxy_amd.xcgpu import Context
    data = synth.stream(0xC5, 16 * MiB, 20, 0)
    offs, lens = synth.chunks_of(data, 128 * KiB)
    exp = oracle.encode_batch(data, offs, lens, mode=1)
    ctx = Context(0, cache_segments=1 << 14)
    got = encode_in_batches(ctx, data, offs, lens, 32)
    assert first_diff(got, exp) is None, filter_mode
    assert ctx.cache_size() > 0
    ctx.close()


def test_mixed_alphabet_global_filter(filter_mode, stream_seed, oracle):
    """Collision-prone and 0xF1-heavy data through both filter modes."""
    from wanproxy_amd.synth import chunks_of
    from wanproxy_amd.xcgpu import Context
    rng = np.random.default_rng(5)
    blocks = [rng.choice(np.array([1, 3, 0xF1, 0xF3], np.uint8), size=2048) for _ in range(24)]
    parts = []
    for _ in range(300):
        b = blocks[int(rng.integers(0, len(blocks)))]
        o = int(rng.integers(0, 2048))
        parts.append(np.concatenate([b, b])[o:o + int(rng.integers(500, 4096))])
    d = np.concatenate(parts).tobytes()
    offs, lens = chunks_of(d, 16 * KiB)
    exp = oracle.encode_batch(d, offs, lens, mode=1)
    ctx = Context(0, cache_segments=1 << 14)
    got = encode_in_batches(ctx, d, offs, lens, 16)
    assert first_diff(got, exp) is None, filter_mode
    ctx.close()
