"""GPU parity for stream semantics (XCG_SEM_STREAM): chunks of one stream share
one persistent GPU cache, exactly as successive XCodecEncoder::encode calls
share their XCodecMemoryCache (programs/tack/tack.cc:301-321)."""
import numpy as np
import pytest

from golden_cases import chunks, data, sha

pytestmark = pytest.mark.gpu


@pytest.fixture(scope='module')
def sctx():
    from wanproxy_amd.xcgpu import Context
    c = Context(0, cache_segments=1 << 18)
    yield c
    c.close()


def enc_stream(ctx, d, offs, lens):
    from wanproxy_amd.xcgpu import XCG_SEM_STREAM
    return ctx.encode_chunks(d, offs, lens, semantics=XCG_SEM_STREAM)


def test_golden_stream(sctx, golden, stream_seed):
    n = 0
    for case in golden['cases']:
        if case['mode'] != 'stream':
            continue
        d, (offs, lens) = chunks(case)
        sctx.cache_clear()
        outs = enc_stream(sctx, d, offs, lens)
        assert [len(o) for o in outs] == case['lens'], (case['input'], case['chunk'], sctx.last_rounds())
        assert [sha(o)[:32] for o in outs] == case['chunk_sha256'], (case['input'], case['chunk'])
        n += 1
    assert n >= 10


def test_baseline_kats_stream(sctx, golden, stream_seed):
    # BASELINE.md "KAT": tack -c over the whole file (64 KiB encode() calls).
    from wanproxy_amd.synth import chunks_of
    for name, b in golden['baseline'].items():
        d = data(name)
        offs, lens = chunks_of(d, 65536)
        sctx.cache_clear()
        whole = b''.join(enc_stream(sctx, d, offs, lens))
        assert (len(whole), sha(whole)) == (b['xc_len'], b['xc']), name


def test_stream_split_batches(sctx, oracle, stream_seed):
    # The cache persists across calls: one stream fed in batches of 1..64
    # chunks encodes exactly like one batch / the sequential oracle.
    from wanproxy_amd.synth import chunks_of
    d = data('c2_small')
    offs, lens = chunks_of(d, 65536)
    exp = oracle.encode_batch(d, offs, lens, mode=1)
    sctx.cache_clear()
    got, i = [], 0
    for step in (1, 3, 7, 1, 20, 32):
        got += enc_stream(sctx, d, offs[i:i + step], lens[i:i + step])
        i += step
    assert i == len(offs)
    assert got == exp
    assert sctx.cache_size() > 0


def test_stream_random_vs_oracle(sctx, oracle, stream_seed):
    rng = np.random.default_rng(77)
    blocks = [rng.integers(0, 256, size=2048, dtype=np.uint8) for _ in range(40)]
    parts = []
    for i in range(400):
        k = rng.random()
        if k < 0.4:
            parts.append(blocks[int(rng.integers(0, len(blocks)))])
        elif k < 0.6:   # unaligned slice of a known block pair
            a = np.concatenate([blocks[int(rng.integers(0, 40))], blocks[int(rng.integers(0, 40))]])
            o = int(rng.integers(1, 2048))
            parts.append(a[o:o + int(rng.integers(100, 3000))])
        elif k < 0.7:
            parts.append(np.full(int(rng.integers(1, 5000)), int(rng.integers(0, 256)), np.uint8))
        else:
            parts.append(rng.integers(0, 256, size=int(rng.integers(1, 4000)), dtype=np.uint8))
    d = np.concatenate(parts).tobytes()
    for csize in (4096, 65536, 100000):
        from wanproxy_amd.synth import chunks_of
        offs, lens = chunks_of(d, csize)
        exp = oracle.encode_batch(d, offs, lens, mode=1)
        sctx.cache_clear()
        got = enc_stream(sctx, d, offs, lens)
        bad = [i for i in range(len(exp)) if got[i] != exp[i]]
        assert not bad, (csize, bad[:10], sctx.last_rounds())


def test_encoder_mirror_tack_loop(oracle):
    # XCodecEncoder mirror: one encode() call per 64 KiB read, like tack -c.
    from wanproxy_amd.xcgpu import Context, XCodecEncoder
    ctx = Context(0, cache_segments=1 << 16)
    enc = XCodecEncoder(ctx)
    d = data('kat_b')
    out = b''.join(enc.encode(d[i:i + 65536]) for i in range(0, len(d), 65536))
    ctx.close()
    assert out == oracle.encode_stream(d)
