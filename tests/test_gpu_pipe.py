"""XCodecPipePair protocol layer over the GPU engine (xcg_pipe_*): framing
against the oracle restatement (oracle/pipe.py), encoder -> decoder round
trips with <ADVANCE>, the <ASK>/<LEARN> exchange, <EOS>/<EOS_ACK>, batched
multi-pipe encoding, and the decoder_error() cases (xcodec/xcodec_pipe_pair.cc)."""
import numpy as np
import pytest

from golden_cases import data

pytestmark = pytest.mark.gpu

UUID_A = b'0d1f4c8e-95a3-4b2d-8f6e-3c7a9b1d2e4f'
UUID_B = b'a7c3e9f1-2b4d-4e6f-8a0c-1e3f5a7c9e0b'


@pytest.fixture
def ctxs():
    from wanproxy_amd.xcgpu import Context
    cs = [Context(0, cache_segments=1 << 15) for _ in range(2)]
    yield cs
    for c in cs:
        c.close()


def payload(seed=3, n=1_700_000):
    rng = np.random.default_rng(seed)
    blocks = [rng.integers(0, 256, 2048, dtype=np.uint8).tobytes() for _ in range(200)]
    out = bytearray()
    while len(out) < n:
        b = blocks[int(rng.integers(0, len(blocks)))]
        out += b if rng.random() < 0.7 else rng.integers(0, 256, int(rng.integers(1, 3000)), dtype=np.uint8).tobytes()
    return bytes(out[:n])


def test_framing_vs_oracle(ctxs, oracle):
    from oracle.pipe import encoder_stream
    from wanproxy_amd.xcgpu import PipePair
    enc, dec = ctxs
    a = PipePair(enc, dec, UUID_A)
    consumes = [data('kat_a'), payload(), b'x' * 100, data('kat_b')[:70000], b'']
    got = b''.join(a.encoder_consume(c) for c in consumes)
    cache = oracle.cache_new()
    try:
        exp = encoder_stream(oracle, cache, UUID_A, consumes)
    finally:
        oracle.cache_free(cache)
    assert got == exp
    assert a.pending_frames() == 2 + 4 + 1 + 1


def test_roundtrip_advance_eos(ctxs):
    from wanproxy_amd.xcgpu import Context, PipePair
    enc, _ = ctxs
    benc, bdec = Context(0, cache_segments=1 << 15), Context(0, cache_segments=1 << 15)
    a = PipePair(enc, ctxs[1], UUID_A)           # a's decoder side hears b's replies
    b = PipePair(benc, bdec, UUID_B)
    msgs = [payload(1), payload(2, 900_000), data('kat_c')]
    for m in msgs:
        wire = a.encoder_consume(m)
        to_a, local, leos, peos = b.decoder_consume(wire)
        assert local == m and not leos and not peos
        assert to_a[:1] == b'\x01'                   # <ADVANCE> for the frames decoded
        nframes = -(-len(m) // (512 * 1024))
        assert int.from_bytes(to_a[1:5], 'big') == nframes
        assert a.pending_frames() == nframes
        back, _, _, _ = a.decoder_consume(to_a)
        assert back == b'' and a.pending_frames() == 0
    # <EOS> -> <EOS_ACK>, local EOS on b; a hears the ack
    wire = a.encoder_consume(b'')
    assert wire == b'\xfc'
    to_a, local, leos, peos = b.decoder_consume(wire)
    assert (to_a, local, leos, peos) == (b'\xfb', b'', True, False)
    back, local, leos, peos = a.decoder_consume(to_a)
    assert (back, local, leos, peos) == (b'', b'', False, False)
    benc.close()
    bdec.close()


def test_ask_learn(ctxs):
    """A decoder whose cache lost segments asks; the encoder answers from the
    frames it still holds (encoder_reference_frames_); decoding resumes."""
    from wanproxy_amd.xcgpu import Context, PipePair
    enc, adec = ctxs
    bdec = Context(0, cache_segments=1 << 15)
    a = PipePair(enc, adec, UUID_A)
    b = PipePair(Context(0, cache_segments=1 << 10), bdec, UUID_B)
    m = payload(9, 600_000)
    to_a, local, _, _ = b.decoder_consume(a.encoder_consume(m))
    assert local == m
    a.decoder_consume(to_a)                          # <ADVANCE>
    bdec.cache_clear()                               # b forgets every segment
    wire = a.encoder_consume(m)                      # now (almost) all REFs
    to_a, local, _, _ = b.decoder_consume(wire)
    assert b'\xf0' in to_a                           # <ASK>
    k = to_a.index(b'\xf0')
    count = int.from_bytes(to_a[k + 1:k + 3], 'big')
    assert count > 0
    learn, _, _, _ = a.decoder_consume(to_a)
    assert learn[:1] == b'\xf1' and int.from_bytes(learn[1:3], 'big') == count
    assert len(learn) == 3 + 2048 * count
    more, local2, _, _ = b.decoder_consume(learn)
    assert local + local2 == m
    bdec.close()


def test_encoder_consume_many_equals_sequential(ctxs, oracle):
    from wanproxy_amd.xcgpu import Context, PipePair
    enc, dec = ctxs
    uu = [UUID_A, UUID_B] * 2
    datas = [payload(20 + i, 300_000 + 170_000 * i) for i in range(4)]
    pipes = [PipePair(enc, dec, u) for u in uu]
    many = PipePair.encoder_consume_many(pipes, datas)
    enc2 = Context(0, cache_segments=1 << 15)
    pipes2 = [PipePair(enc2, dec, u) for u in uu]
    seq = [p.encoder_consume(d) for p, d in zip(pipes2, datas)]
    assert many == seq
    enc2.close()


@pytest.mark.parametrize('wire', [
    b'\x02\x00\x00\x00\x01x',                       # <FRAME> before <HELLO>
    b'\xff\x24' + UUID_B + b'\xff\x24' + UUID_B,    # <HELLO> twice
    b'\xff\x05hello',                               # bad <HELLO> length
    b'\xf0\x00\x01' + b'\x00' * 8,                  # <ASK> before we sent <HELLO>
    b'\xff\x24' + UUID_B + b'\xf1\x00\x01' + b'\x07' * 2048,   # <LEARN> nobody asked for
    b'\xff\x24' + UUID_B + b'\x02\x00\x00\x00\x00',            # zero-length frame
    b'\xfb',                                        # <EOS_ACK> before our <EOS>
    b'\x55',                                        # unsupported op
])
def test_decoder_errors(ctxs, wire):
    from wanproxy_amd.xcgpu import PipePair, XCGError
    p = PipePair(ctxs[0], ctxs[1], UUID_A)
    with pytest.raises(XCGError, match='protocol'):
        p.decoder_consume(wire)


def test_partial_ops_wait_for_more(ctxs):
    from wanproxy_amd.xcgpu import Context, PipePair
    a = PipePair(ctxs[0], ctxs[1], UUID_A)
    b = PipePair(Context(0, cache_segments=1 << 10), Context(0, cache_segments=1 << 15), UUID_B)
    m = payload(33, 200_000)
    wire = a.encoder_consume(m)
    got = b''
    for i in range(0, len(wire), 777):               # arbitrary TCP segmentation
        _, local, _, _ = b.decoder_consume(wire[i:i + 777])
        got += local
    assert got == m


def test_bounded_caches_like_wanproxy_conf(oracle):
    """wanproxy.conf's sized memory caches (LRU eviction) on both sides: the
    frames equal the oracle's with the same bounded cache, and the peer's
    bounded decoder cache stays in step (no <ASK>)."""
    from oracle.pipe import encoder_stream
    from wanproxy_amd.xcgpu import Context, PipePair
    limit = 600 * 2048
    enc, adec = Context(0, memory_cache_limit=limit), Context(0, memory_cache_limit=limit)
    benc, bdec = Context(0, memory_cache_limit=limit), Context(0, memory_cache_limit=limit)
    a = PipePair(enc, adec, UUID_A)
    b = PipePair(benc, bdec, UUID_B)
    # one frame per read (a decode call on a bounded cache holds at most its
    # limit in references); later messages repeat earlier ones, some of whose
    # segments the LRU has evicted by then
    msgs = [payload(40 + i % 7, 400_000 + 9_000 * i) for i in range(14)]
    wires = []
    for m in msgs:
        w = a.encoder_consume(m)
        wires.append(w)
        to_a, local, _, _ = b.decoder_consume(w)
        assert local == m and b'\xf0' not in to_a
        a.decoder_consume(to_a)
    cache = oracle.cache_new(limit)
    try:
        exp = encoder_stream(oracle, cache, UUID_A, msgs)
    finally:
        oracle.cache_free(cache)
    assert b''.join(wires) == exp
    assert enc.cache_size() == bdec.cache_size() <= 600
    for c in (enc, adec, benc, bdec):
        c.close()


UUID_C = b'5e2d8b4a-1c3f-4a6e-9b0d-7f1e3c5a8b2d'


@pytest.mark.parametrize('kind', ['unbounded', 'pair'])
def test_hello_connects_peer_cache_by_uuid(kind):
    """XCodecPipePair::decoder_decode on <HELLO>: decoder_cache_ =
    XCodecCache::connect(uuid, codec_->cache()) (xcodec/xcodec_pipe_pair.cc:
    182-203; xcodec/xcodec_cache.h:101-111).  Two connections from one peer
    (its UUID in both <HELLO>s) decode on ONE connected cache: the second
    connection's frames REF what only the first declared and decode without an
    <ASK>.  A peer with another UUID gets a cache of its own (the codec cache's
    connect: same kind and limit; a pair's is a new front on the same disk) and
    asks; its <LEARN> answers complete the decode."""
    from wanproxy_amd.xcgpu import Context, PipePair, connect_registry_clear, ctx_lookup
    connect_registry_clear()
    if kind == 'pair':
        codec = Context(0, memory_cache_limit=4 << 20, disk_bytes=(18 + 4 * 205) * 2048)
    else:
        codec = Context(0, cache_segments=1 << 15)
    lenc = Context(0, cache_segments=1 << 15)            # the local codec's encoder (unused direction)
    penc = Context(0, cache_segments=1 << 15)            # the peer codec's cache, shared by its connections
    pdec = Context(0, cache_segments=1 << 15)
    try:
        p1, p2, p3 = PipePair(penc, pdec, UUID_A), PipePair(penc, pdec, UUID_A), PipePair(penc, pdec, UUID_C)
        l1, l2, l3 = (PipePair(lenc, codec, UUID_B, connect=True) for _ in range(3))
        assert l1.decoder_ctx() is None
        m = payload(5, 600_000)
        _, got, _, _ = l1.decoder_consume(p1.encoder_consume(m))
        assert got == m
        assert l1.decoder_ctx() == ctx_lookup(UUID_A) and l1.decoder_ctx() not in (None, codec.h.value)
        w2 = p2.encoder_consume(m)                        # REFs to what p1's frames declared
        assert w2.count(b'\xf1\x01') == 0 and w2.count(b'\xf1\x02') > 100
        back, got, _, _ = l2.decoder_consume(w2)
        assert got == m and not back.startswith(b'\xf0')
        assert l2.decoder_ctx() == l1.decoder_ctx()
        back, got, _, _ = l3.decoder_consume(p3.encoder_consume(m))
        assert back.startswith(b'\xf0') and got == b''    # a fresh cache for UUID_C: <ASK>
        assert l3.decoder_ctx() == ctx_lookup(UUID_C) != l1.decoder_ctx()
        out = b''
        for _ in range(8):                                # <ASK> -> <LEARN> until nothing is unknown
            if not back.startswith(b'\xf0'):
                break
            learn, _, _, _ = p3.decoder_consume(back)
            assert learn.startswith(b'\xf1')
            back, got, _, _ = l3.decoder_consume(learn)
            out += got
        assert out == m
        for p in (p1, p2, p3, l1, l2, l3):
            p.close()
    finally:
        connect_registry_clear()
        for c in (codec, lenc, penc, pdec):
            c.close()


def test_registry_clear_under_a_connected_pipe():
    """A registry clear while a pipe still decodes on the context it connected
    at <HELLO> (advisor round 5): the context stays alive for that pipe -- its
    next frames REF what its first ones declared and decode -- and is destroyed
    when the pipe closes; a new connect after the clear gets a fresh cache."""
    from wanproxy_amd.xcgpu import Context, PipePair, connect_registry_clear, ctx_lookup
    connect_registry_clear()
    codec = Context(0, cache_segments=1 << 15)
    lenc = Context(0, cache_segments=1 << 15)
    penc = Context(0, cache_segments=1 << 15)
    pdec = Context(0, cache_segments=1 << 15)
    try:
        p1 = PipePair(penc, pdec, UUID_A)
        l1 = PipePair(lenc, codec, UUID_B, connect=True)
        m = payload(11, 300_000)
        _, got, _, _ = l1.decoder_consume(p1.encoder_consume(m))
        assert got == m and l1.decoder_ctx() == ctx_lookup(UUID_A)
        connect_registry_clear()                          # the pipe still holds its context
        assert ctx_lookup(UUID_A) is None
        w = p1.encoder_consume(m)                         # all REFs to what the first frames declared
        assert w.count(b'\xf1\x02') > 100
        back, got, _, _ = l1.decoder_consume(w)
        assert got == m and not back.startswith(b'\xf0')
        l1.close()                                        # the deferred destroy happens here
        l2 = PipePair(lenc, codec, UUID_B, connect=True)
        back, got, _, _ = l2.decoder_consume(PipePair(penc, pdec, UUID_A).encoder_consume(payload(12, 10_000)))
        assert l2.decoder_ctx() == ctx_lookup(UUID_A)
        l2.close()
        p1.close()
    finally:
        connect_registry_clear()
        for c in (codec, lenc, penc, pdec):
            c.close()
