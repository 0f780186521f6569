"""The quiet-chunk screen of small stream chunks (xcg_encode.hip
stream_screen_kernel): chunks none of whose windows can be found get the cold
parse (the 2048-byte tiling) without the state machine, the rest are parsed.
Every case is encoded with the screen on and off and both equal the oracle's
sequential XCodecEncoder (xcodec/xcodec_encoder.cc:74-274) over the same
encode() calls; the counts show the screen took the chunks it should."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu

KiB = 1024


@pytest.fixture
def screen_mode():
    from wanproxy_amd.xcgpu import lib
    old = lib().xcg_debug_set_screen(2)
    yield
    lib().xcg_debug_set_screen(old)


def _encode(data, offs, lens, per, mode, cache_segments=1 << 15):
    from wanproxy_amd.xcgpu import XCG_SEM_STREAM, Context, lib
    import ctypes as C
    lib().xcg_debug_set_screen(mode)
    ctx = Context(0, cache_segments=cache_segments)
    out = []
    for a in range(0, len(offs), per):
        out += ctx.encode_chunks(data, offs[a:a + per], lens[a:a + per], semantics=XCG_SEM_STREAM)
    ctx.close()
    s, p = C.c_uint64(), C.c_uint64()
    lib().xcg_debug_screen_counts(C.byref(s), C.byref(p))
    return out, int(s.value), int(p.value)


def _check(oracle, data, offs, lens, per):
    exp = oracle.encode_batch(data, offs, lens, mode=1)
    on, seen, parsed = _encode(data, offs, lens, per, 2)
    off, _, _ = _encode(data, offs, lens, per, 0)
    bad = next((i for i in range(len(exp)) if on[i] != exp[i]), None)
    assert bad is None, ('screen on', bad)
    assert off == exp
    return seen, parsed


def test_c4_packets(screen_mode, stream_seed, oracle):
    """C4's workload: 4 KiB packets, 4 % duplicate segments, batches of 1024."""
    from wanproxy_amd import synth
    data = synth.stream(0xC4, 6144 * 4 * KiB, 4, 0)
    offs, lens = synth.chunks_of(data, 4 * KiB)
    seen, parsed = _check(oracle, data, offs, lens, 1024)
    assert seen >= len(offs) and parsed < seen // 3, (seen, parsed)


@pytest.mark.parametrize('dup', [0, 30, 90])
def test_ragged_small_chunks(screen_mode, stream_seed, oracle, dup):
    """Chunk lengths 0 .. 8191 (none, one, two and three tiles, one-window
    pieces at 2048 k), 0xF1-heavy data, duplicates from 0 to 90 %."""
    from wanproxy_amd import synth
    rng = np.random.default_rng(dup + 1)
    data = synth.stream(0x5C0 + dup, 12 << 20, dup, 3)
    lens = rng.choice(np.array([0, 1, 2047, 2048, 2049, 3000, 4095, 4096, 4097, 6144, 6145, 8191], np.uint32),
                      size=3000)
    lens = lens.astype(np.uint32)
    offs = np.zeros(lens.size, np.uint64)
    offs[1:] = np.cumsum(((lens.astype(np.uint64) + 15) // 16) * 16)[:-1]    # 16-byte aligned starts
    assert int(offs[-1]) + int(lens[-1]) <= len(data)
    _check(oracle, data, offs, lens, 500)


def test_repeats_inside_and_across_packets(screen_mode, stream_seed, oracle):
    """Packets whose second tile repeats their first (an own-tile REF at window
    2048), packets equal to an earlier packet, repeats shifted by one byte,
    windows equal to a later tile, and unaligned starts (not screened)."""
    rng = np.random.default_rng(7)
    blk = [rng.integers(0, 256, 2048, dtype=np.uint8) for _ in range(64)]
    parts = []
    for k in range(1500):
        r = k % 6
        if r == 0:
            parts.append(np.concatenate([blk[k % 64], blk[k % 64]]))                 # own repeat
        elif r == 1:
            parts.append(np.concatenate([blk[(k * 7) % 64], blk[(k * 3) % 64]]))     # earlier packets' tiles
        elif r == 2:
            parts.append(np.concatenate([blk[k % 64][1:], blk[(k + 1) % 64], blk[k % 64][:1]]))   # shifted
        elif r == 3:
            parts.append(rng.integers(0, 256, 4096, dtype=np.uint8))                 # fresh
        elif r == 4:
            b = rng.integers(0, 256, 2048, dtype=np.uint8)
            parts.append(np.concatenate([b[:1000], b, b[1000:1048]]))                # a window = its later tile
        else:
            parts.append(rng.integers(0, 4, 5000, dtype=np.uint8))                   # low-entropy
    lens = np.array([p.size for p in parts], np.uint32)
    offs = np.zeros(lens.size, np.uint64)
    step = ((lens.astype(np.uint64) + 15) // 16) * 16
    step[::5] += 3                                                                   # some unaligned starts
    offs[1:] = np.cumsum(step)[:-1]
    data = np.zeros(int(offs[-1]) + int(lens[-1]), np.uint8)
    for o, p in zip(offs, parts):
        data[int(o):int(o) + p.size] = p
    seen, parsed = _check(oracle, data.tobytes(), offs, lens, 300)
    assert parsed < seen


def test_warm_cache_refs(screen_mode, oracle):
    """The same packets twice: the second pass REFs everything from the cache,
    so the screen sends every packet on to the parse."""
    from wanproxy_amd import synth
    data = synth.stream(0x3A3, 2048 * 4 * KiB, 2, 0)
    offs, lens = synth.chunks_of(data, 4 * KiB)
    offs2 = np.concatenate([offs, offs])
    lens2 = np.concatenate([lens, lens])
    _check(oracle, data, offs2, lens2, 1024)


def test_screen_after_large_chunks_on_one_context(screen_mode, oracle):
    """A context whose scratch was grown by a batch of 64 KiB chunks still
    screens its later 4 KiB packets (advisor round 5: the queues used to be
    allocated only by a small-chunk call that grew the scratch), and both
    batches equal the oracle's sequential encoder over the same calls."""
    import ctypes as C
    from wanproxy_amd import synth
    from wanproxy_amd.xcgpu import XCG_SEM_STREAM, Context, lib
    big = synth.stream(0xB6, 64 * 64 * KiB, 10, 0)
    small = synth.stream(0xC4, 2048 * 4 * KiB, 4, 0)
    data = big + small
    bo, bl = synth.chunks_of(big, 64 * KiB)
    so, sl = synth.chunks_of(small, 4 * KiB)
    so = so + len(big)
    offs = np.concatenate([bo, so])
    lens = np.concatenate([bl, sl])
    exp = oracle.encode_batch(data, offs, lens, mode=1)
    ctx = Context(0, cache_segments=1 << 15)
    got = ctx.encode_chunks(data, bo, bl, semantics=XCG_SEM_STREAM)
    s, p = C.c_uint64(), C.c_uint64()
    lib().xcg_debug_screen_counts(C.byref(s), C.byref(p))
    got += ctx.encode_chunks(data, so, sl, semantics=XCG_SEM_STREAM)
    lib().xcg_debug_screen_counts(C.byref(s), C.byref(p))
    ctx.close()
    bad = next((i for i in range(len(exp)) if got[i] != exp[i]), None)
    assert bad is None, bad
    assert s.value >= len(so) and p.value < s.value // 3, (s.value, p.value)
