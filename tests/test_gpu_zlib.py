"""GPU parity of the zlib stage (DeflatePipe, zlib/deflate_pipe.cc:57-115):
xcg_zdeflate_* against the system zlib 1.2.11 driven in DeflatePipe's call
pattern (oracle/zlib_pipe.py) and against the committed fixtures.  Many
streams per batch, successive batches continue them."""
import hashlib
import json
import os
import random
import zlib

import pytest

from oracle.zlib_pipe import DeflatePipeRef
from tests.zlib_cases import cases, fast_cases, gen_bytes, stop_cases, stored_cases, wan_stream

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def run_streams(streams_by_level):
    """streams_by_level: {level: [[call bytes...], ...]} -> {level: [[outputs...]]},
    every level's streams batched together, call k of every stream in batch k."""
    from wanproxy_amd.zpipe import DeflatePipes
    res = {}
    for level, streams in streams_by_level.items():
        ctx = DeflatePipes(level, len(streams))
        outs = [[] for _ in streams]
        for k in range(max(len(s) for s in streams)):
            items = [(i, s[k]) for i, s in enumerate(streams) if k < len(s)]
            got = ctx.consume_many(items)
            for (i, _), g in zip(items, got):
                outs[i].append(g)
        ctx.close()
        res[level] = outs
    return res


def check_vs_zlib(streams_by_level):
    got = run_streams(streams_by_level)
    for level, streams in streams_by_level.items():
        for si, calls in enumerate(streams):
            ref = DeflatePipeRef(level)
            for k, c in enumerate(calls):
                exp = ref.consume(c)
                g = got[level][si][k]
                if g != exp:
                    i = next((i for i in range(min(len(g), len(exp))) if g[i] != exp[i]), min(len(g), len(exp)))
                    raise AssertionError(f'level {level} stream {si} call {k} (len {len(c)}): '
                                         f'got {len(g)} B, zlib {len(exp)} B, first difference at byte {i}')


@pytest.mark.parametrize('key', ['streams', 'fast', 'stops', 'stored'])
def test_golden_fixture_gpu(key):
    with open(os.path.join(ROOT, 'tests/golden/zlib.json')) as f:
        g = json.load(f)
    by_level = {}
    recs = {}
    streams = {'streams': lambda: cases(7, 24), 'fast': lambda: fast_cases(8, 12), 'stops': lambda: stop_cases(9),
               'stored': lambda: stored_cases(10, 10)}[key]()
    for (level, calls), rec in zip(streams, g[key]):
        by_level.setdefault(level, []).append(calls)
        recs.setdefault(level, []).append(rec)
    got = run_streams(by_level)
    for level in by_level:
        for si, rec in enumerate(recs[level]):
            for k, e in enumerate(rec['calls']):
                out = got[level][si][k]
                assert len(out) == e['out_len'] and hashlib.sha256(out).hexdigest() == e['out_sha256'], \
                    (level, si, k)


@pytest.mark.parametrize('seed', [21, 22])
def test_random_streams_vs_zlib(seed):
    by_level = {}
    for level, calls in cases(seed, 14):
        by_level.setdefault(level, []).append(calls)
    check_vs_zlib(by_level)


def test_flush_call_stops_vs_zlib():
    """Consumes whose Z_SYNC_FLUSH call fills DeflatePipe's 64 KiB buffer
    (deflate_pipe.cc:34,86-105): at the final block flush (no marker, bytes
    held back) and inside the flush call's tail (its last positions parsed
    with the next consume's bytes); compressible consumes in between."""
    rng = random.Random(12)
    by_level = {}
    for level, calls in stop_cases(13, (1, 2, 3, 4, 6, 9), range(-2, 272, 11)):
        calls = calls[:2] + [gen_bytes(rng, rng.randint(1, 90000))] + calls[2:]
        by_level.setdefault(level, []).append(calls)
    check_vs_zlib(by_level)


def test_fast_levels_vs_zlib():
    """deflate_fast (levels 1-3): which positions are hashed depends on the parse."""
    by_level = {}
    for level, calls in fast_cases(31, 18):
        by_level.setdefault(level, []).append(calls)
    check_vs_zlib(by_level)


def test_stored_level_segments_vs_zlib():
    """Level 0 (deflate_stored): block sizes follow each deflate() call's
    segment and the pipe's 64 KiB buffer; 24 streams with random Buffer
    segmentations, every consume equal to zlib's on the same segments."""
    from wanproxy_amd.zpipe import DeflatePipes
    rng = random.Random(44)
    streams = [calls for _, calls in stored_cases(45, 24)]
    segs = []
    for calls in streams:
        row = []
        for c in calls:
            out, t = [], 0
            mode = rng.choice(['full', 'random', 'small'])
            while t < len(c):
                k = {'full': 2048, 'random': rng.randint(1, 2048), 'small': rng.randint(1, 64)}[mode]
                out.append(min(k, len(c) - t))
                t += out[-1]
            row.append(out)
        segs.append(row)
    ctx = DeflatePipes(0, len(streams))
    got = [[] for _ in streams]
    for k in range(max(len(x) for x in streams)):
        items = [(i, s[k], segs[i][k] if s[k] else None) for i, s in enumerate(streams) if k < len(s)]
        for (i, _, _), g in zip(items, ctx.consume_many(items)):
            got[i].append(g)
    ctx.close()
    for i, calls in enumerate(streams):
        ref = DeflatePipeRef(0)
        for k, c in enumerate(calls):
            assert got[i][k] == ref.consume(c, segs[i][k] if c else None), (i, k, len(c))


def test_tiny_calls_vs_zlib():
    rng = random.Random(5)
    streams = [[gen_bytes(rng, rng.randint(1, 6)) for _ in range(40)] + [b''] for _ in range(8)]
    check_vs_zlib({6: streams, 9: streams[:3], 4: streams[3:5], 1: streams[5:], 3: streams[:2], 0: streams[2:6]})


def test_many_streams_wan_traffic_round_trip():
    """256 streams x 3 consumes of 64 KiB of XCodec-output-like bytes (level 6,
    wanproxy.conf), each stream inflated back by zlib."""
    streams = [wan_stream(1000 + i, 3, 65536) + [b''] for i in range(256)]
    got = run_streams({6: streams})[6]
    for i, calls in enumerate(streams[:64]):
        ref = DeflatePipeRef(6)
        for k, c in enumerate(calls):
            assert got[i][k] == ref.consume(c), (i, k)
    for i, calls in enumerate(streams):
        assert zlib.decompress(b''.join(got[i])) == b''.join(calls)


def test_long_matches_and_slides():
    """Runs and far copies across several window slides in one call and
    across calls (512 KiB calls, 258-byte matches, nice breaks)."""
    rng = random.Random(77)
    base = rng.randbytes(40000)
    s1 = [base * 13, bytes(300000), base[::-1] * 3 + base] + [b'']
    s2 = [gen_bytes(rng, 524288), gen_bytes(rng, 100000)] + [b'']
    check_vs_zlib({6: [s1, s2], 9: [s1], 4: [s2], 1: [s1, s2], 2: [s2], 3: [s1], 0: [s1, s2]})


def test_errors():
    from wanproxy_amd.xcgpu import XCGError
    from wanproxy_amd.zpipe import DeflatePipes
    with pytest.raises(XCGError):
        DeflatePipes(10, 1)
    ctx = DeflatePipes(6, 2)
    with pytest.raises(XCGError):
        ctx.consume_many([(0, b'a'), (0, b'b')])
    with pytest.raises(XCGError):
        ctx.consume_many([(5, b'a')])
    assert ctx.pipe(1).consume(b'') == DeflatePipeRef(6).consume(b'')
    ctx.reset(1)
    assert ctx.pipe(1).consume(b'hello') == DeflatePipeRef(6).consume(b'hello')
    ctx.close()


# ---------------------------------------------------------------- InflatePipe
@pytest.fixture(params=[1, 2, 3], ids=['wave', 'workgroup', 'quarter-workgroup'])
def inflate_mode(request):
    """Every inflate kernel: a wave per call (batches beyond 4096 streams), a
    1024-thread workgroup per call (the per-call path: speculative Huffman
    regions) and a 256-thread one (batches of 257-4096 calls, 16 KiB regions)."""
    from wanproxy_amd.zpipe import set_inflate_mode
    set_inflate_mode(request.param)
    yield request.param
    set_inflate_mode(0)


def inflate_streams(streams, out_cap=None):
    """streams: [[input cut bytes...]] -> [[(produced, status)...]], call k of
    every stream in batch k (InflatePipe::consume per cut).  out_cap: the first
    output room of every call (consume_many repeats a -2 call with 4x more)."""
    from wanproxy_amd.zpipe import InflatePipes
    ctx = InflatePipes(len(streams))
    outs = [[] for _ in streams]
    for k in range(max(len(s) for s in streams)):
        items = [(i, s[k]) for i, s in enumerate(streams) if k < len(s)]
        for (i, _), g in zip(items, ctx.consume_many(items, out_cap=out_cap)):
            outs[i].append(g)
    ctx.close()
    return outs


def cuts(rng, z: bytes, mode: str):
    if mode == 'bytes':
        return [z[i:i + 1] for i in range(len(z))]
    out, i = [], 0
    while i < len(z):
        n = rng.choice([1, 2, 3, 7, 100, 1500, 65536]) if mode == 'random' else 65536
        out.append(z[i:i + n])
        i += n
    return out


def test_inflate_zlib_streams_any_cut(inflate_mode):
    """zlib-made streams (stored, static, dynamic blocks; levels 1-9) cut at
    random points; every call's output equals zlib's inflate on the same cuts."""
    from oracle.zlib_pipe import InflatePipeRef
    rng = random.Random(31)
    srcs, streams = [], []
    for level, calls in cases(41, 16):
        level = rng.choice([1, 2, 3, level, 9])
        ref = DeflatePipeRef(level)
        z = b''.join(ref.consume(c) for c in calls if c) + ref.consume(b'')
        srcs.append(b''.join(calls))
        streams.append(cuts(rng, z, rng.choice(['random', 'random', 'frames'])) + [b''])
    got = inflate_streams(streams)
    for si, (src, cs) in enumerate(zip(srcs, streams)):
        ref = InflatePipeRef()
        for k, c in enumerate(cs[:-1]):
            exp = ref.consume(c)
            out, st = got[si][k]
            assert out == exp, (si, k, len(out), len(exp))
            assert st in (0, 1), (si, k, st)
        assert b''.join(o for o, _ in got[si]) == src
        assert got[si][-1] == (b'', 1)     # EOS after the end: produce_eos


def test_inflate_byte_by_byte_and_small(inflate_mode):
    streams = []
    srcs = []
    for i, data in enumerate([b'', b'a', b'hello hello hello hello', bytes(1000), random.Random(3).randbytes(700)]):
        z = zlib.compress(data, 6)
        srcs.append(data)
        streams.append([z[j:j + 1] for j in range(len(z))] + [b''])
    got = inflate_streams(streams)
    for si, src in enumerate(srcs):
        assert b''.join(o for o, _ in got[si]) == src
        assert got[si][-1][1] == 1


def test_gpu_deflate_then_gpu_inflate(inflate_mode):
    """wanproxy's zlib stage both ways on the GPU: DeflatePipe output, cut
    into frames, through InflatePipe, for 64 streams."""
    rng = random.Random(8)
    streams = [wan_stream(3000 + i, 3, 65536) + [b''] for i in range(64)]
    z = run_streams({6: streams})[6]
    cut = [cuts(rng, b''.join(zs), 'random') + [b''] for zs in z]
    got = inflate_streams(cut)
    for i in range(64):
        assert b''.join(o for o, _ in got[i]) == b''.join(streams[i])


def test_inflate_errors(inflate_mode):
    good = zlib.compress(b'payload ' * 100, 6)
    bad_adler = good[:-1] + bytes([good[-1] ^ 1])
    bad_header = bytes([0x78, 0x9d]) + good[2:]
    trailing = good + b'x'
    got = inflate_streams([[bad_adler], [bad_header], [trailing], [good, b'']])
    assert got[0][0][1] == -1
    assert got[1][0] == (b'', -1)
    assert got[2][0][1] == -1
    assert got[3][0] == (b'payload ' * 100, 1) and got[3][1] == (b'', 1)


def test_distance_boundaries_both_ways():
    """Back-references at distances around the inflate ring's limits (near copies
    up to 2 KiB, ring 4 KiB, flush every 1 KiB) and zlib's own (258, 32 KiB
    window): GPU deflate equals zlib call by call, and GPU inflate decodes
    zlib's level-9 stream of the same data, cut at random points."""
    rng = random.Random(90)
    dists = [1, 2, 3, 257, 258, 259, 1023, 1024, 1025, 2047, 2048, 2049, 3000, 4095, 4096, 4097,
             6000, 8191, 8192, 8193, 16384, 32506, 32507, 32767]
    parts = []
    for d in dists:
        base = rng.randbytes(d)
        parts.append(base + base[:rng.choice([3, 17, 258, 600])] + rng.randbytes(37))
    data = b''.join(parts)
    calls = [data[i:i + 50000] for i in range(0, len(data), 50000)] + [b'']
    check_vs_zlib({6: [calls], 9: [calls], 1: [calls], 3: [calls]})
    z = zlib.compress(data, 9)
    got = inflate_streams([cuts(rng, z, 'random') + [b'']])[0]
    assert b''.join(o for o, _ in got) == data
    assert got[-1][1] == 1


def test_inflate_retry_after_no_room(inflate_mode):
    """Status -2 (output room too small) commits nothing, wherever it strikes:
    inside a stored block, inside a Huffman block, right after the next
    dynamic block's header.  Calls start with 256 bytes of room and are
    repeated with 4x more; every call's output equals zlib's on the same cuts."""
    from oracle.zlib_pipe import InflatePipeRef
    rng = random.Random(77)
    srcs, streams = [], []
    for si in range(24):
        level = [1, 6, 9, 0][si % 4]
        # blocks of changing statistics: several dynamic blocks per call
        data = b''.join(bytes(rng.choice(b'abcdefgh' if k % 2 else b'0123456789 ') for _ in range(rng.randint(200, 9000)))
                        + rng.randbytes(rng.randint(0, 3000)) for k in range(12))
        z = zlib.compress(data, level)
        srcs.append(data)
        cs, i = [], 0
        while i < len(z):
            n = rng.choice([5, 40, 700, 3000, 9000])
            cs.append(z[i:i + n])
            i += n
        streams.append(cs + [b''])
    got = inflate_streams(streams, out_cap=256)
    for si, (src, cs) in enumerate(zip(srcs, streams)):
        ref = InflatePipeRef()
        for k, c in enumerate(cs[:-1]):
            out, st = got[si][k]
            assert out == ref.consume(c), (si, k)
            assert st in (0, 1), (si, k, st)
        assert b''.join(o for o, _ in got[si]) == src


def test_inflate_slot_reuse_after_reset(inflate_mode):
    """A slot whose stream ended (or failed) serves a fresh InflatePipe after
    xcg_zinflate_reset -- the adapter's constructor on a reused slot."""
    from wanproxy_amd.zpipe import InflatePipes
    ctx = InflatePipes(2)
    a = zlib.compress(b'first stream ' * 50, 6)
    b = zlib.compress(b'second stream ' * 70, 6)
    assert ctx.consume_many([(0, a)]) == [(b'first stream ' * 50, 1)]
    assert ctx.consume_many([(1, b'\x78\x9dgarbage')])[0][1] == -1
    # without a reset the ended / failed slots refuse a new stream
    assert ctx.consume_many([(0, b)])[0][1] == -1
    ctx.reset(0)
    ctx.reset(1)
    head = zlib.decompressobj().decompress(a[:10])
    assert ctx.consume_many([(0, b), (1, a[:10])]) == [(b'second stream ' * 70, 1), (head, 0)]
    assert ctx.consume_many([(1, a[10:])]) == [((b'first stream ' * 50)[len(head):], 1)]
    ctx.close()


def _text(rng, n):
    words = [bytes(rng.choice(b'etaoinshrdlucmfwyp') for _ in range(rng.randint(1, 9))) for _ in range(400)]
    out = bytearray()
    while len(out) < n:
        out += rng.choice(words) + rng.choice([b' ', b' ', b', ', b'.\n'])
    return bytes(out[:n])


def _inflate_both(streams, out_cap=None):
    """Every stream through every kernel: (wave, workgroup, quarter workgroup per call)."""
    from wanproxy_amd.zpipe import set_inflate_mode
    got = []
    try:
        for mode in (1, 2, 3):
            set_inflate_mode(mode)
            got.append(inflate_streams(streams, out_cap=out_cap))
    finally:
        set_inflate_mode(0)
    return got


def test_inflate_workgroup_regions_vs_zlib():
    """The workgroup kernel's speculative regions on the data that exercises
    them: 64 KiB-and-larger consumes of text, of runs (matches on matches,
    distance 1, chains thousands deep), of incompressible bytes (stored and
    Huffman blocks of literals), skewed alphabets (long codes past the primary
    tables), fixed blocks (level 1 on short calls) -- one call, frames and
    random cuts; every call equals zlib's inflate on the same cuts, and the
    wave-per-call kernel's, byte for byte and status for status."""
    from oracle.zlib_pipe import InflatePipeRef
    rng = random.Random(2024)
    datas = [_text(rng, 300000), b'a' * 200000 + b'b' * 70000, bytes(range(256)) * 900,
             rng.randbytes(150000), _text(rng, 5000) * 40,
             bytes(rng.choice(b'\x00\x01\x02\x03' * 50 + bytes(range(256))) for _ in range(120000)),
             b''.join(rng.randbytes(rng.randint(1, 40)) * rng.randint(1, 300) for _ in range(3000))]
    srcs, streams = [], []
    for i, d in enumerate(datas):
        for level in (1, 6, 9):
            z = zlib.compress(d, level)
            for mode in ('whole', 'frames', 'random'):
                srcs.append(d)
                streams.append(([z] if mode == 'whole' else cuts(rng, z, mode)) + [b''])
    # fixed Huffman blocks: zlib's Z_FIXED strategy
    for d in datas[:3]:
        c = zlib.compressobj(6, zlib.DEFLATED, 15, 8, zlib.Z_FIXED)
        z = c.compress(d) + c.flush()
        srcs.append(d)
        streams.append([z, b''])
    wave, wg, quarter = _inflate_both(streams)
    assert quarter == wg
    for si, (src, cs) in enumerate(zip(srcs, streams)):
        assert wg[si] == wave[si], si
        ref = InflatePipeRef()
        for k, c in enumerate(cs[:-1]):
            assert wg[si][k] == (ref.consume(c), wg[si][k][1]), (si, k)
            assert wg[si][k][1] in (0, 1), (si, k)
        assert b''.join(o for o, _ in wg[si]) == src, si


def test_inflate_workgroup_errors_mid_region():
    """Errors deep inside a region decide the call as the one-wave decoder
    does: a distance before the stream's start (a raw stream made against a
    preset dictionary, behind a plain zlib header) after 40 KiB of good output,
    a corrupt code in a long dynamic block, and a bad adler32 after a large
    call.  Both kernels give the same output and status."""
    rng = random.Random(5)
    dic = _text(rng, 8000)
    body = _text(random.Random(6), 40000).upper()   # no match into the (lower-case) dictionary before it
    c = zlib.compressobj(6, zlib.DEFLATED, -15, zdict=dic)
    raw = c.compress(body + dic[1000:3000] + body[:5000]) + c.flush()
    far = bytes([0x78, 0x9c]) + raw + b'\0\0\0\0'
    good = zlib.compress(_text(rng, 200000), 6)
    corrupt = bytearray(good)
    for k in range(20):
        corrupt[len(good) // 2 + k] ^= 0xA5
    bad_adler = good[:-1] + bytes([good[-1] ^ 1])
    streams = [[far], [bytes(corrupt)], [bad_adler], [far[:30000], far[30000:]], [good[:65536], good[65536:], b'']]
    wave, wg, quarter = _inflate_both(streams)
    assert wg == wave and quarter == wave
    assert wg[0][0][1] == -1 and wg[2][0][1] == -1
    assert wg[1][0][1] == -1
    assert wg[4][-1] == (b'', 1)


def _dyn_header_stream(syms, nlen=257, ndist=1):
    """A zlib stream whose one dynamic block header codes the code-length
    symbols `syms` [(symbol, extra value)] with a 2-bit code over {0, 8, 16,
    18} (RFC 1951 3.2.7), nothing after it."""
    bits = []

    def put(v, n):                      # LSB first
        bits.extend((v >> i) & 1 for i in range(n))

    def put_code(c, n):                 # Huffman codes MSB first
        bits.extend((c >> (n - 1 - i)) & 1 for i in range(n))
    put(1, 1)
    put(2, 2)
    put(nlen - 257, 5)
    put(ndist - 1, 5)
    order = [16, 17, 18, 0, 8, 7, 9, 6, 10, 5, 11, 4, 12, 3, 13, 2, 14, 1, 15]
    lens = {0: 2, 8: 2, 16: 2, 18: 2}
    put(len(order) - 4, 4)
    for sym in order:
        put(lens.get(sym, 0), 3)
    code = {0: 0, 8: 1, 16: 2, 18: 3}
    for sym, x in syms:
        put_code(code[sym], 2)
        if sym == 16:
            put(x, 2)
        elif sym == 18:
            put(x, 7)
    bits.extend([0] * (-len(bits) % 8))
    body = bytes(sum(bits[i + k] << k for k in range(8)) for i in range(0, len(bits), 8))
    return bytes([0x78, 0x9c]) + body + bytes(8)


def test_inflate_dynamic_header_errors_both_kernels():
    """Code-length sequences the decoder must refuse, through the serial loop
    (wave kernel) and the lane-speculative decode (workgroup kernels): a first
    symbol 16 (nothing to repeat), a repeat past nlen + ndist, and a sequence
    that leaves the literal/length code incomplete (zlib refuses all three);
    plus a header cut every third byte (the input ends inside it: the call
    stalls, the next one decides).  Every kernel gives the same outputs and
    statuses."""
    first16 = _dyn_header_stream([(16, 0)] + [(8, 0)] * 257)
    over = _dyn_header_stream([(18, 127)] * 2 + [(8, 0)] * 3)
    no_eob = _dyn_header_stream([(18, 127), (18, 107), (8, 0), (8, 0)])   # 256 zeros: length[256] == 0
    cut = _dyn_header_stream([(8, 0)] * 100 + [(16, 3)] * 20 + [(18, 50)] * 2)
    streams = [[first16], [over], [no_eob]] + [[cut[:k], cut[k:]] for k in range(2, len(cut) - 8, 3)]
    wave, wg, quarter = _inflate_both(streams)
    assert wg == wave and quarter == wave
    for si in range(3):
        assert wave[si][0][1] == -1, si


def test_inflate_workgroup_small_room():
    """Output room smaller than a region's output: the region commits the
    threads that fit, the careful path returns -2 where the wave kernel does,
    and the retried calls match zlib."""
    from oracle.zlib_pipe import InflatePipeRef
    rng = random.Random(12)
    srcs, streams = [], []
    for i in range(6):
        d = _text(rng, 150000) if i % 2 else b'xyz' * 60000
        z = zlib.compress(d, 6)
        srcs.append(d)
        streams.append(cuts(rng, z, 'frames') + [b''])
    wave, wg, quarter = _inflate_both(streams, out_cap=3000)
    assert wg == wave and quarter == wave
    for si, (src, cs) in enumerate(zip(srcs, streams)):
        ref = InflatePipeRef()
        for k, c in enumerate(cs[:-1]):
            assert wg[si][k][0] == ref.consume(c), (si, k)
        assert b''.join(o for o, _ in wg[si]) == src


# ------------------------------------------------- drop-in classes (adapter)
def test_dropin_classes_vs_reference_pipes():
    """integration/zlib_pipes_xcgpu.cc -- the engine-backed DeflatePipe /
    InflatePipe bodies -- against the reference's own classes
    (zlib/deflate_pipe.cc, zlib/inflate_pipe.cc compiled from /root/reference),
    both driven through oracle/zpipe_driver.cc with the same Buffers: every
    level 0-9, random segmentations (level 0's blocks follow them), consumes
    whose flush call stops at the 64 KiB buffer, pipes created and destroyed
    while others live (slot reuse), and the inflate side on the same bytes."""
    from oracle.zlib_pipe import ReferencePipes
    ref, gpu = ReferencePipes('ref'), ReferencePipes('dropin')
    rng = random.Random(71)
    streams = (cases(72, 6) + fast_cases(73, 4) + stored_cases(74, 4) + stop_cases(75, (0, 1, 6), range(5, 270, 88)))
    for si, (level, calls) in enumerate(streams):
        a, b = gpu.pipe('deflate', level), ref.pipe('deflate', level)
        z = []
        for k, c in enumerate(calls):
            segs = None
            if c and rng.random() < 0.6:
                segs, t = [], 0
                while t < len(c):
                    segs.append(min(rng.randint(1, 2048), len(c) - t))
                    t += segs[-1]
            g, e = a.consume(c, segs), b.consume(c, segs)
            assert g == e, (si, level, k, len(c), len(g[0]), len(e[0]))
            z.append(g[0])
        if calls and not calls[-1]:
            zz = b''.join(z)
            cut, i = [], 0
            while i < len(zz):
                n = rng.choice([1, 700, 3000, 65536])
                cut.append(zz[i:i + n])
                i += n
            ia, ib = gpu.pipe('inflate'), ref.pipe('inflate')
            for x in cut:
                assert ia.consume(x) == ib.consume(x), (si, len(x))
            assert ia.consume(b'') == ib.consume(b'') == (b'', 1)
            ia.close()
            ib.close()
        a.close()
        b.close()


def test_dropin_pool_grows_past_one_context():
    """More live DeflatePipes than one context's 4096 slots: the adapter's pool
    adds a context (no HALT); pipes on both contexts match the reference."""
    from oracle.zlib_pipe import ReferencePipes
    gpu, ref = ReferencePipes('dropin'), ReferencePipes('ref')
    pipes = [gpu.pipe('deflate', 6) for _ in range(4100)]
    rng = random.Random(5)
    for i in (0, 4095, 4096, 4099):
        data = gen_bytes(rng, 5000)
        assert pipes[i].consume(data) == ref.pipe('deflate', 6).consume(data), i
    for p in pipes:
        p.close()
