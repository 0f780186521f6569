"""zlib stage oracle checks (CPU): the C restatement of zlib 1.2.11's deflate
(oracle/zlib_oracle.c) against the real system zlib in DeflatePipe's call
pattern (zlib/deflate_pipe.cc:57-115) and against the committed fixtures."""
import hashlib
import json
import os
import random
import zlib

import pytest

from oracle.zlib_pipe import DeflatePipeRef, DeflatePipeUnbounded, InflatePipeRef, ZOracle, ZLIB_VERSION
from tests.zlib_cases import cases, fast_cases, gen_bytes, stop_cases, stored_cases, wan_stream

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_zlib_version_pinned():
    assert zlib.ZLIB_RUNTIME_VERSION == ZLIB_VERSION


def test_segmentation_does_not_change_output():
    """DeflatePipe feeds each Buffer segment (<= 2048 bytes, BUFFER_SEGMENT_SIZE)
    to deflate(Z_NO_FLUSH); the output does not depend on where the segments
    are cut (the model's premise), the 64 KiB flush-call stop included."""
    rng = random.Random(3)
    for level, calls in cases(11, 12) + fast_cases(12, 6) + stop_cases(13, (2, 6), range(0, 270, 45)):
        a, b = DeflatePipeRef(level), DeflatePipeRef(level)
        for c in calls:
            segs = []
            left = len(c)
            while left:
                n = min(left, rng.choice([1, 7, 100, 2048, rng.randint(1, 2048)]))
                segs.append(n)
                left -= n
            assert a.consume(c) == b.consume(c, segs or None)


@pytest.mark.parametrize('key', ['streams', 'fast', 'stops'])
def test_golden_fixture(key):
    with open(os.path.join(ROOT, 'tests/golden/zlib.json')) as f:
        g = json.load(f)
    assert g['zlib'] == ZLIB_VERSION
    streams = {'streams': lambda: cases(7, 24), 'fast': lambda: fast_cases(8, 12), 'stops': lambda: stop_cases(9)}[key]()
    assert len(streams) == len(g[key])
    for (level, calls), rec in zip(streams, g[key]):
        assert rec['level'] == level
        o, r = ZOracle(level), DeflatePipeRef(level)
        for c, e in zip(calls, rec['calls']):
            assert hashlib.sha256(c).hexdigest() == e['in_sha256']
            got = o.consume(c)
            assert len(got) == e['out_len'] and hashlib.sha256(got).hexdigest() == e['out_sha256']
            assert r.consume(c) == got


def test_flush_call_stops_at_the_pipe_buffer():
    """The pipe's single Z_SYNC_FLUSH call into its 64 KiB buffer (deflate_pipe.cc:
    34,86-105): a 64 KiB incompressible consume yields exactly 65536 bytes and no
    sync marker, unlike zlib driven with unbounded output; the stream still
    inflates to the input.  Both stop kinds occur: at the final block flush, and
    inside the flush call's tail with positions left for the next consume."""
    import ctypes as C
    lib = ZOracle.lib()
    lib.zr_carry.argtypes = [C.c_void_p, C.POINTER(C.c_uint64), C.POINTER(C.c_uint64)]
    rng = random.Random(21)
    kinds = set()
    for level, calls in stop_cases(22, (1, 6), range(0, 270, 30)):
        o, r, u = ZOracle(level), DeflatePipeRef(level), DeflatePipeUnbounded(level)
        outs = []
        for i, c in enumerate(calls):
            got = o.consume(c)
            assert got == r.consume(c)
            outs.append(got)
            if i == 0 and len(c) > 65536:                  # the first consume always stops
                d, p = C.c_uint64(), C.c_uint64()
                lib.zr_carry(o.s, C.byref(d), C.byref(p))
                assert len(got) == 65536 and p.value > 0
                kinds.add('tail' if d.value else 'final')
            u.consume(c)
        assert zlib.decompress(b''.join(outs)) == b''.join(calls)
    assert kinds == {'tail', 'final'}
    a, b = DeflatePipeRef(6), DeflatePipeUnbounded(6)
    x = rng.randbytes(65536)
    assert len(a.consume(x)) == 65536 and len(b.consume(x)) > 65536


@pytest.mark.parametrize('seed', [1, 2, 3])
def test_oracle_vs_zlib_random(seed):
    for level, calls in cases(100 + seed, 10):
        o, r = ZOracle(level), DeflatePipeRef(level)
        for i, c in enumerate(calls):
            assert o.consume(c) == r.consume(c), (seed, level, i, len(c))


def test_oracle_vs_zlib_wan_stream_round_trip():
    calls = wan_stream(5, 8, 65536) + [b'']
    o, r, inf = ZOracle(6), DeflatePipeRef(6), InflatePipeRef()
    back = b''
    for c in calls:
        z = o.consume(c)
        assert z == r.consume(c)
        back += inf.consume(z)
    assert back == b''.join(calls)


def test_oracle_empty_stream_and_levels():
    for level in range(1, 10):
        assert ZOracle(level).consume(b'') == DeflatePipeRef(level).consume(b'')
    with pytest.raises(ValueError):
        ZOracle(0)


@pytest.mark.parametrize('seed', [1, 2])
def test_oracle_fast_levels_vs_zlib(seed):
    """deflate_fast (levels 1-3): the parse decides which positions are hashed."""
    for level, calls in fast_cases(300 + seed, 10):
        o, r = ZOracle(level), DeflatePipeRef(level)
        for i, c in enumerate(calls):
            assert o.consume(c) == r.consume(c), (seed, level, i, len(c))


def test_oracle_tiny_calls():
    rng = random.Random(9)
    for level in (1, 3, 4, 6, 9):
        o, r = ZOracle(level), DeflatePipeRef(level)
        for _ in range(200):
            c = gen_bytes(rng, rng.randint(1, 6))
            assert o.consume(c) == r.consume(c)
        assert o.consume(b'') == r.consume(b'')


# ------------------------------------------------------------------ level 0
class StoredPlanCPU:
    """The engine's level-0 planner (wanproxy_amd/csrc/xcg_stored_plan.h, the
    host half of the GPU path) run on the CPU by oracle/stored_plan_harness.cc."""
    _lib = None

    def __init__(self):
        import ctypes as C
        if StoredPlanCPU._lib is None:
            L = C.CDLL(os.path.join(ROOT, 'oracle/build/libstoredplan.so'))
            L.sp_new.restype = C.c_void_p
            L.sp_free.argtypes = [C.c_void_p]
            L.sp_consume.restype = C.c_int64
            L.sp_consume.argtypes = [C.c_void_p, C.c_char_p, C.c_uint64, C.c_void_p, C.c_uint32, C.c_char_p,
                                     C.c_uint64]
            StoredPlanCPU._lib = L
        self.C = C
        self.s = StoredPlanCPU._lib.sp_new()

    def consume(self, data, segments=None):
        C = self.C
        arr = (C.c_uint32 * max(1, len(segments)))(*segments) if segments else None
        buf = C.create_string_buffer(2 * len(data) + 300000)
        n = StoredPlanCPU._lib.sp_consume(self.s, data, len(data), arr, len(segments) if segments else 0, buf,
                                          len(buf))
        assert n >= 0
        return buf.raw[:n]

    def __del__(self):
        if getattr(self, 's', None):
            StoredPlanCPU._lib.sp_free(self.s)


def _segments(rng, n):
    out, t = [], 0
    mode = rng.choice(['full', 'random', 'small'])
    while t < n:
        k = {'full': 2048, 'random': rng.randint(1, 2048), 'small': rng.randint(1, 64)}[mode]
        out.append(min(k, n - t))
        t += out[-1]
    return out


@pytest.mark.parametrize('seed', [1, 2, 3])
def test_stored_plan_vs_zlib(seed):
    """Level 0: deflate_stored's block sizes follow the segments each deflate()
    call gets and the pipe's 64 KiB buffer; the planner reproduces zlib's output
    call by call for random segmentations (<= 2048 bytes, BUFFER_SEGMENT_SIZE)."""
    rng = random.Random(seed)
    for _, calls in stored_cases(400 + seed, 12):
        p, r = StoredPlanCPU(), DeflatePipeRef(0)
        for k, c in enumerate(calls):
            segs = _segments(rng, len(c)) if c else None
            assert p.consume(c, segs) == r.consume(c, segs), (seed, k, len(c))


def test_stored_golden():
    with open(os.path.join(ROOT, 'tests/golden/zlib.json')) as f:
        g = json.load(f)
    for (level, calls), rec in zip(stored_cases(10, 10), g['stored']):
        p = StoredPlanCPU()
        for c, e in zip(calls, rec['calls']):
            got = p.consume(c)
            assert len(got) == e['out_len'] and hashlib.sha256(got).hexdigest() == e['out_sha256']


# ---------------------------------------------------------- reference pipes
def _ref_available():
    return os.path.exists(os.path.join(ROOT, 'oracle/_ref/libzpref.so'))


@pytest.mark.skipif(not _ref_available(), reason='oracle/_ref/libzpref.so not built')
def test_checker_is_the_reference_pipe():
    """DeflatePipeRef (oracle/deflate_pipe_ref.c, the loop of deflate_pipe.cc:
    57-115 restated over the system zlib) equals the reference's own
    DeflatePipe class (zlib/deflate_pipe.cc compiled from /root/reference,
    oracle/_ref/libzpref.so) call by call, at every level, on random Buffer
    segmentations; and the reference InflatePipe produces zlib's inflate."""
    from oracle.zlib_pipe import ReferencePipes
    R = ReferencePipes('ref')
    rng = random.Random(17)
    streams = (cases(57, 8) + fast_cases(58, 6) + stored_cases(59, 6) +
               stop_cases(60, (2, 5), range(0, 270, 90)))
    for level, calls in streams:
        a, b = R.pipe('deflate', level), DeflatePipeRef(level)
        z = []
        for c in calls:
            segs = _segments(rng, len(c)) if c and rng.random() < 0.6 else None
            got, st = a.consume(c, segs)
            assert got == b.consume(c, segs), (level, len(c))
            assert st == (0 if c else 1)
            z.append(got)
        if calls and not calls[-1]:
            inf, ref = R.pipe('inflate'), InflatePipeRef()
            zz = b''.join(z)
            cut = [zz[i:i + 3000] for i in range(0, len(zz), 3000)]
            out = b''.join(inf.consume(x)[0] for x in cut)
            assert out == b''.join(ref.consume(x) for x in cut) == b''.join(calls)
            assert inf.consume(b'') == (b'', 1)
