"""zlib stage oracle checks (CPU): the C restatement of zlib 1.2.11's deflate
(oracle/zlib_oracle.c) against the real system zlib in DeflatePipe's call
pattern (zlib/deflate_pipe.cc:57-115) and against the committed fixtures."""
import hashlib
import json
import os
import random
import zlib

import pytest

from oracle.zlib_pipe import DeflatePipeRef, InflatePipeRef, ZOracle, ZLIB_VERSION
from tests.zlib_cases import cases, gen_bytes, wan_stream

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_zlib_version_pinned():
    assert zlib.ZLIB_RUNTIME_VERSION == ZLIB_VERSION


def test_segmentation_does_not_change_output():
    """DeflatePipe feeds each Buffer segment to deflate(Z_NO_FLUSH); the
    output equals one deflate of the call's bytes (the model's premise)."""
    rng = random.Random(3)
    for level, calls in cases(11, 12):
        a, b = DeflatePipeRef(level), DeflatePipeRef(level)
        for c in calls:
            segs = []
            left = len(c)
            while left:
                n = min(left, rng.choice([1, 7, 100, 2048, 4096]))
                segs.append(n)
                left -= n
            assert a.consume(c) == b.consume(c, segs or None)


def test_golden_fixture():
    with open(os.path.join(ROOT, 'tests/golden/zlib.json')) as f:
        g = json.load(f)
    assert g['zlib'] == ZLIB_VERSION
    streams = cases(7, 24)
    assert len(streams) == len(g['streams'])
    for (level, calls), rec in zip(streams, g['streams']):
        assert rec['level'] == level
        o, r = ZOracle(level), DeflatePipeRef(level)
        for c, e in zip(calls, rec['calls']):
            assert hashlib.sha256(c).hexdigest() == e['in_sha256']
            got = o.consume(c)
            assert len(got) == e['out_len'] and hashlib.sha256(got).hexdigest() == e['out_sha256']
            assert r.consume(c) == got


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
    for level in range(4, 10):
        assert ZOracle(level).consume(b'') == DeflatePipeRef(level).consume(b'')
    for level in (0, 1, 2, 3):
        with pytest.raises(ValueError):
            ZOracle(level)


def test_oracle_tiny_calls():
    rng = random.Random(9)
    for level in (4, 6, 9):
        o, r = ZOracle(level), DeflatePipeRef(level)
        for _ in range(200):
            c = gen_bytes(rng, rng.randint(1, 6))
            assert o.consume(c) == r.consume(c)
        assert o.consume(b'') == r.consume(b'')
