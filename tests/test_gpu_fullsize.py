"""Full-size parity on the headline workload (BASELINE.json configs[1], SURVEY
8d C2): all 4096 x 64 KiB chunks, not a sample, compared with the CPU oracle
(pinned to the reference, tests/test_oracle.py) in both semantics, and the
stream encoding decoded back on the GPU.

  S1  every chunk one XCodecEncoder::encode with a fresh XCodecMemoryCache
      (xcodec/xcodec_encoder.cc:74-274, a new cache per call)
  S2  the chunks as successive encode() calls of one encoder (tack's loop,
      programs/tack/tack.cc:298-321)
"""
from concurrent.futures import ThreadPoolExecutor

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

CHUNK, N = 65536, 4096


@pytest.fixture(scope='module')
def c2():
    from wanproxy_amd import synth
    data = np.frombuffer(synth.stream(0xC2, N * CHUNK, 50, 0), np.uint8).copy()
    offs, lens = synth.chunks_of(data.tobytes(), CHUNK)
    return data, offs, lens


def _oracle_independent(data, offs, lens):
    from oracle.lib import Oracle
    o = Oracle()
    parts = np.array_split(np.arange(offs.size), 8)
    with ThreadPoolExecutor(8) as ex:     # (ctypes releases the GIL; one fresh cache per chunk)
        res = list(ex.map(lambda idx: o.encode_batch(data, offs[idx], lens[idx], mode=0), parts))
    return [e for r in res for e in r]


def test_c2_independent_all_chunks(c2):
    from wanproxy_amd.xcgpu import Context
    data, offs, lens = c2
    ctx = Context(0)
    got = ctx.encode_chunks(data, offs, lens)
    ctx.close()
    exp = _oracle_independent(data, offs, lens)
    bad = [i for i in range(N) if got[i] != exp[i]]
    assert not bad, f'{len(bad)} of {N} chunks differ, first {bad[:8]}'
    assert sum(map(len, got)) == sum(map(len, exp))


@pytest.mark.parametrize('seed', [0, 1], ids=['round0', 'seeded'])
def test_c2_stream_all_chunks_and_decode(c2, seed):
    from oracle.lib import Oracle
    from wanproxy_amd.xcgpu import XCG_SEM_STREAM, Context, lib
    data, offs, lens = c2
    old = lib().xcg_debug_set_stream_seed(seed)
    try:
        ctx = Context(0, cache_segments=1 << 18)
        got = ctx.encode_chunks(data, offs, lens, semantics=XCG_SEM_STREAM)
        ndecl = ctx.cache_size()
        ctx.close()
    finally:
        lib().xcg_debug_set_stream_seed(old)
    exp = Oracle().encode_batch(data, offs, lens, mode=1)
    bad = [i for i in range(N) if got[i] != exp[i]]
    assert not bad, f'{len(bad)} of {N} chunks differ, first {bad[:8]}'
    assert 0 < ndecl <= N * (CHUNK // 2048)          # the batch's declarations were committed
    dctx = Context(0, cache_segments=1 << 18)
    outs, st, _, unk = dctx.decode_chunks(got)
    dctx.close()
    assert not (st != 0).any() and not unk
    assert b''.join(outs) == data.tobytes()
