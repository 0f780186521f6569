"""Worst-case stream convergence: the declaration-dependence
chain of tests/chain_case.py, where chunk k's parse depends on chunk k-1's
final declarations, so the Jacobi rounds can fix only about one chunk per
round.  The result must still equal the sequential oracle, the round count
stays within the n + 1 bound of xcg_launch_encode_stream, and the time stays
bounded -- on the unbounded, bounded (LRU) and pair caches, both seed modes."""
import time

import pytest

from chain_case import chain

pytestmark = pytest.mark.gpu
N = 96


@pytest.mark.parametrize('kind', ['unbounded', 'bounded', 'pair'])
def test_chain_converges_exactly(oracle, stream_seed, kind):
    from wanproxy_amd.xcgpu import XCG_SEM_STREAM, Context
    d, offs, lens = chain(N)
    kw = {'unbounded': dict(cache_segments=1 << 14), 'bounded': dict(memory_cache_limit=4096 * 2048),
          'pair': dict(memory_cache_limit=1024 * 2048, disk_bytes=8 << 20)}[kind]
    ctx = Context(0, **kw)
    t0 = time.perf_counter()
    got = ctx.encode_chunks(d, offs, lens, semantics=XCG_SEM_STREAM)
    dt = time.perf_counter() - t0
    rounds = ctx.last_rounds()
    ctx.close()
    if kind == 'unbounded':
        exp = oracle.encode_batch(d, offs, lens, mode=1)
    else:
        c = oracle.cache_new(4096 * 2048) if kind == 'bounded' else oracle.cache_new_pair(1024 * 2048, 8 << 20)
        exp = oracle.encode_batch(d, offs, lens, mode=1, cache=c)
        oracle.cache_free(c)
    bad = [k for k in range(N) if got[k] != exp[k]]
    assert not bad, (kind, bad[:8])
    assert rounds <= N + 1 + 16, rounds          # (pair / LRU passes add a few rounds each)
    if kind == 'unbounded':
        assert rounds >= N // 2, rounds          # the chain really costs ~one round per chunk
    assert dt < 20.0, dt
