"""N > 1 path on CPU: world_size-2 gloo process group, contiguous shards with a
private cache each (the oracle stands in for a rank's GPU here), and the
timing / byte reductions bench.py uses."""
import os
import socket

import numpy as np
import pytest
import torch.multiprocessing as mp

from wanproxy_amd.shard import shard_range


def test_shard_range_covers():
    for n in (0, 1, 7, 4096, 1 << 20):
        for w in (1, 2, 3, 8):
            rs = [shard_range(n, w, r) for r in range(w)]
            assert rs[0][0] == 0 and rs[-1][1] == n
            assert all(rs[i][1] == rs[i + 1][0] for i in range(w - 1))
            assert max(b - a for a, b in rs) - min(b - a for a, b in rs) <= 1


def _free_port():
    s = socket.socket()
    s.bind(('127.0.0.1', 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, q):
    import torch.distributed as dist
    from oracle.lib import Oracle
    from wanproxy_amd import synth
    from wanproxy_amd.shard import reduce_run, shard_range
    os.environ['MASTER_ADDR'] = '127.0.0.1'
    os.environ['MASTER_PORT'] = str(port)
    dist.init_process_group('gloo', rank=rank, world_size=world)
    d = synth.stream(0xC4, 64 * 4096, 4, 0)
    offs, lens = synth.chunks_of(d, 4096)
    lo, hi = shard_range(offs.size, world, rank)
    dist.barrier()
    out = Oracle().encode_batch(d, offs[lo:hi], lens[lo:hi], mode=1)   # private cache per shard
    dist.barrier()
    wall, nbytes = reduce_run(0.1 * (rank + 1), int(lens[lo:hi].sum()))
    q.put((rank, lo, hi, [len(o) for o in out], wall, nbytes))
    dist.destroy_process_group()


@pytest.mark.timeout(120)
def test_two_rank_gloo_shards():
    ctx = mp.get_context('spawn')
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = sorted(q.get(timeout=100) for _ in procs)
    for p in procs:
        p.join(timeout=30)
        assert p.exitcode == 0
    (r0, lo0, hi0, l0, w0, b0), (r1, lo1, hi1, l1, w1, b1) = res
    assert (lo0, hi0, lo1, hi1) == (0, 32, 32, 64)
    assert w0 == w1 == pytest.approx(0.2) and b0 == b1 == 64 * 4096
    # each shard is an independent stream: rank 1's first packet sees an empty cache
    from oracle.lib import Oracle
    from wanproxy_amd import synth
    d = synth.stream(0xC4, 64 * 4096, 4, 0)
    offs, lens = synth.chunks_of(d, 4096)
    exp1 = Oracle().encode_batch(d, offs[32:], lens[32:], mode=1)
    assert l1 == [len(e) for e in exp1]
