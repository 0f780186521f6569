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


SCALE = 64 / (1 << 20)          # C4 at 64 packets; C5 at 8 chunks of 128 KiB


def _worker(rank, world, port, q):
    import torch.distributed as dist
    from oracle.lib import Oracle
    from wanproxy_amd.shard import reduce_run, shard_data
    os.environ['MASTER_ADDR'] = '127.0.0.1'
    os.environ['MASTER_PORT'] = str(port)
    dist.init_process_group('gloo', rank=rank, world_size=world)
    res = {}
    for name, scale in (('C4', SCALE), ('C5', 8 / 65536)):
        # the partition bench.py --gpus N uses (sharded_configs -> configs_bench -> shard_data)
        d, offs, lens, (lo, hi) = shard_data(name, world, rank, scale)
        dist.barrier()
        out = Oracle().encode_batch(d, offs, lens, mode=1)   # a private cache per shard
        dist.barrier()
        wall, nbytes = reduce_run(0.1 * (rank + 1), int(lens.astype(np.int64).sum()))
        res[name] = (lo, hi, d.tobytes(), [len(o) for o in out], wall, nbytes)
    # C5 "with xcodec_cache_disk spill": the same C5 shard on a private pair of
    # wanproxy.conf's geometry, scaled (bench.py sharded_configs -> run_c5pair).
    # A SLICING check only: the oracle stands in for the rank's GPU, so this
    # shows that shard_data cuts the pair's stream as bench.py does and that
    # each rank starts from an empty pair.  The GPU pair path per rank is
    # checked on the GPU (tests/test_gpu_pair.py) and, at N > 1, by bench.py's
    # sharded_configs, which compares every rank's output with the oracle.
    from wanproxy_amd.shard import pair_geometry
    d, offs, lens, _ = shard_data('C5', world, rank, 8 / 65536)
    o = Oracle()
    c = o.cache_new_pair(*pair_geometry(8 / 65536))
    out = o.encode_batch(d, offs, lens, mode=1, cache=c)
    res['C5-PAIR'] = ([len(x) for x in out], o.pair_stats(c))
    o.cache_free(c)
    q.put((rank, res))
    dist.destroy_process_group()


@pytest.mark.timeout(120)
def test_two_rank_gloo_shards():
    ctx = mp.get_context('spawn')
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = dict(q.get(timeout=100) for _ in procs)
    for p in procs:
        p.join(timeout=30)
        assert p.exitcode == 0
    from oracle.lib import Oracle
    from wanproxy_amd import synth
    for name, unit, seed, dup, units in (('C4', 4096, 0xC4, 4, 64), ('C5', 128 << 10, 0xC5, 20, 8)):
        (lo0, hi0, d0, l0, w0, b0), (lo1, hi1, d1, l1, w1, b1) = res[0][name], res[1][name]
        # contiguous ranges of ONE stream that tile it
        assert (lo0, hi0, lo1, hi1) == (0, units // 2 * unit, units // 2 * unit, units * unit)
        full = synth.stream(seed, units * unit, dup, 0)
        assert d0 + d1 == full
        assert w0 == w1 == pytest.approx(0.2) and b0 == b1 == units * unit
        # each shard is an independent stream: rank 1's first call sees an empty cache
        offs, lens = synth.chunks_of(full, unit)
        exp1 = Oracle().encode_batch(full, offs[units // 2:], lens[units // 2:], mode=1)
        assert l1 == [len(e) for e in exp1]
    # C5-PAIR: each rank's shard from an empty pair of the scaled geometry
    from wanproxy_amd.shard import pair_geometry
    full = synth.stream(0xC5, 8 * (128 << 10), 20, 0)
    offs, lens = synth.chunks_of(full, 128 << 10)
    o = Oracle()
    for r, sl in ((0, slice(0, 4)), (1, slice(4, 8))):
        c = o.cache_new_pair(*pair_geometry(8 / 65536))
        part = full[int(offs[sl][0]):int(offs[sl][-1] + lens[sl][-1])]
        po, pl = synth.chunks_of(part, 128 << 10)
        exp = o.encode_batch(part, po, pl, mode=1, cache=c)
        assert res[r]['C5-PAIR'] == ([len(e) for e in exp], o.pair_stats(c))
        o.cache_free(c)
