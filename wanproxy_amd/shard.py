"""Data-parallel sharding for multi-GPU runs.

Each rank owns a contiguous range of work units (chunks / packets / 64 KiB
pieces of a long stream) and a PRIVATE XCodec cache -- the reference
equivalent is one XCodecEncoder + XCodecMemoryCache per shard, which is how
wanproxy runs independent codecs (programs/wanproxy/
wanproxy_config_class_codec.cc:39-80).  Nothing is exchanged while encoding;
the only collectives are the timing barrier and the max/sum reductions after
the timed region.
"""
from __future__ import annotations


def shard_range(n_units: int, world: int, rank: int) -> tuple[int, int]:
    """Contiguous [lo, hi) of rank `rank` out of `world` (sizes differ by <= 1)."""
    if world <= 0 or not 0 <= rank < world:
        raise ValueError('bad rank/world')
    q, r = divmod(n_units, world)
    lo = rank * q + min(rank, r)
    return lo, lo + q + (1 if rank < r else 0)


# BASELINE.json's partitioned datasets: ONE synthetic stream
# per configuration, cut into contiguous unit ranges, one per rank.
#   C4: 1 M x 4 KiB packets (seed 0xC4, dup 4), each packet one encode() call
#   C5: 8 GiB (seed 0xC5, dup 20) in 128 KiB encode() calls
DATASETS = {
    'C4': {'seed': 0xC4, 'dup': 4, 'unit': 4096, 'units': 1 << 20},
    'C5': {'seed': 0xC5, 'dup': 20, 'unit': 128 << 10, 'units': 65536},
}


# C5 "with xcodec_cache_disk spill" (BASELINE.json configs[4]): every rank's
# codec cache is wanproxy.conf's pair, a 128 MiB memory cache over a 1 GiB disk
# (programs/wanproxy/wanproxy.conf:8-26) -- one XCodecCachePair per shard.
C5_PAIR = {'memory_limit': 128 << 20, 'disk_bytes': 1 << 30}


def pair_geometry(scale: float = 1.0):
    """(memory limit bytes, disk bytes) of a C5-PAIR shard's cache, scaled with
    the data (--scale runs keep the cache-to-data ratio)."""
    f = min(1.0, scale * 8)
    return (max(2048, int(C5_PAIR['memory_limit'] * f)), max(1 << 20, int(C5_PAIR['disk_bytes'] * f)))


def config_shard(name: str, world: int, rank: int, scale: float = 1.0):
    """Rank `rank`'s share of dataset `name` split over `world` ranks:
    (seed, dup, unit bytes, first byte, end byte) of the one stream.  bench.py
    (--gpus N), scripts/configs_bench.py (N=1 runs one GPU's shard of 8) and
    tests/test_shard_gloo.py all cut the data through here."""
    d = DATASETS[name]
    units = max(world, int(d['units'] * scale))
    lo, hi = shard_range(units, world, rank)
    return d['seed'], d['dup'], d['unit'], lo * d['unit'], hi * d['unit']


def shard_data(name: str, world: int, rank: int, scale: float = 1.0):
    """The shard's bytes and its encode() calls (offsets relative to the
    shard): (data, offsets, lengths, (first byte, end byte) in the stream)."""
    import numpy as np
    from wanproxy_amd import synth
    seed, dup, unit, lo, hi = config_shard(name, world, rank, scale)
    data = synth.stream_range(seed, dup, 0, lo, hi)
    offs = np.arange(0, hi - lo, unit, dtype=np.uint64)
    lens = np.minimum(unit, (hi - lo) - offs.astype(np.int64)).astype(np.uint32)
    return data, offs, lens, (lo, hi)


def reduce_run(wall_s: float, bytes_done: int, device=None):
    """Whole-job (max wall over ranks, total bytes) -- identity without a
    process group."""
    import torch
    import torch.distributed as dist
    if not (dist.is_available() and dist.is_initialized()):
        return wall_s, bytes_done
    t = torch.tensor([wall_s], dtype=torch.float64, device=device)
    b = torch.tensor([float(bytes_done)], dtype=torch.float64, device=device)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    dist.all_reduce(b, op=dist.ReduceOp.SUM)
    return float(t.item()), int(b.item())
