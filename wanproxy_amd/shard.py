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
