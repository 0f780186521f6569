#!/usr/bin/env python3
"""Stream-semantics throughput on BASELINE.json's other configurations, one
GPU (the headline C2 independent-chunk line
is bench.py's).  Every figure is checked: a prefix against the CPU oracle
(sequential XCodecEncoder semantics from an empty cache) and the whole run by
a GPU decode round trip.

  c2s  4096 x 64 KiB, seed 0xC2, dup 50, one cache, chunk order (tack loop)
  c3   64 streams x 16 MiB (seeds 100..163, dup 5), chunks round-robin at
       64 KiB; untimed warm-up encode into one shared cache, then the timed
       re-encode against the warm cache, and the decode of that output with a
       decoder cache warmed by decoding the warm-up output
  c4   131072 x 4 KiB packets (one GPU's shard of 1 M), seed 0xC4, dup 4
  c5   1 GiB (one GPU's shard of 8 GiB) in 128 KiB chunks, seed 0xC5, dup 20,
       cold unbounded cache, batches of --batch-mib
  c5lru  c5 with a bounded --lru-mib (128) MiB LRU cache (wanproxy.conf's
       memory cache), checked against the oracle's bounded cache
  c5pair c5 with wanproxy.conf's XCodecCachePair: the --lru-mib memory cache
       over a --disk-mib (1024) MiB disk, checked against the oracle's pair

Prints one JSON line per config.  --scale shrinks the inputs (tests).
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

KiB, MiB = 1024, 1 << 20


class Batches:
    """Host data resident on the GPU, cut into encode() chunks, encoded in
    batches of `per` chunks with stream semantics on one context."""

    def __init__(self, ctx, data: np.ndarray, offs, lens, per: int):
        import torch
        self.ctx, self.per = ctx, per
        self.dev = torch.device('cuda', ctx.device)
        self.data = data
        self.offs = np.ascontiguousarray(offs, np.uint64)
        self.lens = np.ascontiguousarray(lens, np.uint32)
        n = self.offs.size
        self.n = n
        bounds = 2 * self.lens.astype(np.uint64) + 16
        self.oo = np.zeros(n, np.uint64)
        self.oo[1:] = np.cumsum(bounds)[:-1]
        self.d_in = torch.from_numpy(data).to(self.dev)
        self.d_off = torch.from_numpy(self.offs.view(np.int64)).to(self.dev)
        self.d_len = torch.from_numpy(self.lens.view(np.int32)).to(self.dev)
        self.d_oo = torch.from_numpy(self.oo.view(np.int64)).to(self.dev)
        self.d_out = torch.empty(int(bounds.sum()), dtype=torch.uint8, device=self.dev)
        self.d_ol = torch.zeros(n, dtype=torch.int64, device=self.dev)
        self.maxlen = int(self.lens.max())
        self.rounds = []

    def encode_all(self):
        from wanproxy_amd.xcgpu import XCG_SEM_STREAM
        self.rounds = []
        for a in range(0, self.n, self.per):
            b = min(self.n, a + self.per)
            self.ctx.encode_batch_device(self.d_in, self.d_off[a:b], self.d_len[a:b], b - a, self.maxlen,
                                         self.d_out, self.d_oo[a:b], self.d_ol[a:b], semantics=XCG_SEM_STREAM)
            self.rounds.append(self.ctx.last_rounds())

    def outputs(self):
        out = self.d_out.cpu().numpy()
        ol = self.d_ol.cpu().numpy()
        return [out[int(self.oo[i]):int(self.oo[i]) + int(ol[i])].tobytes() for i in range(self.n)]

    def out_bytes(self) -> int:
        return int(self.d_ol.sum().item())


def decode_device(ctx, encs, per: int, chunk: int, rehearse: bool = True):
    """Decode a list of encoded chunks (one stream) on ctx in batches of `per`;
    returns (decoded bytes, seconds of the timed decode).  rehearse: decode
    once untimed first (the context allocates its scratch then), clear the
    cache and time the second pass."""
    if rehearse:
        decode_device(ctx, encs, per, chunk, rehearse=False)
        ctx.cache_clear()
    import ctypes as C
    import torch
    from wanproxy_amd.xcgpu import _check, lib
    dev = torch.device('cuda', ctx.device)
    n = len(encs)
    lens = np.array([len(e) for e in encs], np.uint32)
    offs = np.zeros(n, np.uint64)
    offs[1:] = np.cumsum(lens.astype(np.uint64))[:-1]
    blob = np.frombuffer(b''.join(encs), np.uint8)
    d_enc = torch.from_numpy(blob.copy()).to(dev)
    d_eoff = torch.from_numpy(offs.view(np.int64)).to(dev)
    d_elen = torch.from_numpy(lens.view(np.int32)).to(dev)
    cap = per * chunk + 4096           # decoded bytes of one batch
    d_dout = torch.empty(n * chunk + 4096, dtype=torch.uint8, device=dev)   # every batch, back to back
    d_doo = torch.zeros(per, dtype=torch.int64, device=dev)
    d_dol = torch.zeros(per, dtype=torch.int64, device=dev)
    d_dst = torch.zeros(n, dtype=torch.int32, device=dev)
    d_dcons = torch.zeros(per, dtype=torch.int64, device=dev)
    unk = np.zeros(16, np.uint64)
    nunk = np.zeros(1, np.uint32)
    tot = np.zeros(1, np.uint64)
    maxlen = [int(lens[a:min(n, a + per)].max()) for a in range(0, n, per)]
    o, nbad = 0, 0
    torch.cuda.synchronize(dev)
    t0 = time.perf_counter()
    for k, a in enumerate(range(0, n, per)):
        b = min(n, a + per)
        _check(lib().xcg_decode_batch(ctx.h, C.c_void_p(d_enc.data_ptr()), C.c_void_p(d_eoff[a:].data_ptr()),
                                      C.c_void_p(d_elen[a:].data_ptr()), b - a, maxlen[k],
                                      C.c_void_p(d_dout.data_ptr() + o), min(cap, d_dout.numel() - o),
                                      C.c_void_p(d_doo.data_ptr()), C.c_void_p(d_dol.data_ptr()),
                                      C.c_void_p(d_dst[a:].data_ptr()), C.c_void_p(d_dcons.data_ptr()),
                                      unk.ctypes.data, unk.size, nunk.ctypes.data, tot.ctypes.data, None))
        nbad += int(nunk[0])
        o += int(tot[0])
    torch.cuda.synchronize(dev)
    secs = time.perf_counter() - t0
    st = d_dst.cpu().numpy()
    if (st != 0).any() or nbad:
        raise SystemExit(f'decode status {np.unique(st)} unknown {nbad}')
    return d_dout[:o].cpu().numpy().tobytes(), secs


def check_prefix(data, offs, lens, got, k, what, cache=None):
    """The first k chunks (None: all) equal the oracle's sequential encoder
    (from an empty cache, or `cache`)."""
    from oracle.lib import Oracle
    k = len(got) if k is None else min(k, len(got))
    exp = Oracle().encode_batch(data, offs[:k], lens[:k], mode=1, cache=cache)
    if got[:k] != exp:
        bad = next(i for i in range(k) if got[i] != exp[i])
        raise SystemExit(f'PARITY FAILURE ({what}) at chunk {bad}')
    return k


def checked(k, n, unit='chunks'):
    return f'all {n} {unit}' if k == n else f'first {k} of {n} {unit}'


class KernelClock:
    """Stream-parse kernel time (HIP events on its launch stream,
    xcg_debug_stream_kernel_timing) over a region: tells a change in the
    kernel from one in the host side around it."""

    def __enter__(self):
        from wanproxy_amd.xcgpu import lib, stream_kernel_time
        self.prev = lib().xcg_debug_stream_kernel_timing(1)
        stream_kernel_time()                      # (reset)
        return self

    def __exit__(self, *exc):
        from wanproxy_amd.xcgpu import lib, stream_kernel_time
        self.ms, self.launches = stream_kernel_time()
        lib().xcg_debug_stream_kernel_timing(self.prev)
        return False


def torch_dev(args) -> int:
    import torch
    return torch.cuda.current_device()


def timed_encode(B: 'Batches', reps: int, clear_ctx=True, reduce=None, clock=None):
    """Best of `reps` cold-cache encodes of the whole shard.  reduce: the
    multi-GPU run's max-over-ranks (a barrier precedes every rep).  clock
    (a dict): the last rep's stream-kernel ms and launches go there."""
    import torch
    walls = []
    for r in range(reps):
        if clear_ctx:
            B.ctx.cache_clear()
        torch.cuda.synchronize(B.dev)
        if reduce is not None:
            reduce(None)
        kc = KernelClock() if clock is not None and r == reps - 1 else None
        if kc:
            kc.__enter__()
        t0 = time.perf_counter()
        B.encode_all()
        torch.cuda.synchronize(B.dev)
        w = time.perf_counter() - t0
        if kc:
            kc.__exit__(None, None, None)
            clock.update(stream_kernel_ms=round(kc.ms, 3), stream_kernel_launches=kc.launches,
                         last_rep_wall_ms=round(w * 1e3, 3))
        walls.append(reduce(w) if reduce is not None else w)
    B.ctx.status()
    return min(walls)


def run_c2s(args):
    from wanproxy_amd import synth
    from wanproxy_amd.xcgpu import Context
    n = max(16, int(4096 * args.scale))
    data = np.frombuffer(synth.stream(0xC2, n * 64 * KiB, 50, 0), np.uint8).copy()
    offs, lens = synth.chunks_of(data.tobytes(), 64 * KiB)
    ctx = Context(0, cache_segments=args.c2s_segs)
    B = Batches(ctx, data, offs, lens, per=n)
    clock = {}
    wall = timed_encode(B, args.reps, clock=clock)
    got = B.outputs()
    k = check_prefix(data, offs, lens, got, None, 'c2s')
    dec, dsec = data.tobytes(), float('nan')
    if not args.no_decode:
        dctx = Context(0, cache_segments=1 << 18)
        dec, dsec = decode_device(dctx, got, per=n, chunk=64 * KiB)
    if dec != data.tobytes():
        raise SystemExit('ROUND TRIP FAILURE (c2s)')
    inb = data.size
    return {'config': 'C2-S2: %d x 64 KiB, dup 50, one cache, chunk order' % n,
            'encode_GiBps': round(inb / 2**30 / wall, 2), 'encode_ms': round(wall * 1e3, 3),
            'decode_GiBps': round(inb / 2**30 / dsec, 2), 'out_in': round(B.out_bytes() / inb, 5),
            'rounds': B.rounds, 'kernel': clock,
            'checked': f'{checked(k, len(got))} vs the oracle; full decode round trip'}


def run_c3(args):
    from wanproxy_amd import synth
    from wanproxy_amd.xcgpu import Context
    nstreams = 64
    per_stream = max(64 * KiB, int(16 * MiB * args.scale) // (64 * KiB) * 64 * KiB)
    streams = [np.frombuffer(synth.stream(100 + i, per_stream, 5, 0), np.uint8) for i in range(nstreams)]
    # round-robin: stream 0 chunk 0, stream 1 chunk 0, ...
    cps = per_stream // (64 * KiB)
    data = np.empty(nstreams * per_stream, np.uint8)
    offs = np.zeros(nstreams * cps, np.uint64)
    lens = np.full(nstreams * cps, 64 * KiB, np.uint32)
    o = 0
    for c in range(cps):
        for s in range(nstreams):
            i = c * nstreams + s
            data[o:o + 64 * KiB] = streams[s][c * 64 * KiB:(c + 1) * 64 * KiB]
            offs[i] = o
            o += 64 * KiB
    segs = int(data.size // 2048 * 1.05) + 4096
    ctx = Context(0, cache_segments=segs)
    per = 4096
    B = Batches(ctx, data, offs, lens, per=per)
    B.encode_all()                                   # warm-up (untimed)
    warm = B.outputs()
    warm_rounds = B.rounds
    import torch
    torch.cuda.synchronize(B.dev)
    with KernelClock() as kc:
        t0 = time.perf_counter()
        B.encode_all()                               # timed: against the warm cache
        torch.cuda.synchronize(B.dev)
        wall = time.perf_counter() - t0
    ctx.status()
    hot = B.outputs()
    # both passes against the oracle's sequential encoder on ONE cache: the
    # warm-up from empty, the timed re-encode against what the warm-up entered
    from oracle.lib import Oracle
    o = Oracle()
    oc = o.cache_new()
    k = check_prefix(data, offs, lens, warm, None, 'c3 warm-up', cache=oc)
    k2 = check_prefix(data, offs, lens, hot, None, 'c3 timed re-encode', cache=oc)
    o.cache_free(oc)
    dctx = Context(0, cache_segments=segs)
    dec0, _ = decode_device(dctx, warm, per=per, chunk=64 * KiB, rehearse=False)     # warms the decoder cache
    if dec0 != data.tobytes():
        raise SystemExit('ROUND TRIP FAILURE (c3 warm-up)')
    dec1, dsec = decode_device(dctx, hot, per=per, chunk=64 * KiB, rehearse=False)
    if dec1 != data.tobytes():
        raise SystemExit('ROUND TRIP FAILURE (c3 warm)')
    inb = data.size
    return {'config': 'C3: %d streams x %d MiB round-robin 64 KiB chunks, warm shared cache' % (nstreams, per_stream >> 20),
            'encode_GiBps': round(inb / 2**30 / wall, 2), 'encode_ms': round(wall * 1e3, 2),
            'decode_GiBps': round(inb / 2**30 / dsec, 2), 'out_in': round(B.out_bytes() / inb, 5),
            'warm_rounds': warm_rounds, 'rounds': B.rounds, 'batch_chunks': per,
            'kernel': {'stream_kernel_ms': round(kc.ms, 3), 'stream_kernel_launches': kc.launches},
            'checked': f'warm-up and timed re-encode: {checked(k2, len(hot))} each vs the oracle on one cache; '
                       'both passes decoded back to the input'}


def _shard(name, args):
    """This GPU's shard of dataset `name` (wanproxy_amd/shard.py): by default
    one GPU's share of the 8-GPU split (rank 0 of 8), or --world / --rank."""
    from wanproxy_amd.shard import shard_data
    return shard_data(name, getattr(args, 'world', 8), getattr(args, 'rank', 0), args.scale)


def _shard_desc(args, rng):
    return 'rank %d of %d: stream bytes [%d, %d)' % (getattr(args, 'rank', 0), getattr(args, 'world', 8), *rng)


def run_c4(args):
    from wanproxy_amd.xcgpu import Context
    data, offs, lens, rng = _shard('C4', args)
    n = offs.size
    dev = torch_dev(args)
    ctx = Context(dev, cache_segments=int(n * 2 * 1.05) + 4096)
    B = Batches(ctx, data, offs, lens, per=args.c4_batch)
    clock = {}
    wall = timed_encode(B, args.reps, reduce=getattr(args, 'reduce', None), clock=clock)
    got = B.outputs()
    k = check_prefix(data, offs, lens, got, getattr(args, 'check_c4', None), 'c4')
    dec, dsec = data.tobytes(), float('nan')
    if not args.no_decode:
        dctx = Context(dev, cache_segments=int(n * 2 * 1.05) + 4096)
        dec, dsec = decode_device(dctx, got, per=args.c4_batch, chunk=4 * KiB)
        dctx.close()
    if dec != data.tobytes():
        raise SystemExit('ROUND TRIP FAILURE (c4)')
    inb = data.size
    r = {'config': 'C4 shard: %d x 4 KiB packets, dup 4, one cache' % n, 'shard': _shard_desc(args, rng),
         'batch_chunks': args.c4_batch, 'in_bytes': inb, 'encode_wall_s': wall,
         'encode_GiBps': round(inb / 2**30 / wall, 2), 'encode_ms': round(wall * 1e3, 2),
         'decode_GiBps': round(inb / 2**30 / dsec, 2), 'out_in': round(B.out_bytes() / inb, 5),
         'rounds': B.rounds[:8], 'kernel': clock,
         'checked': f'{checked(k, len(got), "packets")} of the shard vs the oracle; full decode round trip'}
    ctx.close()
    return r


def run_c5(args):
    from wanproxy_amd.xcgpu import Context
    data, offs, lens, rng = _shard('C5', args)
    nbytes = data.size
    segs = nbytes // 2048 + 4096
    dev = torch_dev(args)
    ctx = Context(dev, cache_segments=segs)
    per = max(1, args.batch_mib * MiB // (128 * KiB))
    B = Batches(ctx, data, offs, lens, per=per)
    clock = {}
    wall = timed_encode(B, args.reps, reduce=getattr(args, 'reduce', None), clock=clock)
    got = B.outputs()
    k = check_prefix(data, offs, lens, got, getattr(args, 'check_c5', None), 'c5')
    dec, dsec = data.tobytes(), float('nan')
    if not args.no_decode:
        dctx = Context(dev, cache_segments=segs)
        dec, dsec = decode_device(dctx, got, per=per, chunk=128 * KiB)
        dctx.close()
    if dec != data.tobytes():
        raise SystemExit('ROUND TRIP FAILURE (c5)')
    inb = data.size
    r = {'config': 'C5 shard: %d MiB in 128 KiB chunks, dup 20, cold unbounded cache' % (nbytes >> 20),
         'shard': _shard_desc(args, rng), 'in_bytes': inb, 'encode_wall_s': wall,
         'batch_chunks': per, 'encode_GiBps': round(inb / 2**30 / wall, 2), 'encode_ms': round(wall * 1e3, 2),
         'decode_GiBps': round(inb / 2**30 / dsec, 2), 'out_in': round(B.out_bytes() / inb, 5),
         'rounds': B.rounds, 'kernel': clock,
         'checked': f'{checked(k, len(got))} of the shard vs the oracle; full decode round trip'}
    ctx.close()
    return r


def run_c5lru(args):
    """C5 with wanproxy.conf's primary cache: a bounded 128 MiB
    XCodecMemoryCache (LRU eviction) instead of an unbounded one."""
    from oracle.lib import Oracle
    from wanproxy_amd.xcgpu import Context
    data, offs, lens, rng = _shard('C5', args)
    nbytes = data.size
    limit = args.lru_mib * MiB
    ctx = Context(torch_dev(args), memory_cache_limit=limit)
    per = max(1, args.batch_mib * MiB // (128 * KiB))
    B = Batches(ctx, data, offs, lens, per=per)
    clock = {}
    wall = timed_encode(B, args.reps, clock=clock)
    got = B.outputs()
    k = min(len(got), max(64, int(args.lru_check * len(got))))
    o = Oracle()
    c = o.cache_new(limit)
    exp = o.encode_batch(data, offs[:k], lens[:k], mode=1, cache=c)
    o.cache_free(c)
    if got[:k] != exp:
        bad = next(i for i in range(k) if got[i] != exp[i])
        raise SystemExit(f'PARITY FAILURE (c5lru) at chunk {bad}')
    dec = data.tobytes()
    if not args.no_decode:
        dctx = Context(0, cache_segments=nbytes // 2048 + 4096)
        dec, _ = decode_device(dctx, got, per=per, chunk=128 * KiB)
    if dec != data.tobytes():
        raise SystemExit('ROUND TRIP FAILURE (c5lru)')
    inb = data.size
    return {'config': 'C5 shard: %d MiB in 128 KiB chunks, dup 20, bounded %d MiB LRU cache' % (nbytes >> 20,
                                                                                                 args.lru_mib),
            'batch_chunks': per, 'encode_GiBps': round(inb / 2**30 / wall, 2), 'encode_ms': round(wall * 1e3, 2),
            'out_in': round(B.out_bytes() / inb, 5), 'rounds': B.rounds, 'kernel': clock,
            'checked': f'{checked(k, len(got))} vs the oracle with the same bounded cache; '
                       'decoded back (unbounded decoder)'}


def run_c5pair(args):
    """C5 with wanproxy.conf's whole cache: XCodecCachePair of a bounded
    --lru-mib memory primary and a --disk-mib disk secondary
    (programs/wanproxy/wanproxy.conf:8-26; xcodec/xcodec_cache.h:140-237,
    xcodec/xcodec_cache_disk.cc), every chunk checked against the oracle's
    pair.  On N > 1 every rank runs its own pair over its shard (bench.py
    sharded_configs; wanproxy_amd/shard.py C5_PAIR).  --disk-laps: a smaller
    disk (the data laps it that many times), so FIFO eviction is in the figure."""
    from oracle.lib import Oracle
    from wanproxy_amd.xcgpu import Context
    data, offs, lens, rng = _shard('C5', args)
    nbytes = data.size
    limit = max(2048, int(args.lru_mib * MiB * min(1.0, args.scale * 8)))
    disk = max(1 << 20, int(args.disk_mib * MiB * min(1.0, args.scale * 8)))
    if getattr(args, 'disk_laps', 0):
        disk = max(1 << 20, int(nbytes * (1 - getattr(args, 'dup_hint', 0.2)) / args.disk_laps))
    ctx = Context(torch_dev(args), memory_cache_limit=limit, disk_bytes=disk)
    per = max(1, args.batch_mib * MiB // (128 * KiB))
    B = Batches(ctx, data, offs, lens, per=per)
    clock = {}
    wall = timed_encode(B, args.reps, reduce=getattr(args, 'reduce', None), clock=clock)
    got = B.outputs()
    st = ctx.pair_stats()
    k = min(len(got), max(64, int(args.lru_check * len(got))))
    o = Oracle()
    c = o.cache_new_pair(limit, disk)
    exp = o.encode_batch(data, offs[:k], lens[:k], mode=1, cache=c)
    ost = o.pair_stats(c) if k == len(got) else None
    o.cache_free(c)
    if got[:k] != exp:
        bad = next(i for i in range(k) if got[i] != exp[i])
        raise SystemExit(f'PARITY FAILURE (c5pair) at chunk {bad}')
    if ost is not None and ost != (st[1], st[2]):
        raise SystemExit(f'PARITY FAILURE (c5pair disk counters {st} vs {ost})')
    dec = data.tobytes()
    if not args.no_decode:
        dctx = Context(torch_dev(args), cache_segments=nbytes // 2048 + 4096)
        dec, _ = decode_device(dctx, got, per=per, chunk=128 * KiB)
        dctx.close()
    if dec != data.tobytes():
        raise SystemExit('ROUND TRIP FAILURE (c5pair)')
    ctx.close()
    inb = data.size
    d_entries = (disk // 2048 - 18) // 205 * 204
    return {'config': 'C5 shard: %d MiB in 128 KiB chunks, dup 20, XCodecCachePair(%d MiB LRU memory, %d MiB disk)'
                      % (nbytes >> 20, limit >> 20, disk >> 20),
            'shard': _shard_desc(args, rng), 'in_bytes': inb, 'encode_wall_s': wall,
            'batch_chunks': per, 'encode_GiBps': round(inb / 2**30 / wall, 2), 'encode_ms': round(wall * 1e3, 2),
            'out_in': round(B.out_bytes() / inb, 5), 'rounds': B.rounds, 'kernel': clock,
            'pair_stats': {'primary_entries': st[0], 'disk_entries': st[1], 'disk_written': st[2],
                           'disk_index_blocks': st[3], 'disk_laps': round(st[2] / max(1, d_entries), 2)},
            'checked': f'{checked(k, len(got))} and the disk counters vs the oracle with the same pair; '
                       'decoded back (unbounded decoder)'}


def run_c5dense(args):
    """The C5-PAIR cache (wanproxy.conf's pair, --lru-mib / --disk-mib) on
    REF-dense data: the shard's size drawn from a pool of --dense-pool
    segments (synth.dense), so an entity takes thousands of references per
    sub-batch -- the pair replay's long-run case.  Checked against the oracle's
    pair and decoded back."""
    from oracle.lib import Oracle
    from wanproxy_amd import synth
    from wanproxy_amd.xcgpu import Context
    nbytes = int(1 << 30 if args.scale >= 1 else max(1 << 22, int((1 << 30) * args.scale)))
    if args.dense_pool:
        data = np.frombuffer(synth.dense(0xC5D, nbytes, args.dense_pool), np.uint8).copy()
    else:                                            # --dense-pool 0: an all-zero stream
        data = np.zeros(nbytes, np.uint8)
    offs, lens = synth.chunks_of(data.tobytes(), 128 * KiB)
    limit = max(2048, int(args.lru_mib * MiB * min(1.0, args.scale * 8)))
    disk = max(1 << 20, int(args.disk_mib * MiB * min(1.0, args.scale * 8)))
    unb = args.dense_cache == 'unbounded'
    ctx = Context(torch_dev(args), cache_segments=1 << 20) if unb else \
        Context(torch_dev(args), memory_cache_limit=limit, disk_bytes=disk)
    per = max(1, args.batch_mib * MiB // (128 * KiB))
    B = Batches(ctx, data, offs, lens, per=per)
    clock = {}
    wall = timed_encode(B, args.reps, clock=clock)
    got = B.outputs()
    st = (0, 0, 0) if unb else ctx.pair_stats()
    k = min(len(got), max(64, int(args.lru_check * len(got))))
    o = Oracle()
    c = o.cache_new() if unb else o.cache_new_pair(limit, disk)
    exp = o.encode_batch(data, offs[:k], lens[:k], mode=1, cache=c)
    o.cache_free(c)
    if got[:k] != exp:
        bad = next(i for i in range(k) if got[i] != exp[i])
        raise SystemExit(f'PARITY FAILURE (c5dense) at chunk {bad}')
    dec = data.tobytes()
    if not args.no_decode:
        dctx = Context(torch_dev(args), cache_segments=max(1, args.dense_pool) + 4096)
        dec, _ = decode_device(dctx, got, per=per, chunk=128 * KiB)
        dctx.close()
    if dec != data.tobytes():
        raise SystemExit('ROUND TRIP FAILURE (c5dense)')
    ctx.close()
    inb = data.size
    what = 'from a pool of %d segments' % args.dense_pool if args.dense_pool else 'all zero bytes'
    cache = 'unbounded cache' if unb else 'XCodecCachePair(%d MiB LRU memory, %d MiB disk)' % (limit >> 20, disk >> 20)
    return {'config': 'REF-dense: %d MiB in 128 KiB chunks %s, %s' % (nbytes >> 20, what, cache),
            'batch_chunks': per, 'encode_GiBps': round(inb / 2**30 / wall, 2), 'encode_ms': round(wall * 1e3, 2),
            'out_in': round(B.out_bytes() / inb, 5), 'rounds': B.rounds, 'kernel': clock,
            'pair_stats': {'primary_entries': st[0], 'disk_entries': st[1], 'disk_written': st[2]},
            'checked': f'{checked(k, len(got))} vs the oracle with the same pair; decoded back'}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('configs', nargs='*', default=['c2s', 'c3', 'c4', 'c5'])
    ap.add_argument('--scale', type=float, default=1.0)
    ap.add_argument('--reps', type=int, default=3)
    ap.add_argument('--batch-mib', type=int, default=512)
    ap.add_argument('--c4-batch', type=int, default=65536)
    ap.add_argument('--c2s-segs', type=int, default=1 << 18, help='c2s: the context\'s cache capacity in segments')
    ap.add_argument('--lru-mib', type=int, default=128)
    ap.add_argument('--disk-mib', type=int, default=1024)
    ap.add_argument('--lru-check', type=float, default=1.0, help='share of c5lru chunks checked vs the oracle')
    ap.add_argument('--disk-laps', type=float, default=0, help='c5pair: size the disk so the data laps it')
    ap.add_argument('--dense-cache', default='pair', choices=['pair', 'unbounded'], help='c5dense: the cache')
    ap.add_argument('--dense-pool', type=int, default=4096, help='c5dense: distinct segments (0: all-zero data)')
    ap.add_argument('--no-decode', action='store_true', help='skip the decode round trips (profiling runs)')
    args = ap.parse_args()
    import torch
    torch.cuda.set_device(0)
    fns = {'c2s': run_c2s, 'c3': run_c3, 'c4': run_c4, 'c5': run_c5, 'c5lru': run_c5lru, 'c5pair': run_c5pair,
           'c5dense': run_c5dense}
    for c in args.configs:
        t0 = time.perf_counter()
        r = fns[c](args)
        r['wall_s'] = round(time.perf_counter() - t0, 1)
        print(json.dumps(r), flush=True)


if __name__ == '__main__':
    main()
