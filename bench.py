#!/usr/bin/env python3
"""XCodec encode throughput on MI355X (BASELINE.json metric).

Workload (BASELINE.json configs[1]): 4096 x 64 KiB chunks of
the survey generator (seed 0xC2, 50 % duplicate 2 KiB segments), each chunk
one independent XCodecEncoder::encode call with its own fresh
XCodecMemoryCache (XCG_SEM_INDEPENDENT).  A step = one batched encode launch
over all chunks; inputs, offsets and output slots are resident in HBM before
the timed region.  Output is bit-exact with the reference encoder (checked
against the CPU oracle on a sample every run).

Multi-GPU (torchrun, one rank per GPU): every rank encodes its own 4096-chunk
shard (seed 0xC2 + rank) with no collective in the timed loop -> weak scaling.

rank 0 prints ONE JSON line (see DESIGN.md "Measurement").
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

CHUNK = 65536
NCHUNKS = 4096
PEAK_HBM_GBS = 8000.0          # MI355X HBM3E peak, MI355X_MICROARCH.md "Chip-level parameters"


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument('--gpus', type=int, default=1)
    ap.add_argument('--steps', type=int, default=20)
    ap.add_argument('--warmup', type=int, default=3)
    ap.add_argument('--chunks', type=int, default=NCHUNKS)
    ap.add_argument('--no-cpu-baseline', action='store_true')
    ap.add_argument('--cpu-passes', type=int, default=8)
    ap.add_argument('--no-extras', action='store_true', help='skip the stream / decode / PCIe side measurements')
    ap.add_argument('--no-configs', action='store_true',
                    help='skip the C3 / C4 / C5 stream-configuration figures (scripts/configs_bench.py)')
    return ap.parse_args()


def cpu_baseline(data: np.ndarray, offs, lens, passes: int):
    """Reference XCodecEncoder (oracle/_ref, compiled from the reference
    sources) on this host's cores: contiguous chunk shards, one thread each,
    independent-chunk semantics (same output as the GPU run)."""
    from concurrent.futures import ThreadPoolExecutor
    from oracle.lib import Oracle
    kind = 'reference'
    try:
        o = Oracle(ref=True)
    except FileNotFoundError:
        o, kind = Oracle(), 'port'
    threads = max(1, min(16, os.cpu_count() or 1))
    n = offs.size
    shards = np.array_split(np.arange(n), threads)

    def run(idx):
        if idx.size:
            o.encode_batch(data, offs[idx], lens[idx], mode=0)

    total = 0
    t0 = time.perf_counter()
    with ThreadPoolExecutor(threads) as ex:
        for _ in range(passes):
            list(ex.map(run, shards))
            total += int(lens.astype(np.int64).sum())
    dt = time.perf_counter() - t0
    gib = total / 2**30
    return {'value': round(gib / dt, 4), 'unit': 'GiB/s', 'cores': threads, 'kind': kind,
            'sample': f'{passes} passes over the full {n} x 64 KiB batch ({total / 2**20:.0f} MiB), '
                      f'{threads} threads x contiguous shards, fresh XCodecMemoryCache per chunk; {dt:.1f} s wall'}


def pmc_traffic(n):
    """HBM bytes per launch of this kernel from the committed rocprofv3 PMC
    summary (scripts/profile.sh + scripts/prof_summary.py: FETCH_SIZE doubled
    per MI355X_MICROARCH.md "HBM", plus WRITE_SIZE), when it was taken on this
    same workload; PMC counters cannot be read from inside the timed run."""
    p = os.path.join(ROOT, 'profiles', 'r01_c2_independent_summary.json')
    if n != NCHUNKS or not os.path.exists(p):
        return None, None
    s = json.load(open(p))
    if 'hbm_traffic_bytes_per_launch' not in s:
        return None, None
    return int(s['hbm_traffic_bytes_per_launch']), 'profiles/r01_c2_independent_summary.json (rocprofv3 --pmc)'


def timed(fn, steps, stream):
    import torch
    for _ in range(2):
        fn()
    torch.cuda.synchronize()
    ev0 = torch.cuda.Event(enable_timing=True)
    ev1 = torch.cuda.Event(enable_timing=True)
    t0 = time.perf_counter()
    ev0.record(stream)
    for _ in range(steps):
        fn()
    ev1.record(stream)
    torch.cuda.synchronize()
    return (time.perf_counter() - t0) / steps, ev0.elapsed_time(ev1) / steps * 1e-3


def side_measurements(ctx, data, offs, lens, d_in, d_off, d_len, d_oo, d_out, d_ol, d_st, n, stream, dev, rank):
    """Same C2 batch under stream semantics (one cache, chunk order), its GPU
    decode, and the host-inclusive (PCIe) encode rate.  Each is checked."""
    import torch
    from oracle.lib import Oracle
    from wanproxy_amd.xcgpu import XCG_SEM_STREAM, Context
    in_bytes = int(lens.astype(np.int64).sum())
    res = {}
    # -- stream semantics: every step starts from an empty cache
    sctx = Context(dev.index, cache_segments=1 << 18)

    def s2():
        sctx.cache_clear()
        sctx.encode_batch_device(d_in, d_off, d_len, n, CHUNK, d_out, d_oo, d_ol, d_st, stream=stream,
                                 semantics=XCG_SEM_STREAM)
    wall, _ = timed(s2, 5, stream)
    sctx.status()
    ol = d_ol.cpu().numpy()
    outh = d_out.cpu().numpy()
    oo = d_oo.cpu().numpy()
    enc = [outh[int(oo[i]):int(oo[i]) + int(ol[i])].tobytes() for i in range(n)]
    k = min(n, 256)                       # sequential oracle on a prefix (same stream order)
    exp = Oracle().encode_batch(data, offs[:k], lens[:k], mode=1)
    if enc[:k] != exp:
        raise SystemExit('PARITY FAILURE (stream semantics)')
    res['stream_semantics'] = {'metric': 'XCodec encode GiB/s, one cache across the batch (tack loop order)',
                               'value': round(in_bytes / 2**30 / wall, 3), 'ms_per_step': round(wall * 1e3, 3),
                               'rounds': sctx.last_rounds(), 'out_in_ratio': round(int(ol.sum()) / in_bytes, 5),
                               'includes': 'cache clear + Jacobi rounds + commit'}
    # -- decode of that stream with a fresh decoder cache
    dctx = Context(dev.index, cache_segments=1 << 18)
    elens = ol.astype(np.uint32)
    eoffs = np.zeros(n, dtype=np.uint64)
    eoffs[1:] = np.cumsum(elens.astype(np.uint64))[:-1]
    blob = np.concatenate([np.frombuffer(e, np.uint8) for e in enc])
    d_enc = torch.from_numpy(blob).to(dev)
    d_eoff = torch.from_numpy(eoffs.view(np.int64)).to(dev)
    d_elen = torch.from_numpy(elens.view(np.int32)).to(dev)
    d_dout = torch.empty(in_bytes + 4096, dtype=torch.uint8, device=dev)
    d_doo = torch.zeros(n, dtype=torch.int64, device=dev)
    d_dol = torch.zeros(n, dtype=torch.int64, device=dev)
    d_dst = torch.zeros(n, dtype=torch.int32, device=dev)
    d_dcons = torch.zeros(n, dtype=torch.int64, device=dev)
    import ctypes as C
    from wanproxy_amd.xcgpu import _check, lib
    unk = np.zeros(16, np.uint64)
    nunk = np.zeros(1, np.uint32)
    tot = np.zeros(1, np.uint64)

    def dec():
        dctx.cache_clear()
        _check(lib().xcg_decode_batch(dctx.h, C.c_void_p(d_enc.data_ptr()), C.c_void_p(d_eoff.data_ptr()),
                                      C.c_void_p(d_elen.data_ptr()), n, int(elens.max()),
                                      C.c_void_p(d_dout.data_ptr()), d_dout.numel(), C.c_void_p(d_doo.data_ptr()),
                                      C.c_void_p(d_dol.data_ptr()), C.c_void_p(d_dst.data_ptr()),
                                      C.c_void_p(d_dcons.data_ptr()), unk.ctypes.data, unk.size, nunk.ctypes.data,
                                      tot.ctypes.data, C.c_void_p(stream.cuda_stream)))
    wall, _ = timed(dec, 5, stream)
    if int(tot[0]) != in_bytes or d_dout[:in_bytes].cpu().numpy().tobytes() != data.tobytes():
        raise SystemExit('PARITY FAILURE (decode round trip)')
    res['decode'] = {'metric': 'XCodec decode GiB/s of decoded bytes (that stream, fresh decoder cache)',
                     'value': round(in_bytes / 2**30 / wall, 3), 'ms_per_step': round(wall * 1e3, 3),
                     'includes': 'cache clear + scan + size + emit + commit, one host sync'}
    sctx.close()
    dctx.close()
    # -- host-inclusive independent encode: pinned H2D of the input, encode,
    #    pack the slots, D2H of exactly the encoded bytes
    ctx.encode_batch_device(d_in, d_off, d_len, n, CHUNK, d_out, d_oo, d_ol, d_st, stream=stream)
    torch.cuda.synchronize()
    enc_bytes = int(d_ol.sum().item())
    h_in = torch.from_numpy(data.copy()).pin_memory()
    h_out = torch.empty(enc_bytes, dtype=torch.uint8).pin_memory()
    d_packed = torch.empty(enc_bytes + 16, dtype=torch.uint8, device=dev)
    d_poff = torch.zeros(n, dtype=torch.int64, device=dev)
    d_ptot = torch.zeros(1, dtype=torch.int64, device=dev)

    def pcie():
        d_in.copy_(h_in, non_blocking=True)
        ctx.encode_batch_device(d_in, d_off, d_len, n, CHUNK, d_out, d_oo, d_ol, d_st, stream=stream)
        _check(lib().xcg_pack_outputs(ctx.h, C.c_void_p(d_out.data_ptr()), C.c_void_p(d_oo.data_ptr()),
                                      C.c_void_p(d_ol.data_ptr()), n, C.c_void_p(d_packed.data_ptr()),
                                      C.c_void_p(d_poff.data_ptr()), C.c_void_p(d_ptot.data_ptr()),
                                      C.c_void_p(stream.cuda_stream)))
        h_out.copy_(d_packed[:enc_bytes], non_blocking=True)
    wall, _ = timed(pcie, 5, stream)
    if int(d_ptot.item()) != enc_bytes:
        raise SystemExit('pack size mismatch')
    res['host_inclusive'] = {'metric': 'independent-chunk encode GiB/s incl. pinned H2D of input and D2H of output',
                             'value': round(in_bytes / 2**30 / wall, 3), 'ms_per_step': round(wall * 1e3, 3)}
    return res


def other_configs():
    """BASELINE.json's other configurations on this GPU (stream semantics,
    one cache; scripts/configs_bench.py): each figure is parity-checked
    against the oracle on a prefix and decoded back in full.  A failure is
    reported in the line, never hidden."""
    import importlib.util
    spec = importlib.util.spec_from_file_location('configs_bench', os.path.join(ROOT, 'scripts', 'configs_bench.py'))
    cb = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(cb)
    # C5-LRU: C5 on wanproxy.conf's bounded 128 MiB memory cache (LRU
    # eviction), every chunk checked against the oracle's bounded cache
    # C5-PAIR: C5 on wanproxy.conf's whole cache, the 128 MiB memory cache over
    # a 1 GiB disk (XCodecCachePair), every chunk checked against the oracle's pair
    a = argparse.Namespace(scale=1.0, reps=2, batch_mib=512, c4_batch=16384, lru_mib=128, lru_check=1.0,
                           disk_mib=1024, no_decode=False)
    out = {}
    for name, fn in (('C3', cb.run_c3), ('C4', cb.run_c4), ('C5', cb.run_c5), ('C5-LRU', cb.run_c5lru),
                     ('C5-PAIR', cb.run_c5pair)):
        try:
            out[name] = fn(a)
        except BaseException as e:          # SystemExit from a parity check included
            out[name] = {'error': f'{type(e).__name__}: {e}'}
    return out


def main():
    args = parse()
    import torch
    world = int(os.environ.get('WORLD_SIZE', '1'))
    rank = int(os.environ.get('RANK', '0'))
    local = int(os.environ.get('LOCAL_RANK', '0'))
    if world > 1:
        import torch.distributed as dist
        torch.cuda.set_device(local)
        dist.init_process_group('nccl', device_id=torch.device('cuda', local))
    else:
        torch.cuda.set_device(0)
    dev = torch.device('cuda', torch.cuda.current_device())

    from wanproxy_amd import synth
    from wanproxy_amd.xcgpu import Context

    n = args.chunks
    data = np.frombuffer(synth.stream(0xC2 + rank, n * CHUNK, 50, 0), dtype=np.uint8)
    offs, lens = synth.chunks_of(data.tobytes(), CHUNK)
    bounds = 2 * lens.astype(np.uint64) + 16
    oo = np.zeros(n, dtype=np.uint64)
    oo[1:] = np.cumsum(bounds)[:-1]

    d_in = torch.from_numpy(data.copy()).to(dev)
    d_off = torch.from_numpy(offs.view(np.int64)).to(dev)
    d_len = torch.from_numpy(lens.view(np.int32)).to(dev)
    d_oo = torch.from_numpy(oo.view(np.int64)).to(dev)
    d_out = torch.empty(int(bounds.sum()), dtype=torch.uint8, device=dev)
    d_ol = torch.zeros(n, dtype=torch.int64, device=dev)
    d_st = torch.zeros(4 * n, dtype=torch.int32, device=dev)
    ctx = Context(dev.index)
    stream = torch.cuda.current_stream(dev)

    def step():
        ctx.encode_batch_device(d_in, d_off, d_len, n, CHUNK, d_out, d_oo, d_ol, d_st, stream=stream)

    for _ in range(args.warmup):
        step()
    torch.cuda.synchronize(dev)
    ctx.status()

    # Parity check of this run's output against the CPU oracle (sampled chunks).
    from oracle.lib import Oracle
    ol = d_ol.cpu().numpy()
    sample = np.unique(np.linspace(0, n - 1, 16).astype(np.int64))
    exp = Oracle().encode_batch(data, offs[sample], lens[sample], mode=0)
    outh = d_out.cpu().numpy()
    for k, i in enumerate(sample):
        got = outh[int(oo[i]):int(oo[i]) + int(ol[i])].tobytes()
        if got != exp[k]:
            raise SystemExit(f'PARITY FAILURE on chunk {i}')
    out_bytes = int(ol.sum())
    in_bytes = int(lens.astype(np.int64).sum())

    if world > 1:
        torch.distributed.barrier()
    torch.cuda.synchronize(dev)
    ev0 = torch.cuda.Event(enable_timing=True)
    ev1 = torch.cuda.Event(enable_timing=True)
    t0 = time.perf_counter()
    ev0.record(stream)
    for _ in range(args.steps):
        step()
    ev1.record(stream)
    torch.cuda.synchronize(dev)
    if world > 1:
        torch.distributed.barrier()
    wall = time.perf_counter() - t0
    kern_ms = ev0.elapsed_time(ev1) / args.steps          # HIP events on the launch stream
    ctx.status()

    extras = {} if args.no_extras else side_measurements(ctx, data, offs, lens, d_in, d_off, d_len, d_oo, d_out, d_ol,
                                                          d_st, n, stream, dev, rank)

    from wanproxy_amd.shard import reduce_run
    wall, job_bytes = reduce_run(wall, in_bytes, device=dev)   # max wall, total bytes over ranks
    total_bytes = float(job_bytes) * args.steps
    value = total_bytes / 2**30 / wall

    if rank == 0:
        achieved = (in_bytes + out_bytes) / (kern_ms * 1e-3) / 1e9
        traffic, tsrc = pmc_traffic(n)
        line = {
            'metric': 'XCodec encode GiB/s device-resident, batched 64 KiB chunks, 1/2/4/8 GPU',
            'value': round(value, 3),
            'unit': 'GiB/s',
            'n_gpus': world,
            'steps': args.steps,
            'warmup': args.warmup,
            'ms_per_step': round(wall * 1e3 / args.steps, 4),
            'higher_is_better': True,
            'scaling': 'weak',
            'vs_baseline': None,
            'dtype': 'u8',
            'data': 'synthetic (survey splitmix64 generator, seed 0xC2+rank, 50% duplicate 2 KiB segments)',
            'config': {'workload': 'C2: 4096 x 64 KiB independent chunks per GPU, 50% dup segments, '
                                   'fresh XCodecMemoryCache per chunk (XCG_SEM_INDEPENDENT)',
                       'chunks_per_gpu': n, 'chunk_bytes': CHUNK, 'out_in_ratio': round(out_bytes / in_bytes, 5),
                       'parallelism': f'dp{world} (shard per GPU, no collective)'},
            'roofline': {'bound': 'hbm', 'achieved': round(achieved, 2), 'peak': PEAK_HBM_GBS, 'unit': 'GB/s',
                         'frac': round(achieved / PEAK_HBM_GBS, 5), 'traffic': traffic, 'traffic_source': tsrc,
                         'kernel': 'encode_independent_kernel', 'kernel_ms': round(kern_ms, 4),
                         'algorithmic_bytes_per_launch': in_bytes + out_bytes},
        }
        line.update(extras)
        if world == 1 and not args.no_extras and not args.no_configs:
            line['configs'] = other_configs()
        if world == 1 and not args.no_cpu_baseline:
            line['cpu_baseline'] = cpu_baseline(data, offs, lens, args.cpu_passes)
        print(json.dumps(line), flush=True)
    ctx.close()
    if world > 1:
        torch.distributed.destroy_process_group()


if __name__ == '__main__':
    main()
