#!/usr/bin/env python3
"""XCodec encode throughput on MI355X (BASELINE.json metric).

Workload (BASELINE.json configs[1]): 4096 x 64 KiB chunks of
the survey generator (seed 0xC2, 50 % duplicate 2 KiB segments), each chunk
one independent XCodecEncoder::encode call with its own fresh
XCodecMemoryCache (XCG_SEM_INDEPENDENT).  A step = one batched encode launch
over all chunks; inputs, offsets and output slots are resident in HBM before
the timed region.  Output is bit-exact with the reference encoder: every run
checks ALL 4096 chunks against the CPU oracle (and the stream-semantics side
figure all 4096 too).

Multi-GPU (torchrun, one rank per GPU): every rank encodes its own 4096-chunk
shard (seed 0xC2 + rank) with no collective in the timed loop -> weak scaling.
With N > 1 the line also carries `sharded_configs`: BASELINE configs C4 (1 M x
4 KiB packets, a private unbounded cache per rank) and C5 (8 GiB in 128 KiB
calls, "cold cache with xcodec_cache_disk spill": a private XCodecCachePair of
wanproxy.conf's 128 MiB memory cache over a 1 GiB disk per rank), ONE stream
each cut into contiguous per-rank ranges (wanproxy_amd/shard.py config_shard),
every chunk of every shard checked against the oracle run on that shard alone.

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
    ap.add_argument('--gpus', type=int, default=None,
                    help='ranks (one per GPU); without an outer launcher N > 1 starts N ranks itself')
    ap.add_argument('--steps', type=int, default=20)
    ap.add_argument('--warmup', type=int, default=3)
    ap.add_argument('--chunks', type=int, default=NCHUNKS)
    ap.add_argument('--no-cpu-baseline', action='store_true')
    ap.add_argument('--cpu-seconds', type=float, default=10.0,
                    help='minimum wall of the headline CPU baseline (the reference on T threads)')
    ap.add_argument('--no-extras', action='store_true', help='skip the stream / decode / PCIe side measurements')
    ap.add_argument('--no-configs', action='store_true',
                    help='skip the C3 / C4 / C5 stream-configuration figures (scripts/configs_bench.py)')
    ap.add_argument('--no-zlib', action='store_true', help='skip the zlib stage figures (scripts/zlib_bench.py)')
    ap.add_argument('--dist-backend', default='nccl',
                    help='torch.distributed backend for N > 1 (nccl = RCCL; gloo rehearses the N > 1 path with '
                         'several ranks sharing one GPU: device = LOCAL_RANK mod the visible GPUs)')
    return ap.parse_args()


def host_cpus():
    """This host's CPUs: nproc, the affinity set, the cgroup quota, the model,
    and the threads the CPU baselines use -- the share of the machine this
    process may use (affinity, cgroup quota and OMP_NUM_THREADS, the GPU box's
    per-GPU CPU share), not the whole machine's nproc."""
    nproc = os.cpu_count() or 1
    try:
        aff = len(os.sched_getaffinity(0))
    except AttributeError:
        aff = nproc
    quota = None
    try:
        q, per = open('/sys/fs/cgroup/cpu.max').read().split()
        if q != 'max':
            quota = int(q) / int(per)
    except (OSError, ValueError):
        pass
    model = ''
    try:
        for ln in open('/proc/cpuinfo'):
            if ln.startswith('model name'):
                model = ln.split(':', 1)[1].strip()
                break
    except OSError:
        pass
    t = aff
    if quota:
        t = min(t, max(1, int(quota)))
    if os.environ.get('OMP_NUM_THREADS', '').isdigit():
        t = min(t, int(os.environ['OMP_NUM_THREADS']))
    return {'nproc': nproc, 'affinity': aff, 'cgroup_cpus': quota, 'omp_num_threads': os.environ.get('OMP_NUM_THREADS'),
            'model': model, 'threads': max(1, t)}


def _threads_rate(o, jobs, threads, min_s):
    """Run `jobs` (callables returning bytes encoded) on `threads` threads,
    repeating the whole set until min_s have passed; GiB/s over the wall."""
    from concurrent.futures import ThreadPoolExecutor
    total, t0 = 0, time.perf_counter()
    with ThreadPoolExecutor(threads) as ex:
        while True:
            total += sum(ex.map(lambda f: f(), jobs))
            dt = time.perf_counter() - t0
            if dt >= min_s:
                break
    return total / 2**30 / dt, total, dt


def cpu_baseline(data: np.ndarray, offs, lens, min_s: float = 10.0):
    """The reference XCodecEncoder (oracle/_ref, compiled from the reference
    sources; the C restatement if that is absent) on this host's cores, same
    semantics and inputs as the GPU figures.  Headline: independent chunks
    (S1) on T threads x contiguous shards, repeated over the batch for >=
    min_s.  `extra`: S1 on one thread, the S2 tack loop (one encoder + cache,
    programs/tack/tack.cc:298-321 -- inherently one thread), and bounded
    samples of C3 / C4 / C5 on one thread and (C4 / C5, a private cache per
    thread as per GPU) on T threads."""
    from oracle.lib import Oracle
    kind = 'reference'
    try:
        o = Oracle(ref=True)
    except FileNotFoundError:
        o, kind = Oracle(), 'port'
    hc = host_cpus()
    T = hc['threads']
    n = offs.size
    shards = [idx for idx in np.array_split(np.arange(n), T) if idx.size]

    def s1_job(idx):
        return lambda: (o.encode_batch(data, offs[idx], lens[idx], mode=0), int(lens[idx].astype(np.int64).sum()))[1]
    v, tot, dt = _threads_rate(o, [s1_job(i) for i in shards], T, min_s)
    res = {'value': round(v, 4), 'unit': 'GiB/s', 'cores': T, 'kind': kind,
           'sample': f'S1 (independent chunks): the full {n} x 64 KiB C2 batch repeated to {tot / 2**30:.1f} GiB, '
                     f'{T} threads x contiguous shards, fresh XCodecMemoryCache per chunk; {dt:.1f} s wall',
           'host': hc}
    extra = {}
    first = np.arange(min(n, 256))
    v1, tot, dt = _threads_rate(o, [s1_job(first)], 1, 3.0)
    extra['S1_1thread'] = {'value': round(v1, 4), 'unit': 'GiB/s', 'sample': f'{tot >> 20} MiB, {dt:.1f} s'}
    t0 = time.perf_counter()
    o.encode_batch(data, offs, lens, mode=1)
    dt = time.perf_counter() - t0
    extra['S2_1thread'] = {'value': round(int(lens.astype(np.int64).sum()) / 2**30 / dt, 4), 'unit': 'GiB/s',
                           'sample': f'the full C2 batch as one tack loop (one encoder + cache), {dt:.1f} s'}
    extra.update(cpu_configs(o, T))
    res['extra'] = extra
    return res


def cpu_configs(o, T):
    """C3 / C4 / C5 on the CPU reference, bounded samples of the GPU figures'
    workloads (scripts/configs_bench.py)."""
    from wanproxy_amd import synth
    from wanproxy_amd.shard import shard_data
    out = {}
    # C3: 16 of the 64 streams x 16 MiB (seeds 100..115, dup 5), round-robin
    # 64 KiB calls, warm-up encode then the timed re-encode on the warm cache
    ns, per = 16, 16 << 20
    streams = [np.frombuffer(synth.stream(100 + i, per, 5, 0), np.uint8) for i in range(ns)]
    data = np.stack([st.reshape(-1, 65536) for st in streams], 1).reshape(-1).copy()
    offs = np.arange(0, data.size, 65536, dtype=np.uint64)
    lens = np.full(data.size // 65536, 65536, np.uint32)
    c = o.cache_new()
    o.encode_batch(data, offs, lens, mode=1, cache=c)
    t0 = time.perf_counter()
    o.encode_batch(data, offs, lens, mode=1, cache=c)
    dt = time.perf_counter() - t0
    o.cache_free(c)
    out['C3_1thread'] = {'value': round(data.size / 2**30 / dt, 4), 'unit': 'GiB/s',
                         'sample': f'{ns} streams x 16 MiB round-robin, warm shared cache, {dt:.1f} s'}
    for name, k1 in (('C4', 8192), ('C5', 512)):
        d, offs, lens, _ = shard_data(name, 8, 0)
        unit = int(lens[0])
        t0 = time.perf_counter()
        o.encode_batch(d, offs[:k1], lens[:k1], mode=1)
        dt = time.perf_counter() - t0
        out[f'{name}_1thread'] = {'value': round(k1 * unit / 2**30 / dt, 4), 'unit': 'GiB/s',
                                  'sample': f'first {k1} calls of the rank-0 shard ({k1 * unit >> 20} MiB), cold '
                                            f'cache, {dt:.1f} s'}
        kt = max(1, min(offs.size // T, k1 // 2))
        jobs = [(lambda a: (lambda: (o.encode_batch(d, offs[a:a + kt], lens[a:a + kt], mode=1), kt * unit)[1]))(
            t * kt) for t in range(T)]
        v, tot, dt = _threads_rate(o, jobs, T, 0.0)
        out[f'{name}_{T}threads'] = {'value': round(v, 4), 'unit': 'GiB/s',
                                     'sample': f'{T} threads x {kt} calls ({kt * unit >> 20} MiB) each, a private '
                                               f'cold cache per thread (as per GPU), {dt:.1f} s'}
    return out


def pmc_traffic(n):
    """HBM bytes per launch of this kernel from the committed rocprofv3 PMC
    summary (scripts/profile.sh + scripts/prof_summary.py: FETCH_SIZE doubled
    per MI355X_MICROARCH.md "HBM", plus WRITE_SIZE), when it was taken on this
    same workload; PMC counters cannot be read from inside the timed run."""
    for name in ('r06_c2_independent_summary.json', 'r05_c2_independent_summary.json', 'r04_c2_independent_summary.json',
                 'r03_c2_independent_summary.json', 'r02_c2_independent_summary.json',
                 'r01_c2_independent_summary.json'):
        p = os.path.join(ROOT, 'profiles', name)
        if n != NCHUNKS or not os.path.exists(p):
            continue
        s = json.load(open(p))
        if 'hbm_traffic_bytes_per_launch' in s:
            return int(s['hbm_traffic_bytes_per_launch']), f'profiles/{name} (rocprofv3 --pmc)'
    return None, None


def pmc_stream_traffic():
    """HBM bytes of the seeded C2-S2 stream-parse launch (the bench's S2 step)
    from the committed scripts/profile_stream.sh summary."""
    for name in ('r06_stream_pmc_summary.json', 'r05_stream_pmc_summary.json', 'r04_stream_pmc_summary.json',
                 'r03_stream_pmc_summary.json',
                 'r02_stream_pmc_summary.json'):
        p = os.path.join(ROOT, 'profiles', name)
        if not os.path.exists(p):
            continue
        g = json.load(open(p)).get('c2s_seeded', {})
        if 'hbm_bytes' in g:
            return int(g['hbm_bytes'] / max(1, g['dispatches'])), f'profiles/{name} c2s_seeded (rocprofv3 --pmc)'
    return None, None


def pmc_decode_traffic():
    """HBM bytes of one C2-S2 batch decode (every decode kernel of one call)
    from the committed scripts/profile_decode.sh summary."""
    p = os.path.join(ROOT, 'profiles', 'r06_decode_summary.json')
    if os.path.exists(p):
        g = json.load(open(p)).get('decode_step', {})
        if 'hbm_bytes_per_call' in g:
            return int(g['hbm_bytes_per_call']), 'profiles/r06_decode_summary.json decode_step (rocprofv3 --pmc)'
    return None, None


def timed(fn, steps, stream, kernel_time=False):
    """(wall s / step, HIP-event s / step on `stream`, stream-parse kernel ms /
    step, its launches / step) over `steps` calls after 2 untimed ones."""
    import torch
    from wanproxy_amd.xcgpu import lib, stream_kernel_time
    for _ in range(2):
        fn()
    torch.cuda.synchronize()
    if kernel_time:
        lib().xcg_debug_stream_kernel_timing(1)
        stream_kernel_time()                       # (drop anything earlier)
    ev0 = torch.cuda.Event(enable_timing=True)
    ev1 = torch.cuda.Event(enable_timing=True)
    t0 = time.perf_counter()
    ev0.record(stream)
    for _ in range(steps):
        fn()
    ev1.record(stream)
    torch.cuda.synchronize()
    wall = (time.perf_counter() - t0) / steps
    kms, kl = 0.0, 0
    if kernel_time:
        lib().xcg_debug_stream_kernel_timing(0)
        kms, kl = stream_kernel_time()
    return wall, ev0.elapsed_time(ev1) / steps * 1e-3, kms / steps, kl / steps


def oracle_all(data, offs, lens, mode, threads=None):
    """The CPU oracle over every chunk (independent chunks split over threads;
    a stream is one sequential walk)."""
    from concurrent.futures import ThreadPoolExecutor
    from oracle.lib import Oracle
    o = Oracle()
    if mode == 1:
        return o.encode_batch(data, offs, lens, mode=1)
    parts = [p for p in np.array_split(np.arange(offs.size), threads or host_cpus()['threads']) if p.size]
    with ThreadPoolExecutor(len(parts)) as ex:
        res = list(ex.map(lambda idx: o.encode_batch(data, offs[idx], lens[idx], mode=0), parts))
    return [e for r in res for e in r]


def side_measurements(ctx, data, offs, lens, d_in, d_off, d_len, d_oo, d_out, d_ol, d_st, n, stream, dev, rank):
    """Same C2 batch under stream semantics (one cache, chunk order), its GPU
    decode, the host-inclusive (PCIe) encode rate, and the drop-in's per-call
    tack loop.  Each is checked."""
    import torch
    from wanproxy_amd.xcgpu import XCG_SEM_STREAM, Context
    in_bytes = int(lens.astype(np.int64).sum())
    res = {}
    # -- stream semantics: every step starts from an empty cache
    sctx = Context(dev.index, cache_segments=1 << 18)

    def s2():
        sctx.cache_clear()
        sctx.encode_batch_device(d_in, d_off, d_len, n, CHUNK, d_out, d_oo, d_ol, d_st, stream=stream,
                                 semantics=XCG_SEM_STREAM)
    wall, _, kms, kl = timed(s2, 5, stream, kernel_time=True)
    sctx.status()
    ol = d_ol.cpu().numpy()
    outh = d_out.cpu().numpy()
    oo = d_oo.cpu().numpy()
    enc = [outh[int(oo[i]):int(oo[i]) + int(ol[i])].tobytes() for i in range(n)]
    exp = oracle_all(data, offs, lens, mode=1)        # every chunk, sequential oracle (same stream order)
    if enc != exp:
        bad = next(i for i in range(n) if enc[i] != exp[i])
        raise SystemExit(f'PARITY FAILURE (stream semantics) at chunk {bad}')
    out_bytes = int(ol.sum())
    ach = (in_bytes + out_bytes) / (kms * 1e-3) / 1e9
    res['stream_semantics'] = {
        'metric': 'XCodec encode GiB/s, one cache across the batch (tack loop order)',
        'value': round(in_bytes / 2**30 / wall, 3), 'ms_per_step': round(wall * 1e3, 3),
        'rounds': sctx.last_rounds(), 'out_in_ratio': round(out_bytes / in_bytes, 5),
        'includes': 'cache clear + tiling seed + Jacobi rounds + verification + commit',
        'checked': f'all {n} chunks vs the sequential oracle',
        'roofline': {'bound': 'hbm', 'achieved': round(ach, 2), 'peak': PEAK_HBM_GBS, 'unit': 'GB/s',
                     'frac': round(ach / PEAK_HBM_GBS, 5),
                     'frac_read': round(in_bytes / (kms * 1e-3) / 1e9 / PEAK_HBM_GBS, 5),
                     'kernel': 'encode_stream_kernel', 'kernel_ms_per_step': round(kms, 4),
                     'launches_per_step': kl, 'algorithmic_bytes_per_step': in_bytes + out_bytes,
                     'traffic': pmc_stream_traffic()[0], 'traffic_source': pmc_stream_traffic()[1]}}
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
    wall, _, _, _ = timed(dec, 5, stream)
    # device time of the decode kernels: HIP events around each device segment
    # of 5 more calls (after the warm-up ones above)
    step_ms, emit_ms, segs = C.c_double(), C.c_double(), C.c_uint32()
    lib().xcg_debug_decode_kernel_time(None, None, None)
    lib().xcg_debug_decode_kernel_timing(1)
    for _ in range(5):
        dec()
    torch.cuda.synchronize()
    lib().xcg_debug_decode_kernel_timing(0)
    lib().xcg_debug_decode_kernel_time(C.byref(step_ms), C.byref(emit_ms), C.byref(segs))
    calls = max(1, segs.value // 3)                   # (three device segments per decode call)
    if int(tot[0]) != in_bytes or d_dout[:in_bytes].cpu().numpy().tobytes() != data.tobytes():
        raise SystemExit('PARITY FAILURE (decode round trip)')
    # Roofline (decode): algorithmic bytes = encoded bytes read + decoded bytes written.
    dms, ems = step_ms.value / calls, emit_ms.value / calls
    alg = out_bytes + in_bytes
    traffic, tsrc = pmc_decode_traffic()
    res['decode'] = {'metric': 'XCodec decode GiB/s of decoded bytes (that stream, fresh decoder cache)',
                     'value': round(in_bytes / 2**30 / wall, 3), 'ms_per_step': round(wall * 1e3, 3),
                     'includes': 'cache clear + scan + size + emit + commit, two host readbacks (sizes)',
                     'roofline': {'bound': 'hbm', 'achieved': round(alg / (dms * 1e-3) / 1e9, 2), 'peak': PEAK_HBM_GBS,
                                  'unit': 'GB/s', 'frac': round(alg / (dms * 1e-3) / 1e9 / PEAK_HBM_GBS, 5),
                                  'kernel': 'decode step: scan + refcheck/sizing + emit + commit kernels '
                                            '(HIP events per device segment, host readbacks excluded)',
                                  'kernel_ms_per_step': round(dms, 4), 'emit_kernel_ms': round(ems, 4),
                                  'emit_frac': round(alg / (ems * 1e-3) / 1e9 / PEAK_HBM_GBS, 5) if ems else None,
                                  'algorithmic_bytes_per_step': alg, 'traffic': traffic, 'traffic_source': tsrc}}
    sctx.close()
    dctx.close()
    del d_enc, d_dout
    res['host_inclusive'] = host_inclusive(ctx, data, offs, lens, d_in, d_off, d_len, d_oo, d_out, d_ol, n, dev)
    res['tack_loop'] = tack_loop(data, offs, lens)
    return res


def host_inclusive(ctx, data, offs, lens, d_in, d_off, d_len, d_oo, d_out, d_ol, n, dev, nsub=8, zero_copy=True):
    """Independent-chunk encode from pinned host memory to pinned host memory:
    H2D of the input, encode, pack, D2H of exactly the encoded bytes -- cut
    into `nsub` sub-batches pipelined over three HIP streams (copy in /
    compute / copy out), so the two PCIe directions and the kernels overlap.
    The host learns each sub-batch's packed size (zero_copy: the pack kernel
    writes it straight into pinned host memory; else an 8-byte readback on the
    compute stream) and issues its D2H then; checked byte for byte against the
    device result."""
    import ctypes as C
    import torch
    from wanproxy_amd.xcgpu import _check, lib
    per = (n + nsub - 1) // nsub
    subs = [(a, min(n, a + per)) for a in range(0, n, per)]
    bnd = [(int(offs[a]), int(offs[b - 1]) + int(lens[b - 1])) for a, b in subs]
    h_in = torch.from_numpy(data.copy()).pin_memory()
    slot = [(int(d_oo[a].item()), int(d_oo[b - 1].item()) + 2 * CHUNK + 16) for a, b in subs]
    d_packed = torch.empty(int(d_out.numel()) + 16, dtype=torch.uint8, device=dev)
    d_poff = torch.zeros(n, dtype=torch.int64, device=dev)
    d_ptot = torch.zeros(len(subs), dtype=torch.int64, device=dev)
    h_tot = torch.zeros(len(subs), dtype=torch.int64).pin_memory()
    h_out = torch.empty(int(d_out.numel()), dtype=torch.uint8).pin_memory()
    s_in, s_cmp, s_out = torch.cuda.Stream(dev), torch.cuda.Stream(dev), torch.cuda.Stream(dev)
    ev_in = [torch.cuda.Event() for _ in subs]
    ev_c = [torch.cuda.Event() for _ in subs]
    L = lib()
    sizes = [0] * len(subs)

    def run():
        for i, (a, b) in enumerate(subs):
            x0, x1 = bnd[i]
            with torch.cuda.stream(s_in):
                d_in[x0:x1].copy_(h_in[x0:x1], non_blocking=True)
                ev_in[i].record(s_in)
            s_cmp.wait_event(ev_in[i])
            ctx.encode_batch_device(d_in, d_off[a:b], d_len[a:b], b - a, CHUNK, d_out, d_oo[a:b], d_ol[a:b],
                                    stream=s_cmp)
            p0 = slot[i][0]
            tot_ptr = h_tot[i:].data_ptr() if zero_copy else d_ptot[i:].data_ptr()
            _check(L.xcg_pack_outputs(ctx.h, C.c_void_p(d_out.data_ptr()), C.c_void_p(d_oo[a:].data_ptr()),
                                      C.c_void_p(d_ol[a:].data_ptr()), b - a, C.c_void_p(d_packed.data_ptr() + p0),
                                      C.c_void_p(d_poff[a:].data_ptr()), C.c_void_p(tot_ptr),
                                      C.c_void_p(s_cmp.cuda_stream)))
            with torch.cuda.stream(s_cmp):
                if not zero_copy:
                    h_tot[i:i + 1].copy_(d_ptot[i:i + 1], non_blocking=True)
                ev_c[i].record(s_cmp)
        o = 0
        for i in range(len(subs)):
            ev_c[i].synchronize()
            sz = int(h_tot[i])
            sizes[i] = sz
            s_out.wait_event(ev_c[i])
            with torch.cuda.stream(s_out):
                h_out[o:o + sz].copy_(d_packed[slot[i][0]:slot[i][0] + sz], non_blocking=True)
            o += sz
        s_out.synchronize()
        return o

    run()
    torch.cuda.synchronize(dev)
    walls = []
    for _ in range(5):
        t0 = time.perf_counter()
        tot = run()
        walls.append(time.perf_counter() - t0)
    wall = sorted(walls)[len(walls) // 2]
    ol = d_ol.cpu().numpy()
    oo = d_oo.cpu().numpy()
    dout = d_out.cpu().numpy()
    want = b''.join(dout[int(oo[i]):int(oo[i]) + int(ol[i])].tobytes() for i in range(n))
    if tot != len(want) or h_out[:tot].numpy().tobytes() != want:
        raise SystemExit('host-inclusive output differs from the device-resident encode')
    in_bytes = int(lens.astype(np.int64).sum())
    # the link's own ceiling on this box: plain pinned copies of the same sizes,
    # each direction alone and both at once (two streams)
    def copy_rate(h2d, d2h):
        torch.cuda.synchronize(dev)
        t0 = time.perf_counter()
        for _ in range(3):
            if h2d:
                with torch.cuda.stream(s_in):
                    d_in.copy_(h_in, non_blocking=True)
            if d2h:
                with torch.cuda.stream(s_out):
                    h_out[:tot].copy_(d_packed[:tot], non_blocking=True)
        torch.cuda.synchronize(dev)
        return ((in_bytes if h2d else 0) + (tot if d2h else 0)) * 3 / (time.perf_counter() - t0) / 1e9
    link = {'h2d_GBps': round(copy_rate(True, False), 1), 'd2h_GBps': round(copy_rate(False, True), 1),
            'both_GBps': round(copy_rate(True, True), 1)}
    return {'metric': 'independent-chunk encode GiB/s incl. pinned H2D of input and D2H of the packed output',
            'value': round(in_bytes / 2**30 / wall, 3), 'ms_per_step': round(wall * 1e3, 3),
            'pcie_GBps': round((in_bytes + tot) / wall / 1e9, 2), 'sub_batches': len(subs),
            'link_copies_only': link,
            'includes': 'H2D + encode + pack + size readback + D2H, 3 streams (median of 5)',
            'size_readback': 'pack kernel writes pinned host memory' if zero_copy else '8-byte D2H per sub-batch'}


def tack_loop(data, offs, lens, ncalls=1024):
    """The drop-in path as tack calls it (programs/tack/tack.cc:298-321): one
    XCodecEncoder::encode per 64 KiB read on one encoder + cache, through the
    reference's own driver and Buffer classes with integration/'s encoder over
    the GPU engine (oracle/_ref/libxcdropin.so), beside the compiled reference
    (libxcref.so) on the same calls; outputs must be identical."""
    from oracle.lib import Oracle
    try:
        gpu, ref = Oracle(dropin=True), Oracle(ref=True)
    except FileNotFoundError as e:
        return {'error': f'not built: {e}'}
    k = min(ncalls, offs.size)
    res, outs = {}, {}
    for name, o in (('gpu_dropin', gpu), ('reference_cpu', ref)):
        o.encode_batch(data, offs[:8], lens[:8], mode=1)       # (warm: HIP init, allocations)
        t0 = time.perf_counter()
        outs[name] = o.encode_batch(data, offs[:k], lens[:k], mode=1)
        dt = time.perf_counter() - t0
        b = int(lens[:k].astype(np.int64).sum())
        res[name] = {'us_per_call': round(dt / k * 1e6, 1), 'GiBps': round(b / 2**30 / dt, 3)}
    if outs['gpu_dropin'] != outs['reference_cpu']:
        raise SystemExit('PARITY FAILURE (drop-in tack loop vs the reference)')
    # tack -d: one XCodecDecoder::decode per encoded call output, one decoder + cache
    encs = outs['reference_cpu']
    decs = {}
    for name, o in (('gpu_dropin', gpu), ('reference_cpu', ref)):
        c = o.cache_new()
        dec = o.decoder_new(c)
        o.decode(encs[0], c, decoder=dec)                        # (warm)
        o.decoder_free(dec)
        o.cache_free(c)
        c = o.cache_new()
        dec = o.decoder_new(c)
        t0 = time.perf_counter()
        got = [o.decode(e, c, decoder=dec, out_cap=2 * CHUNK) for e in encs]
        dt = time.perf_counter() - t0
        o.decoder_free(dec)
        o.cache_free(c)
        decs[name] = got
        b = int(lens[:k].astype(np.int64).sum())
        res[name].update({'decode_us_per_call': round(dt / k * 1e6, 1), 'decode_GiBps': round(b / 2**30 / dt, 3)})
    if decs['gpu_dropin'] != decs['reference_cpu'] or b''.join(r[1] for r in decs['gpu_dropin']) != \
            data[:int(lens[:k].astype(np.int64).sum())].tobytes():
        raise SystemExit('PARITY FAILURE (drop-in tack decode loop vs the reference)')
    res.update({'calls': k, 'call_bytes': int(lens[0]),
                'checked': 'drop-in output == reference output, every encode and decode call; decode == input',
                'includes': 'per call: Buffer -> H2D, one stream-semantics launch, D2H, host cache mirror'})
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
    # (C4: the shard's 131072 packets in one call -- one seed, screen and commit
    # instead of two: +4 %, profiles/r06_s3_lfk.txt)
    a = argparse.Namespace(scale=1.0, reps=2, batch_mib=512, c4_batch=131072, lru_mib=128, lru_check=1.0,
                           disk_mib=1024, no_decode=False, disk_laps=0)
    # C5-PAIR-LAPS: the same with a disk the shard laps ~3 times (FIFO eviction
    # and re-entry inside the measured figure)
    lap = argparse.Namespace(**{**vars(a), 'disk_laps': 3})
    # C5-PAIR-DENSE: the pair on REF-dense data -- 1 GiB drawn from 16 hot 2 KiB
    # segments (synth.dense), thousands of references per entity per sub-batch
    # (not a BASELINE dataset: the replay's long-run case; a prefix checked)
    dense = argparse.Namespace(**{**vars(a), 'dense_pool': 16, 'dense_cache': 'pair', 'lru_check': 0.1})
    # C5-LRU in one call of the shard's 8192 chunks: its sub-batches (N + H <= C,
    # ~900 chunks) then split 8192 into 9 equal parts instead of 4096 into 5
    # twice -- a launch costs one chunk's serial parse however few it holds
    lru1 = argparse.Namespace(**{**vars(a), 'batch_mib': 1024})
    # C5-PAIR likewise in one call: once the pair has measured its disk write
    # rate (the first sub-batch), the shard fits one sub-batch under a disk lap
    # instead of two (each costs a replay and a commit; profiles/r06_pair_*)
    # (three reps: the first, without the fit hint, runs two sub-batches and
    # sizes the scratch for them; the second then grows it for one 8192-chunk
    # sub-batch inside its timed region)
    pair1 = argparse.Namespace(**{**vars(a), 'batch_mib': 1024, 'reps': 3})
    out = {}
    for name, fn, ar in (('C3', cb.run_c3, a), ('C4', cb.run_c4, a), ('C5', cb.run_c5, a), ('C5-LRU', cb.run_c5lru, lru1),
                         ('C5-PAIR', cb.run_c5pair, pair1), ('C5-PAIR-LAPS', cb.run_c5pair, lap),
                         ('C5-PAIR-DENSE', cb.run_c5dense, dense)):
        try:
            out[name] = fn(ar)
        except BaseException as e:          # SystemExit from a parity check included
            out[name] = {'error': f'{type(e).__name__}: {e}'}
    return out


def zlib_stage(streams=2048, steps=3, check=0.25, threads=16):
    """wanproxy's zlib stage after the codec (DeflatePipe / InflatePipe,
    zlib/deflate_pipe.cc:57-115, inflate_pipe.cc:54-139) on the GPU, level 6
    as wanproxy.conf: `streams` pipes, one consume() of 64 KiB per pipe per
    step, on the XCodec output of C2 and on protocol-like text; every checked
    output equal to the system zlib's in DeflatePipe's call pattern, every
    stream inflated back (scripts/zlib_bench.py)."""
    import importlib.util
    spec = importlib.util.spec_from_file_location('zlib_bench', os.path.join(ROOT, 'scripts', 'zlib_bench.py'))
    zb = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(zb)
    out = {}
    for kind, level in (('xcodec', 6), ('text', 6), ('text', 1)):
        a = argparse.Namespace(kind=kind, streams=streams, call_bytes=65536, steps=steps, level=level, check=check,
                               cpu_threads=threads)
        try:
            out[kind if level == 6 else f'{kind}_level{level}'] = zb.run(a)
        except BaseException as e:
            out[kind if level == 6 else f'{kind}_level{level}'] = {'error': f'{type(e).__name__}: {e}'}
    # the drop-in classes one consume at a time (wanproxy's call pattern) beside the reference's
    try:
        out['per_call'] = {k: zb.per_call(k, 6, 256) for k in ('xcodec', 'text')}
    except BaseException as e:
        out['per_call'] = {'error': f'{type(e).__name__}: {e}'}
    return out


def summary(line):
    """The line's figures in one short object, printed last (a record that
    keeps only the tail of stdout still carries every headline number)."""
    def g(d, *path):
        for p in path:
            if not isinstance(d, dict) or p not in d:
                return None
            d = d[p]
        return d
    s = {'headline_GiBps': line.get('value'), 'headline_frac': g(line, 'roofline', 'frac'),
         'S2_stream_GiBps': g(line, 'stream_semantics', 'value'),
         'S2_stream_frac': g(line, 'stream_semantics', 'roofline', 'frac'),
         'S2_decode_GiBps': g(line, 'decode', 'value'),
         'tack_loop_us_per_call': {
             'encode': [g(line, 'tack_loop', 'gpu_dropin', 'us_per_call'),
                        g(line, 'tack_loop', 'reference_cpu', 'us_per_call')],
             'decode': [g(line, 'tack_loop', 'gpu_dropin', 'decode_us_per_call'),
                        g(line, 'tack_loop', 'reference_cpu', 'decode_us_per_call')],
             'order': '[drop-in, reference]'},
         'host_inclusive_GiBps': g(line, 'host_inclusive', 'value'),
         'cpu_baseline_GiBps': g(line, 'cpu_baseline', 'value')}
    cf = line.get('configs') or {}
    s['configs_encode_GiBps'] = {k: (v.get('encode_GiBps') if 'error' not in v else 'error')
                                 for k, v in cf.items()}
    s['configs_rounds'] = {k: v.get('rounds') for k, v in cf.items() if k.startswith('C5-')}
    z = line.get('zlib_stage') or {}
    if z:
        s['zlib_GiBps'] = {k: [g(z, k, 'value'), g(z, k, 'inflate', 'GiBps')]
                           for k in ('xcodec', 'text', 'text_level1') if k in z}
        pc = z.get('per_call') or {}
        s['zlib_per_call_us'] = {k: {'deflate': [g(pc, k, 'gpu_dropin', 'deflate_us_per_call'),
                                                 g(pc, k, 'reference_cpu', 'deflate_us_per_call')],
                                     'inflate': [g(pc, k, 'gpu_dropin', 'inflate_us_per_call'),
                                                 g(pc, k, 'reference_cpu', 'inflate_us_per_call')]}
                                 for k in ('xcodec', 'text') if k in pc}
    return s


def sharded_configs(world, rank, dev, backend='nccl'):
    """N > 1: BASELINE configs C4 and C5 as ONE dataset each, split into
    contiguous per-rank ranges (wanproxy_amd/shard.py config_shard: C4 2^20/N
    packets, C5 8 GiB/N), every rank encoding its range with a private cache
    (wanproxy's one encoder + cache per codec,
    programs/wanproxy/wanproxy_config_class_codec.cc:39-80).  Timed between
    barriers, max wall over ranks; each rank checks all of its range against
    the oracle run on that range alone (C5: with the same pair) and decodes
    all of it back.
    Returns aggregate GiB/s (strong scaling: the dataset is fixed)."""
    import importlib.util
    import torch
    import torch.distributed as dist
    spec = importlib.util.spec_from_file_location('configs_bench', os.path.join(ROOT, 'scripts', 'configs_bench.py'))
    cb = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(cb)

    def reduce(w):
        if w is None:
            dist.barrier()
            return None
        t = torch.tensor([w], dtype=torch.float64, device=dev if backend == 'nccl' else None)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        return float(t.item())
    a = argparse.Namespace(scale=1.0, reps=2, batch_mib=1024, c4_batch=131072, world=world, rank=rank, reduce=reduce,
                           no_decode=False, lru_mib=128, disk_mib=1024, lru_check=1.0, disk_laps=0)
    out = {}
    # C5 as BASELINE.json configs[4] words it: "cold cache with xcodec_cache_disk
    # spill" -- every rank's cache is wanproxy.conf's pair (shard.C5_PAIR)
    for name, fn in (('C4', cb.run_c4), ('C5', cb.run_c5pair)):
        err = ''
        try:
            r = fn(a)
        except BaseException as e:          # SystemExit from a parity check included
            r, err = None, f'{type(e).__name__}: {e}'
        t = torch.tensor([0.0 if r is None else float(r['in_bytes']), 1.0 if err else 0.0, 0.0 if r is None else
                          float(r['encode_wall_s'])], dtype=torch.float64,
                         device=dev if backend == 'nccl' else None)
        dist.all_reduce(t[:2], op=dist.ReduceOp.SUM)
        tot, fails = float(t[0]), int(t[1])
        if fails:
            out[name] = {'error': f'{fails} rank(s) failed; rank {rank}: {err or "ok"}'}
            continue
        wall = r['encode_wall_s']           # already the max over ranks (reduce)
        out[name] = {'value': round(tot / 2**30 / wall, 2), 'unit': 'GiB/s', 'scaling': 'strong',
                     'dataset_bytes': int(tot), 'ms': round(wall * 1e3, 2), 'ranks': world,
                     'rank0': {k: r[k] for k in ('config', 'shard', 'out_in', 'checked', 'kernel') if k in r}}
    return out


def launch_plan(gpus, env):
    """How this invocation runs: ('rank', world) -- one rank of an outer
    launcher (torchrun sets WORLD_SIZE) or the only rank; ('spawn', N) -- no
    outer launcher and --gpus N > 1: start N ranks as children.  An outer
    launcher whose world differs from --gpus is an error (ValueError)."""
    outer = env.get('WORLD_SIZE')
    if outer is not None:
        world = int(outer)
        if gpus is not None and gpus != world:
            raise ValueError(f'--gpus {gpus} under a launcher of WORLD_SIZE {world}')
        return 'rank', world
    n = 1 if gpus is None else gpus
    if n < 1:
        raise ValueError(f'--gpus {n}')
    return ('spawn', n) if n > 1 else ('rank', 1)


def spawn_ranks(n, argv):
    """--gpus N without an outer launcher: N ranks under torch.distributed.run
    as a child process (this process never touches the GPU, and is not
    replaced: the child's exit status is returned), rendezvous on 127.0.0.1."""
    import socket
    import subprocess
    s = socket.socket()
    s.bind(('127.0.0.1', 0))
    port = s.getsockname()[1]
    s.close()
    cmd = [sys.executable, '-m', 'torch.distributed.run', '--nnodes=1', f'--nproc-per-node={n}',
           '--master-addr=127.0.0.1', f'--master-port={port}', os.path.abspath(__file__)] + argv
    env = dict(os.environ)
    env.setdefault('HSA_ENABLE_IPC_MODE_LEGACY', '0')
    return subprocess.run(cmd, env=env).returncode


def main():
    args = parse()
    try:
        how, world = launch_plan(args.gpus, os.environ)
    except ValueError as e:
        raise SystemExit(f'bench.py: {e}')
    if how == 'spawn':
        raise SystemExit(spawn_ranks(world, sys.argv[1:]))
    import torch
    rank = int(os.environ.get('RANK', '0'))
    local = int(os.environ.get('LOCAL_RANK', '0'))
    if world > 1:
        import torch.distributed as dist
        local %= max(1, torch.cuda.device_count())
        torch.cuda.set_device(local)
        if args.dist_backend == 'nccl':
            dist.init_process_group('nccl', device_id=torch.device('cuda', local))
        else:
            dist.init_process_group(args.dist_backend)
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

    # Parity of this run's output: every chunk against the CPU oracle.
    ol = d_ol.cpu().numpy()
    outh = d_out.cpu().numpy()
    exp = oracle_all(data, offs, lens, mode=0)
    for i in range(n):
        if outh[int(oo[i]):int(oo[i]) + int(ol[i])].tobytes() != exp[i]:
            raise SystemExit(f'PARITY FAILURE on chunk {i}')
    del exp
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

    extras = {}
    if world == 1 and not args.no_extras:
        extras = side_measurements(ctx, data, offs, lens, d_in, d_off, d_len, d_oo, d_out, d_ol, d_st, n, stream, dev,
                                   rank)
    sharded = sharded_configs(world, rank, dev, args.dist_backend) if world > 1 and not args.no_configs else None

    from wanproxy_amd.shard import reduce_run
    red_dev = dev if args.dist_backend == 'nccl' else None
    wall, job_bytes = reduce_run(wall, in_bytes, device=red_dev)   # max wall, total bytes over ranks
    total_bytes = float(job_bytes) * args.steps
    value = total_bytes / 2**30 / wall

    if rank == 0:
        achieved = (in_bytes + out_bytes) / (kern_ms * 1e-3) / 1e9
        read = in_bytes / (kern_ms * 1e-3) / 1e9
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
                         'frac': round(achieved / PEAK_HBM_GBS, 5),
                         'frac_read': round(read / PEAK_HBM_GBS, 5),
                         'frac_note': 'frac: (input + output bytes) / kernel time / peak; frac_read: input bytes '
                                      'only (the north star\'s HBM-read roofline)',
                         'traffic': traffic, 'traffic_source': tsrc,
                         'kernel': 'encode_independent_kernel', 'kernel_ms': round(kern_ms, 4),
                         'algorithmic_bytes_per_launch': in_bytes + out_bytes},
        }
        # Order: the bulky side tables first, the figures a reader looks for
        # last -- a record that keeps only the tail of stdout still holds the
        # stream / decode / tack-loop figures and the summary.
        if sharded is not None:
            line['sharded_configs'] = sharded
        if world == 1 and not args.no_extras and not args.no_configs:
            line['configs'] = other_configs()
        if world == 1 and not args.no_extras and not args.no_zlib:
            line['zlib_stage'] = zlib_stage(threads=host_cpus()['threads'])
        if 'host_inclusive' in extras:
            line['host_inclusive'] = extras.pop('host_inclusive')
        if world == 1 and not args.no_cpu_baseline:
            line['cpu_baseline'] = cpu_baseline(data, offs, lens, args.cpu_seconds)
        line.update(extras)
        line['summary'] = summary(line)
        print(json.dumps(line), flush=True)
    ctx.close()
    if world > 1:
        torch.distributed.destroy_process_group()


if __name__ == '__main__':
    main()
