#!/usr/bin/env python3
"""zlib stage throughput (DeflatePipe, zlib/deflate_pipe.cc:57-115) on the GPU:
S streams, each step = one consume() of B bytes per stream (Z_SYNC_FLUSH),
inputs resident in HBM; every output checked against the system zlib 1.2.11
driven in DeflatePipe's call pattern.  Prints one JSON object.

Workloads: `xcodec` = the XCodec stream encoding of C2 (what wanproxy feeds its
DeflatePipe: wanproxy_codec_pipe_pair.cc:97-106), cut into per-stream calls;
`text` = compressible protocol-like traffic (tests/zlib_cases.wan_stream)."""
from __future__ import annotations

import argparse
import json
import os
import sys
import time
import zlib
from concurrent.futures import ThreadPoolExecutor

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def workload(kind: str, streams: int, call_bytes: int, steps: int):
    """list over steps of list over streams of bytes"""
    if kind == 'text':
        from tests.zlib_cases import wan_stream
        per = [wan_stream(5000 + s, steps, call_bytes) for s in range(streams)]
        return [[per[s][k] for s in range(streams)] for k in range(steps)]
    from wanproxy_amd import synth
    from wanproxy_amd.xcgpu import XCG_SEM_STREAM, Context
    d = synth.stream(0xC2, 4096 * 65536, 50, 0)
    offs, lens = synth.chunks_of(d, 65536)
    ctx = Context(0, cache_segments=1 << 18)
    enc = b''.join(ctx.encode_chunks(d, offs, lens, semantics=XCG_SEM_STREAM))
    ctx.close()
    need = streams * call_bytes * steps
    while len(enc) < need:
        enc += enc
    out, o = [], 0
    for _ in range(steps):
        row = []
        for _ in range(streams):
            row.append(enc[o:o + call_bytes])
            o += call_bytes
        out.append(row)
    return out


def zlib_ref(streams_calls, level, threads):
    """outputs of the reference call pattern, streams in parallel (zlib releases the GIL)"""
    from oracle.zlib_pipe import DeflatePipeRef

    def one(calls):
        r = DeflatePipeRef(level)
        return [r.consume(c) for c in calls]
    with ThreadPoolExecutor(threads) as ex:
        return list(ex.map(one, streams_calls))


def per_call(kind: str = 'xcodec', level: int = 6, calls: int = 256) -> dict:
    """DeflatePipe::consume / InflatePipe::consume one call at a time, as wanproxy
    makes them (one per read per connection): the drop-in classes
    (integration/zlib_pipes_xcgpu.cc over the engine) beside the reference's own
    classes over the system zlib on this host (zlib/deflate_pipe.cc,
    inflate_pipe.cc), both through oracle/zpipe_driver.cc, same Buffers; every
    call's output compared."""
    from oracle.zlib_pipe import ReferencePipes
    data = [row[0] for row in workload(kind, 1, 65536, calls)]
    res = {'kind': kind, 'level': level, 'calls': calls, 'call_bytes': 65536}
    outs = {}
    for which in ('dropin', 'ref'):
        R = ReferencePipes(which)
        d = R.pipe('deflate', level)
        zs, t = [], []
        for k, c in enumerate(data):
            t0 = time.perf_counter()
            z, _ = d.consume(c)
            if k:                                   # (the first call: header, context warm-up)
                t.append(time.perf_counter() - t0)
            zs.append(z)
        i = R.pipe('inflate')
        back, ti = [], []
        for k, z in enumerate(zs):
            t0 = time.perf_counter()
            o, _ = i.consume(z)
            if k:
                ti.append(time.perf_counter() - t0)
            back.append(o)
        # end both streams cleanly (an empty consume is EOS: deflate(Z_FINISH)),
        # so neither class logs an unfinished stream when it is destroyed
        tail, _ = d.consume(b'')
        zs.append(tail)
        o, _ = i.consume(tail)
        back.append(o)
        outs[which] = zs
        key = 'gpu_dropin' if which == 'dropin' else 'reference_cpu'
        res[key] = {'deflate_us_per_call': round(1e6 * float(np.median(t)), 1),
                    'inflate_us_per_call': round(1e6 * float(np.median(ti)), 1),
                    'inflated_ok': b''.join(back) == b''.join(data)}
        d.close()
        i.close()
    res['checked'] = ('every deflate call equal to the reference class' if outs['dropin'] == outs['ref']
                      else 'MISMATCH')
    return res


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('--kind', default='xcodec', choices=['xcodec', 'text'])
    ap.add_argument('--streams', type=int, default=4096)
    ap.add_argument('--call-bytes', type=int, default=65536)
    ap.add_argument('--steps', type=int, default=4)
    ap.add_argument('--level', type=int, default=6)
    ap.add_argument('--check', type=float, default=1.0, help='fraction of streams checked against zlib')
    ap.add_argument('--cpu-threads', type=int, default=16)
    ap.add_argument('--per-call', action='store_true', help='the drop-in classes one consume at a time vs the reference')
    args = ap.parse_args()
    if args.per_call:
        print(json.dumps(per_call(args.kind, args.level, 256)))
        return
    res = run(args)
    print(json.dumps(res))
    if res.get('mismatches') or 'MISMATCH' in res['inflate']['checked']:
        sys.exit(1)


def run(args) -> dict:
    import torch
    from wanproxy_amd.zpipe import DeflatePipes, bound
    dev = torch.device('cuda', 0)
    S, B, K = args.streams, args.call_bytes, args.steps
    data = workload(args.kind, S, B, K)
    ctx = DeflatePipes(args.level, S)
    lens = np.full(S, B, dtype=np.uint32)
    sids = np.arange(S, dtype=np.uint32)
    in_off = (np.arange(S, dtype=np.uint64) * B)
    ob = (bound(B) + 255) & ~255
    out_off = np.arange(S, dtype=np.uint64) * ob
    d_ins = [torch.frombuffer(bytearray(b''.join(row)), dtype=torch.uint8).to(dev) for row in data]
    d_out = [torch.empty(S * ob, dtype=torch.uint8, device=dev) for _ in range(K)]
    d_len = [torch.zeros(S, dtype=torch.int32, device=dev) for _ in range(K)]
    d_dl = [torch.zeros(S, dtype=torch.int64, device=dev) for _ in range(K)]
    torch.cuda.synchronize()
    times, rounds = [], []
    for k in range(K):
        t0 = time.perf_counter()
        ctx.batch_device(d_ins[k], in_off, lens, sids, d_out[k], out_off, d_len[k], d_dl[k])
        torch.cuda.synchronize()
        times.append(time.perf_counter() - t0)
        rounds.append(ctx.last_rounds)
    # what each consume produces: the stream's undelivered bytes, then the new ones, cut at d_deliver
    outs, held = [], [b''] * S
    for k in range(K):
        ol = d_len[k].cpu().numpy()
        dl = d_dl[k].cpu().numpy()
        o = d_out[k].cpu().numpy()
        row = []
        for s in range(S):
            q = held[s] + o[s * ob:s * ob + int(ol[s])].tobytes()
            row.append(q[:int(dl[s])])
            held[s] = q[int(dl[s]):]
        outs.append(row)
    # InflatePipe on the GPU over the same streams: step k consumes deflate output k
    from wanproxy_amd.zpipe import InflatePipes
    ictx = InflatePipes(S)
    icap = 2 * B + 65536
    zi_times, zi_ok = [], True
    dec = [b''] * S
    for k in range(K):
        zl = np.array([len(outs[k][s]) for s in range(S)], dtype=np.uint32)
        zo = np.zeros(S, dtype=np.uint64)
        zo[1:] = np.cumsum(zl.astype(np.uint64))[:-1]
        d_z = torch.frombuffer(bytearray(b''.join(outs[k])), dtype=torch.uint8).to(dev)
        d_o = torch.empty(S * icap, dtype=torch.uint8, device=dev)
        d_ol = torch.zeros(S, dtype=torch.int32, device=dev)
        d_st = torch.zeros(S, dtype=torch.int32, device=dev)
        caps = np.full(S, icap, dtype=np.uint32)
        ooff = np.arange(S, dtype=np.uint64) * icap
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        ictx.batch_device(d_z, zo, zl, sids, d_o, ooff, caps, d_ol, d_st)
        torch.cuda.synchronize()
        zi_times.append(time.perf_counter() - t0)
        st = d_st.cpu().numpy()
        ol = d_ol.cpu().numpy()
        o = d_o.cpu().numpy()
        zi_ok = zi_ok and bool((st == 0).all())
        for s in range(S):
            dec[s] += o[s * icap:s * icap + int(ol[s])].tobytes()
    # decoded so far = a prefix of the input (a consume may hold bytes back), and all of it
    # once the held-back bytes follow
    for s in range(S):
        whole = b''.join(data[k][s] for k in range(K))
        zi_ok = zi_ok and whole.startswith(dec[s])
        if s < 64:
            d = zlib.decompressobj()
            zi_ok = zi_ok and d.decompress(b''.join(outs[k][s] for k in range(K)) + held[s]) == whole
    ictx.close()
    zi_ms = 1e3 * float(np.median(zi_times[1:] if K > 1 else zi_times))
    nchk = max(1, int(S * args.check))
    t0 = time.perf_counter()

    def inf_one(s):
        d = zlib.decompressobj()
        return [d.decompress(outs[k][s]) for k in range(K)]
    with ThreadPoolExecutor(args.cpu_threads) as ex:
        list(ex.map(inf_one, range(nchk)))
    cpu_inf_s = time.perf_counter() - t0
    t0 = time.perf_counter()
    ref = zlib_ref([[data[k][s] for k in range(K)] for s in range(nchk)], args.level, args.cpu_threads)
    cpu_s = time.perf_counter() - t0
    bad = sum(1 for s in range(nchk) for k in range(K) if ref[s][k] != outs[k][s])
    # steady state: steps after the first (the first carries the zlib header)
    steady = times[1:] if K > 1 else times
    ms = 1e3 * float(np.median(steady))
    in_bytes = S * B
    out_bytes = sum(len(outs[K - 1][s]) for s in range(S))
    res = {
        'metric': 'DeflatePipe consume GiB/s (device-resident, one consume per stream per step)',
        'kind': args.kind, 'level': args.level, 'streams': S, 'call_bytes': B, 'steps': K,
        'value': round(in_bytes / (ms / 1e3) / 2**30, 3), 'ms_per_step': round(ms, 3),
        'out_in': round(out_bytes / in_bytes, 5),
        'parse_rounds': rounds if args.level in (1, 2, 3) else None,
        'checked': f'{nchk} of {S} streams x {K} calls vs zlib {zlib.ZLIB_RUNTIME_VERSION}, {bad} mismatches',
        'mismatches': bad,
        'inflate': {'GiBps': round(in_bytes / (zi_ms / 1e3) / 2**30, 3), 'ms_per_step': round(zi_ms, 3),
                    'checked': 'every stream decoded to a prefix of its input; with the held-back bytes, '
                               'to all of it (64 streams, CPU zlib)' + ('' if zi_ok else ' -- MISMATCH')},
        'cpu_zlib': {'GiBps': round(nchk * K * B / cpu_s / 2**30, 4), 'threads': args.cpu_threads,
                     'inflate_GiBps': round(nchk * K * B / cpu_inf_s / 2**30, 4),
                     'sample': f'{nchk} streams x {K} calls'},
    }
    ctx.close()
    return res


if __name__ == '__main__':
    main()
