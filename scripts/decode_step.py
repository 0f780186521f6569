#!/usr/bin/env python3
"""The bench's C2-S2 decode step alone, for rocprofv3 (scripts/profile_decode.sh):
4096 x 64 KiB chunks (seed 0xC2, 50 % duplicate segments) encoded once with
stream semantics on the GPU, then --calls batch decodes of that stream
(xcg_decode_batch, fresh decoder cache each call), the last one checked
against the input.  Prints one JSON line: per-call wall time and the
HIP-event device time of the decode segments."""
import argparse
import ctypes as C
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('--calls', type=int, default=5)
    ap.add_argument('--chunks', type=int, default=4096)
    args = ap.parse_args()
    import torch
    from wanproxy_amd import synth
    from wanproxy_amd.xcgpu import XCG_SEM_STREAM, Context, _check, lib
    CH = 65536
    n = args.chunks
    dev = torch.device('cuda', 0)
    data = np.frombuffer(synth.stream(0xC2, n * CH, 50, 0), dtype=np.uint8)
    offs, lens = synth.chunks_of(data.tobytes(), CH)
    d_in = torch.from_numpy(data.copy()).to(dev)
    d_off = torch.from_numpy(offs.view(np.int64)).to(dev)
    d_len = torch.from_numpy(lens.view(np.int32)).to(dev)
    oo = np.arange(n, dtype=np.uint64) * (2 * CH + 16)
    d_oo = torch.from_numpy(oo.view(np.int64)).to(dev)
    d_out = torch.empty(int(n * (2 * CH + 16)), dtype=torch.uint8, device=dev)
    d_ol = torch.zeros(n, dtype=torch.int64, device=dev)
    sctx = Context(0, cache_segments=1 << 18)
    sctx.encode_batch_device(d_in, d_off, d_len, n, CH, d_out, d_oo, d_ol, semantics=XCG_SEM_STREAM)
    torch.cuda.synchronize()
    ol = d_ol.cpu().numpy()
    outh = d_out.cpu().numpy()
    blob = np.concatenate([outh[int(oo[i]):int(oo[i]) + int(ol[i])] for i in range(n)])
    elens = ol.astype(np.uint32)
    eoffs = np.zeros(n, dtype=np.uint64)
    eoffs[1:] = np.cumsum(elens.astype(np.uint64))[:-1]
    sctx.close()
    del d_out
    in_bytes = int(lens.astype(np.int64).sum())
    d_enc = torch.from_numpy(blob).to(dev)
    d_eoff = torch.from_numpy(eoffs.view(np.int64)).to(dev)
    d_elen = torch.from_numpy(elens.view(np.int32)).to(dev)
    d_dout = torch.empty(in_bytes + 4096, dtype=torch.uint8, device=dev)
    d_doo = torch.zeros(n, dtype=torch.int64, device=dev)
    d_dol = torch.zeros(n, dtype=torch.int64, device=dev)
    d_dst = torch.zeros(n, dtype=torch.int32, device=dev)
    d_dcons = torch.zeros(n, dtype=torch.int64, device=dev)
    unk = np.zeros(16, np.uint64)
    nunk = np.zeros(1, np.uint32)
    tot = np.zeros(1, np.uint64)
    dctx = Context(0, cache_segments=1 << 18)
    stream = torch.cuda.current_stream()
    lib().xcg_debug_decode_kernel_timing(1)
    t0 = time.perf_counter()
    for _ in range(args.calls):
        dctx.cache_clear()
        _check(lib().xcg_decode_batch(dctx.h, C.c_void_p(d_enc.data_ptr()), C.c_void_p(d_eoff.data_ptr()),
                                      C.c_void_p(d_elen.data_ptr()), n, int(elens.max()),
                                      C.c_void_p(d_dout.data_ptr()), d_dout.numel(), C.c_void_p(d_doo.data_ptr()),
                                      C.c_void_p(d_dol.data_ptr()), C.c_void_p(d_dst.data_ptr()),
                                      C.c_void_p(d_dcons.data_ptr()), unk.ctypes.data, unk.size, nunk.ctypes.data,
                                      tot.ctypes.data, C.c_void_p(stream.cuda_stream)))
    torch.cuda.synchronize()
    wall = (time.perf_counter() - t0) / args.calls
    lib().xcg_debug_decode_kernel_timing(0)
    sm, em, sg = C.c_double(), C.c_double(), C.c_uint32()
    lib().xcg_debug_decode_kernel_time(C.byref(sm), C.byref(em), C.byref(sg))
    ok = int(tot[0]) == in_bytes and d_dout[:in_bytes].cpu().numpy().tobytes() == data.tobytes()
    dctx.close()
    print(json.dumps({'calls': args.calls, 'in_bytes': in_bytes, 'enc_bytes': int(elens.sum()),
                      'wall_ms_per_call': round(wall * 1e3, 4), 'device_ms_per_call': round(sm.value / args.calls, 4),
                      'emit_ms_per_call': round(em.value / args.calls, 4), 'segments': sg.value, 'decoded_ok': ok}))
    if not ok:
        raise SystemExit('PARITY FAILURE (decode round trip)')


if __name__ == '__main__':
    main()
