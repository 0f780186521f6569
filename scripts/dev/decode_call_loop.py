#!/usr/bin/env python3
"""Diagnostics: the drop-in per-call decode (tack -d, one XCodecDecoder::decode
per 64 KiB call's encoding) through oracle/_ref/libxcdropin.so beside the
reference (libxcref.so), us per call; run under rocprofv3 --kernel-trace
--stats to split the GPU's share."""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
import numpy as np  # noqa: E402

from oracle.lib import Oracle  # noqa: E402
from wanproxy_amd import synth  # noqa: E402

k = int(sys.argv[1]) if len(sys.argv) > 1 else 512
d = synth.stream(0xC2, k * 65536, 50, 0)
offs, lens = synth.chunks_of(d, 65536)
ref = Oracle(ref=True)
encs = ref.encode_batch(d, offs, lens, mode=1)
for name, o in (('gpu_dropin', Oracle(dropin=True)), ('reference_cpu', ref)):
    for rep in range(2):
        c = o.cache_new()
        dec = o.decoder_new(c)
        t0 = time.perf_counter()
        got = [o.decode(e, c, decoder=dec, out_cap=2 * 65536) for e in encs]
        dt = time.perf_counter() - t0
        o.decoder_free(dec)
        o.cache_free(c)
    assert b''.join(g[1] for g in got) == bytes(d)
    print(name, f'{dt / len(encs) * 1e6:.1f} us per decode call')

# xcg_decode_call alone (no class adapter, no host cache mirror), preallocated
import ctypes as C  # noqa: E402
from wanproxy_amd import xcgpu  # noqa: E402
L = xcgpu.lib()
L.xcg_debug_decode_phases.argtypes = [C.c_void_p, C.c_uint32]
L.xcg_debug_decode_phases.restype = C.c_uint32
out = np.zeros(4 * 65536, np.uint8)
ol, cons = np.zeros(1, np.uint64), np.zeros(1, np.uint64)
st = np.zeros(1, np.int32)
unk = np.zeros(1 << 16, np.uint64)
nunk, ne = np.zeros(1, np.uint32), np.zeros(1, np.uint32)
ext = np.zeros(1024, np.uint64)
args = (out.ctypes.data, out.size, ol.ctypes.data, cons.ctypes.data, st.ctypes.data, unk.ctypes.data, unk.size,
        nunk.ctypes.data, ext.ctypes.data, ext.size, ne.ctypes.data)
ph = np.zeros(16, np.float64)
for rep in range(2):
    ctx = xcgpu.Context()
    L.xcg_debug_decode_phases(ph.ctypes.data, 16)
    t0 = time.perf_counter()
    tot = 0
    for e in encs:
        assert L.xcg_decode_call(ctx.h, e, len(e), *args) == 0
        tot += int(ol[0])
    dt = time.perf_counter() - t0
    calls = L.xcg_debug_decode_phases(ph.ctypes.data, 16)
    ctx.close()
    assert tot == len(d)
print('xcg_decode_call', f'{dt / len(encs) * 1e6:.1f} us per call')
if calls:
    names = ['kernel', 'stage', 'walk', 'extract hashes', 'resolve', 'precheck', 'output size', 'output copy', 'window',
             'commit', 'results']
    print('phases (us per call):', ', '.join(f'{n} {ph[i] / calls:.2f}' for i, n in enumerate(names)))
