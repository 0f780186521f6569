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
