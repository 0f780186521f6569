#!/usr/bin/env python3
"""Per-call inflate on one stream, both kernels (xcg_debug_set_zinflate_mode
1 / 2): median us per 64 KiB consume (InflatePipes.consume_many, host copies
included) and the workgroup kernel's region statistics."""
import ctypes as C
import os
import sys
import time
import zlib

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from tests.zlib_cases import wan_stream  # noqa: E402
from wanproxy_amd.zpipe import InflatePipes, _lib, set_inflate_mode  # noqa: E402


def main():
    calls = int(sys.argv[1]) if len(sys.argv) > 1 else 64
    data = wan_stream(5000, calls, 65536)
    co = zlib.compressobj(6)
    zs = [co.compress(d) + co.flush(zlib.Z_SYNC_FLUSH) for d in data]
    L = _lib()
    L.xcg_debug_zinflate_regions.argtypes = [C.c_void_p]
    st = np.zeros(4, np.uint64)
    timing = 'zitime' in os.environ.get('XCGPU_LIB', '')
    zt = np.zeros(16, np.uint64)
    if timing:
        L.xcg_debug_zi_times.argtypes = [C.c_void_p]
    for mode in (1, 2, 1, 2):
        set_inflate_mode(mode)
        ip = InflatePipes(1)
        L.xcg_debug_zinflate_regions(st.ctypes.data)
        if timing:
            L.xcg_debug_zi_times(zt.ctypes.data)
        t, out = [], []
        for z in zs:
            t0 = time.perf_counter()
            (o, s), = ip.consume_many([(0, z)])
            t.append(time.perf_counter() - t0)
            out.append(o)
        ip.close()
        L.xcg_debug_zinflate_regions(st.ctypes.data)
        ok = b''.join(out) == b''.join(data)
        if timing:
            L.xcg_debug_zi_times(zt.ctypes.data)
            names = ['setup', 'fastlit', 'fastmatch', 'careful', 'flush', 'stored', 'tail', 'header', 'region', 'cl_loop']
            print(f'mode {mode} cycles per call:', {n: int(zt[i]) // len(zs) for i, n in enumerate(names)})
            rn = ['stage', 'fixpoint', 'scan', 'write', 'resolve', 'out']
            print(f'mode {mode} region cycles per call:', {n: int(zt[10 + i]) // len(zs) for i, n in enumerate(rn)})
        print(f'mode {mode}: {1e6 * float(np.median(t[1:])):.1f} us per call, ok={ok}, regions {int(st[0])} '
              f'iters {int(st[1])} bytes {int(st[2])} resolve_rounds {int(st[3])}', flush=True)
    set_inflate_mode(0)


if __name__ == '__main__':
    main()
