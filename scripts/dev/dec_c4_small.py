import sys, os, time, ctypes as C
sys.path.insert(0, os.environ.get('GRAFT_REPO_ROOT', '.'))
import numpy as np, torch
import importlib.util
spec = importlib.util.spec_from_file_location('cb', 'scripts/configs_bench.py'); cb = importlib.util.module_from_spec(spec); spec.loader.exec_module(cb)
from wanproxy_amd import synth
from wanproxy_amd.xcgpu import Context, lib, _check
n = 65536
data = np.frombuffer(synth.stream(0xC4, n * 4096, 4, 0), np.uint8).copy()
offs, lens = synth.chunks_of(data.tobytes(), 4096)
ctx = Context(0, cache_segments=300000)
B = cb.Batches(ctx, data, offs, lens, per=16384)
B.encode_all(); encs = B.outputs()
dctx = Context(0, cache_segments=300000)
dev = torch.device('cuda', 0)
per = 16384
elens = np.array([len(e) for e in encs], np.uint32)
eoffs = np.zeros(n, np.uint64); eoffs[1:] = np.cumsum(elens.astype(np.uint64))[:-1]
d_enc = torch.from_numpy(np.frombuffer(b''.join(encs), np.uint8).copy()).to(dev)
d_eoff = torch.from_numpy(eoffs.view(np.int64)).to(dev); d_elen = torch.from_numpy(elens.view(np.int32)).to(dev)
cap = per * 4096 + 4096
d_dout = torch.empty(cap, dtype=torch.uint8, device=dev)
d_doo, d_dol, d_dcons = [torch.zeros(per, dtype=torch.int64, device=dev) for _ in range(3)]
d_dst = torch.zeros(per, dtype=torch.int32, device=dev)
unk = np.zeros(16, np.uint64); nunk = np.zeros(1, np.uint32); tot = np.zeros(1, np.uint64)
for rep in range(2):
    dctx.cache_clear()
    for a in range(0, n, per):
        b = min(n, a + per)
        torch.cuda.synchronize(dev)
        t0 = time.perf_counter()
        mx = int(elens[a:b].max())
        t1 = time.perf_counter()
        rc = lib().xcg_decode_batch(dctx.h, C.c_void_p(d_enc.data_ptr()), C.c_void_p(d_eoff[a:].data_ptr()),
                                    C.c_void_p(d_elen[a:].data_ptr()), b - a, mx, C.c_void_p(d_dout.data_ptr()), cap,
                                    C.c_void_p(d_doo.data_ptr()), C.c_void_p(d_dol.data_ptr()), C.c_void_p(d_dst.data_ptr()),
                                    C.c_void_p(d_dcons.data_ptr()), unk.ctypes.data, unk.size, nunk.ctypes.data,
                                    tot.ctypes.data, None)
        t2 = time.perf_counter()
        torch.cuda.synchronize(dev)
        t3 = time.perf_counter()
        print(rep, a, rc, f'max {1e3*(t1-t0):.2f} ms  decode_batch {1e3*(t2-t1):.2f} ms  sync {1e3*(t3-t2):.2f} ms')
