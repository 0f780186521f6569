"""Host-side mirror of wanproxy's zlib stage over libxcgpu.so's xcg_zdeflate_*.

Reference interface (wanproxy tree):
  DeflatePipe(int level) / consume(Buffer *in)      zlib/deflate_pipe.h:33-42,
                                                    zlib/deflate_pipe.cc:36-115
  chained after the XCodec pipe pair                programs/wanproxy/
                                                    wanproxy_codec_pipe_pair.cc:97-106,148-157

`DeflatePipes(level, nstreams)` is a GPU context holding `nstreams`
DeflatePipe instances; `consume_many` runs one consume() per listed stream in
one batch (what a proxy serving many connections issues per event-loop turn);
`InflatePipes(nstreams)` is the receiving side, InflatePipe
(zlib/inflate_pipe.cc:54-139): consume() takes any cut of the peer's stream.
`pipe(i).consume(data)` is the single-pipe form with DeflatePipe's exact
signature semantics: non-empty input -> the bytes produced after
deflate(Z_SYNC_FLUSH); b'' -> EOS, deflate(Z_FINISH).  Errors raise; there is
no CPU fallback.
"""
from __future__ import annotations

import ctypes as C

import numpy as np

from .xcgpu import XCGError, _check, _stream_ptr, lib as _xlib

XCG_ENOTSUP = -95


def _lib():
    L = _xlib()
    if not getattr(L, '_zd_bound', False):
        vp = C.c_void_p
        L.xcg_zdeflate_bound.argtypes = [C.c_uint32]
        L.xcg_zdeflate_bound.restype = C.c_uint64
        L.xcg_zdeflate_create.argtypes = [C.c_int, C.c_int, C.c_uint32, C.POINTER(vp)]
        L.xcg_zdeflate_create.restype = C.c_int
        L.xcg_zdeflate_destroy.argtypes = [vp]
        L.xcg_zdeflate_destroy.restype = None
        L.xcg_zdeflate_reset.argtypes = [vp, C.c_uint32]
        L.xcg_zdeflate_reset.restype = C.c_int
        L.xcg_zdeflate_batch.argtypes = [vp, vp, vp, vp, vp, C.c_uint32, vp, vp, vp, vp, vp]
        L.xcg_zdeflate_batch.restype = C.c_int
        L.xcg_zdeflate_host.argtypes = [vp, vp, vp, vp, vp, C.c_uint32, vp, vp, vp, vp, vp, vp]
        L.xcg_zdeflate_batch_seg.argtypes = [vp, vp, vp, vp, vp, C.c_uint32, vp, vp, vp, vp, vp, vp, vp]
        L.xcg_zdeflate_batch_seg.restype = C.c_int
        L.xcg_debug_zdeflate_rounds.argtypes = [vp]
        L.xcg_debug_zdeflate_rounds.restype = C.c_uint32
        L.xcg_zdeflate_host.restype = C.c_int
        L.xcg_zinflate_create.argtypes = [C.c_int, C.c_uint32, C.POINTER(vp)]
        L.xcg_zinflate_create.restype = C.c_int
        L.xcg_zinflate_destroy.argtypes = [vp]
        L.xcg_zinflate_destroy.restype = None
        L.xcg_zinflate_reset.argtypes = [vp, C.c_uint32]
        L.xcg_zinflate_reset.restype = C.c_int
        L.xcg_zinflate_batch.argtypes = [vp, vp, vp, vp, vp, C.c_uint32, vp, vp, vp, vp, vp, vp]
        L.xcg_zinflate_batch.restype = C.c_int
        L.xcg_debug_set_zinflate_mode.argtypes = [C.c_int]
        L.xcg_debug_set_zinflate_mode.restype = C.c_int
        L._zd_bound = True
    return L


def set_inflate_mode(mode: int) -> None:
    """Which inflate kernel runs (xcg_debug_set_zinflate_mode): 0 by batch
    size, 1 a wave per call, 2 a 1024-thread workgroup per call, 3 a
    256-thread workgroup per call."""
    _check(_lib().xcg_debug_set_zinflate_mode(mode))


def bound(n: int) -> int:
    return int(_lib().xcg_zdeflate_bound(int(n)))


class DeflatePipes:
    def __init__(self, level: int = 6, nstreams: int = 1, device: int = 0):
        import torch
        if not torch.cuda.is_available():
            raise XCGError('DeflatePipes needs a GPU (no CPU fallback)')
        self.level, self.nstreams, self.device = level, nstreams, device
        h = C.c_void_p()
        rc = _lib().xcg_zdeflate_create(device, level, nstreams, C.byref(h))
        self.undelivered = {}           # stream -> bytes the pipe made but has not produced yet
        if rc == XCG_ENOTSUP:
            raise XCGError(f'zlib level {level}: not supported')
        _check(rc)
        self.h = h

    def close(self):
        if getattr(self, 'h', None):
            _lib().xcg_zdeflate_destroy(self.h)
            self.h = None

    def __del__(self):
        self.close()

    def reset(self, stream: int):
        _check(_lib().xcg_zdeflate_reset(self.h, stream))
        self.undelivered.pop(stream, None)

    @property
    def last_rounds(self) -> int:
        """levels 1-3: parse rounds the last batch took"""
        return int(_lib().xcg_debug_zdeflate_rounds(self.h))

    def pipe(self, stream: int) -> 'DeflatePipe':
        return DeflatePipe(self, stream)

    def batch_device(self, d_in, in_off, lens, streams, d_out, out_off, d_out_len, d_deliver, stream=None,
                     segments=None):
        """Device-resident batch: d_in / d_out / d_out_len (int32) / d_deliver
        (int64) are torch CUDA tensors; in_off / lens / streams / out_off host
        numpy arrays.  d_out_len: the new stream bytes at out_off; d_deliver:
        what the consume produces (the stream's undelivered bytes first)."""
        in_off = np.ascontiguousarray(in_off, dtype=np.uint64)
        lens = np.ascontiguousarray(lens, dtype=np.uint32)
        streams = np.ascontiguousarray(streams, dtype=np.uint32)
        out_off = np.ascontiguousarray(out_off, dtype=np.uint64)
        n = int(lens.size)
        seg = nseg = None
        if segments is not None:     # per call: the Buffer's segment lengths (None: 2048-byte cuts)
            per = [list(sg) if sg is not None else [min(2048, int(lens[i]) - k) for k in range(0, int(lens[i]), 2048)]
                   for i, sg in enumerate(segments)]
            nseg = np.array([len(x) for x in per], dtype=np.uint32)
            seg = np.array([v for x in per for v in x] or [0], dtype=np.uint32)
        _check(_lib().xcg_zdeflate_batch_seg(self.h, C.c_void_p(d_in.data_ptr()), in_off.ctypes.data,
                                             lens.ctypes.data, streams.ctypes.data, n,
                                             seg.ctypes.data if seg is not None else None,
                                             nseg.ctypes.data if nseg is not None else None,
                                             C.c_void_p(d_out.data_ptr()), out_off.ctypes.data,
                                             C.c_void_p(d_out_len.data_ptr()), C.c_void_p(d_deliver.data_ptr()),
                                             _stream_ptr(stream)))

    def consume_many(self, items):
        """items: [(stream, bytes)] or [(stream, bytes, segments)] (each stream
        at most once; segments: the Buffer's segment lengths, which level 0's
        stored blocks follow).  Returns the produced bytes per item, in order."""
        import torch
        dev = torch.device('cuda', self.device)
        n = len(items)
        if n == 0:
            return []
        segs = [it[2] if len(it) > 2 else None for it in items]
        items = [(it[0], it[1]) for it in items]
        lens = np.array([len(d) for _, d in items], dtype=np.uint32)
        streams = np.array([s for s, _ in items], dtype=np.uint32)
        in_off = np.zeros(n, dtype=np.uint64)
        in_off[1:] = np.cumsum(lens.astype(np.uint64))[:-1]
        bounds = np.array([(bound(x) + 3) & ~3 for x in lens], dtype=np.uint64)
        out_off = np.zeros(n, dtype=np.uint64)
        out_off[1:] = np.cumsum(bounds)[:-1]
        blob = b''.join(d for _, d in items)
        d_in = torch.frombuffer(bytearray(blob or b'\0'), dtype=torch.uint8).to(dev)
        d_out = torch.empty(int(bounds.sum()), dtype=torch.uint8, device=dev)
        d_len = torch.zeros(n, dtype=torch.int32, device=dev)
        d_dl = torch.zeros(n, dtype=torch.int64, device=dev)
        self.batch_device(d_in, in_off, lens, streams, d_out, out_off, d_len, d_dl,
                          segments=segs if any(x is not None for x in segs) else None)
        torch.cuda.synchronize(dev)
        ol = d_len.cpu().numpy().astype(np.uint64)
        dl = d_dl.cpu().numpy()
        out = d_out.cpu().numpy()
        res = []
        for i in range(n):
            st = int(streams[i])
            q = self.undelivered.get(st, b'') + out[int(out_off[i]):int(out_off[i] + ol[i])].tobytes()
            k = int(dl[i])
            if k > len(q):
                raise XCGError(f'deflate stream {st}: delivers {k} of {len(q)} bytes')
            res.append(q[:k])
            self.undelivered[st] = q[k:]
        return res


class DeflatePipe:
    """One DeflatePipe(level) of a DeflatePipes context."""

    def __init__(self, ctx: DeflatePipes, stream: int):
        self.ctx, self.stream = ctx, stream

    def consume(self, data: bytes) -> bytes:
        return self.ctx.consume_many([(self.stream, data)])[0]


class InflateError(XCGError):
    pass


class InflatePipes:
    """`nstreams` InflatePipe instances on one GPU."""

    def __init__(self, nstreams: int = 1, device: int = 0):
        import torch
        if not torch.cuda.is_available():
            raise XCGError('InflatePipes needs a GPU (no CPU fallback)')
        self.nstreams, self.device = nstreams, device
        h = C.c_void_p()
        _check(_lib().xcg_zinflate_create(device, nstreams, C.byref(h)))
        self.h = h

    def close(self):
        if getattr(self, 'h', None):
            _lib().xcg_zinflate_destroy(self.h)
            self.h = None

    def __del__(self):
        self.close()

    def reset(self, stream: int):
        """Slot `stream` becomes a fresh InflatePipe (inflateInit)."""
        _check(_lib().xcg_zinflate_reset(self.h, stream))

    def batch_device(self, d_in, in_off, lens, streams, d_out, out_off, out_cap, d_out_len, d_status, stream=None):
        in_off = np.ascontiguousarray(in_off, dtype=np.uint64)
        lens = np.ascontiguousarray(lens, dtype=np.uint32)
        streams = np.ascontiguousarray(streams, dtype=np.uint32)
        out_off = np.ascontiguousarray(out_off, dtype=np.uint64)
        out_cap = np.ascontiguousarray(out_cap, dtype=np.uint32)
        _check(_lib().xcg_zinflate_batch(self.h, C.c_void_p(d_in.data_ptr()), in_off.ctypes.data, lens.ctypes.data,
                                         streams.ctypes.data, int(lens.size), C.c_void_p(d_out.data_ptr()),
                                         out_off.ctypes.data, out_cap.ctypes.data, C.c_void_p(d_out_len.data_ptr()),
                                         C.c_void_p(d_status.data_ptr()), _stream_ptr(stream)))

    def consume_many(self, items, out_cap: int = None):
        """items: [(stream, bytes)] -> [(produced bytes, status)] with status
        0 ok, 1 stream end (EOS for an empty consume), -1 data error.  A call
        that needs more output room is repeated with more (-2 commits nothing)."""
        import torch
        dev = torch.device('cuda', self.device)
        n = len(items)
        if n == 0:
            return []
        lens = np.array([len(d) for _, d in items], dtype=np.uint32)
        streams = np.array([s for s, _ in items], dtype=np.uint32)
        in_off = np.zeros(n, dtype=np.uint64)
        in_off[1:] = np.cumsum(lens.astype(np.uint64))[:-1]
        cap = out_cap or max(1 << 20, 8 * int(lens.max()) + 65536)
        blob = b''.join(d for _, d in items)
        d_in = torch.frombuffer(bytearray(blob or b'\0'), dtype=torch.uint8).to(dev)
        while True:
            caps = np.full(n, cap, dtype=np.uint32)
            out_off = np.arange(n, dtype=np.uint64) * cap
            d_out = torch.empty(n * cap, dtype=torch.uint8, device=dev)
            d_len = torch.zeros(n, dtype=torch.int32, device=dev)
            d_st = torch.zeros(n, dtype=torch.int32, device=dev)
            self.batch_device(d_in, in_off, lens, streams, d_out, out_off, caps, d_len, d_st)
            torch.cuda.synchronize(dev)
            st = d_st.cpu().numpy()
            if (st == -2).any():
                # calls with enough room committed; repeat only the others with more room
                ol = d_len.cpu().numpy()
                out = d_out.cpu().numpy()
                done = {i: (out[int(out_off[i]):int(out_off[i]) + int(ol[i])].tobytes(), int(st[i]))
                        for i in range(n) if st[i] != -2}
                redo = [i for i in range(n) if st[i] == -2]
                more = self.consume_many([items[i] for i in redo], out_cap=cap * 4)
                for i, r in zip(redo, more):
                    done[i] = r
                return [done[i] for i in range(n)]
            ol = d_len.cpu().numpy()
            out = d_out.cpu().numpy()
            return [(out[int(out_off[i]):int(out_off[i]) + int(ol[i])].tobytes(), int(st[i])) for i in range(n)]
