"""ctypes binding of libxcgpu.so (include/xcgpu.h) plus a host-side mirror of
the reference's XCodec encoder interface.

The product path is the HIP library; this module only moves buffers (torch is
used for device memory and streams) and never falls back to a CPU codec: if
the library or a GPU is missing, every entry point raises.

Reference interface mirrored (wanproxy tree):
  XCodecEncoder(XCodecCache*) / encode(Buffer*, Buffer*)   xcodec/xcodec_encoder.h:40-43
  XCodecMemoryCache / TackNullCache / out_of_band()         xcodec/xcodec_cache.h:245-365,
                                                            programs/tack/tack.cc:70-101
  XCodecHash::hash / mix                                    xcodec/xcodec_hash.h:155-174
"""
from __future__ import annotations

import ctypes as C
import os

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
# XCGPU_LIB selects a diagnostic build of the same library (scripts/dev).
LIB_PATH = os.environ.get('XCGPU_LIB') or os.path.join(HERE, 'libxcgpu.so')
SEG = 2048

XCG_FLAG_OOB = 0x1
XCG_FLAG_NULLCACHE = 0x2
XCG_SEM_INDEPENDENT = 0
XCG_SEM_STREAM = 1
XCG_EOVERFLOW = -75

_lib = None


XCG_ENOENT = -2


class XCGError(RuntimeError):
    pass


class _PipeOut(C.Structure):
    _fields_ = [('to_peer', C.c_void_p), ('to_peer_len', C.c_uint64), ('to_local', C.c_void_p),
                ('to_local_len', C.c_uint64), ('local_eos', C.c_int), ('peer_eos', C.c_int)]

    def peer(self) -> bytes:
        return C.string_at(self.to_peer, self.to_peer_len) if self.to_peer_len else b''

    def local(self) -> bytes:
        return C.string_at(self.to_local, self.to_local_len) if self.to_local_len else b''


def lib():
    """Load libxcgpu.so (after torch, so both share one HIP runtime)."""
    global _lib
    if _lib is not None:
        return _lib
    import torch  # noqa: F401  -- load torch's libamdhip64 first
    if not os.path.exists(LIB_PATH):
        raise XCGError(f'{LIB_PATH} missing: run `python -c "import __graft_entry__ as g; g.build()"`')
    L = C.CDLL(LIB_PATH)
    vp, u8p, u32p, u64p = C.c_void_p, C.c_void_p, C.c_void_p, C.c_void_p
    L.xcg_version.restype = C.c_char_p
    L.xcg_strerror.restype = C.c_char_p
    L.xcg_strerror.argtypes = [C.c_int]
    L.xcg_encode_bound.restype = C.c_uint64
    L.xcg_encode_bound.argtypes = [C.c_uint32]
    L.xcg_ctx_create.argtypes = [C.c_int, C.c_uint32, C.POINTER(C.c_void_p)]
    L.xcg_ctx_create.restype = C.c_int
    L.xcg_ctx_create_ex.argtypes = [C.c_int, C.c_uint32, C.c_uint64, C.POINTER(C.c_void_p)]
    L.xcg_ctx_create_ex.restype = C.c_int
    L.xcg_ctx_create_bounded.argtypes = [C.c_int, C.c_uint32, C.c_uint64, C.POINTER(C.c_void_p)]
    L.xcg_ctx_create_bounded.restype = C.c_int
    L.xcg_ctx_create_pair.argtypes = [C.c_int, C.c_uint32, C.c_uint64, C.c_uint64, C.POINTER(C.c_void_p)]
    L.xcg_ctx_create_pair.restype = C.c_int
    L.xcg_disk_create.argtypes = [C.c_uint64, C.POINTER(C.c_void_p)]
    L.xcg_disk_create.restype = C.c_int
    L.xcg_disk_destroy.argtypes = [vp]
    L.xcg_disk_destroy.restype = None
    L.xcg_disk_stats.argtypes = [vp, vp]
    L.xcg_disk_stats.restype = C.c_int
    L.xcg_disk_create_ex.argtypes = [C.c_uint64, C.c_uint32, C.POINTER(C.c_void_p)]
    L.xcg_disk_create_ex.restype = C.c_int
    L.xcg_disk_tier.argtypes = [vp]
    L.xcg_disk_tier.restype = C.c_int
    L.xcg_disk_open.argtypes = [C.c_char_p, C.c_uint64, C.c_uint32, C.POINTER(C.c_void_p)]
    L.xcg_disk_open.restype = C.c_int
    L.xcg_disk_save.argtypes = [vp, C.c_char_p]
    L.xcg_disk_save.restype = C.c_int
    L.xcg_ctx_create_pair_uuid.argtypes = [C.c_int, C.c_uint32, C.c_uint64, vp, C.c_char_p, C.POINTER(C.c_void_p)]
    L.xcg_ctx_create_pair_uuid.restype = C.c_int
    L.xcg_ctx_create_pair_on.argtypes = [C.c_int, C.c_uint32, C.c_uint64, vp, C.POINTER(C.c_void_p)]
    L.xcg_ctx_create_pair_on.restype = C.c_int
    L.xcg_ctx_create_pair_xuid.argtypes = [C.c_int, C.c_uint32, C.c_uint64, vp, C.c_char_p, C.c_int,
                                           C.POINTER(C.c_void_p)]
    L.xcg_ctx_create_pair_xuid.restype = C.c_int
    L.xcg_disk_open_fd.argtypes = [C.c_int, C.c_uint64, C.c_uint32, C.POINTER(C.c_void_p)]
    L.xcg_disk_open_fd.restype = C.c_int
    L.xcg_disk_head.argtypes = [vp, C.POINTER(C.c_uint64), C.POINTER(C.c_uint64)]
    L.xcg_disk_head.restype = C.c_int
    L.xcg_pair_xuid.argtypes = [vp]
    L.xcg_pair_xuid.restype = C.c_int
    L.xcg_pair_stats.argtypes = [vp, vp]
    L.xcg_pair_stats.restype = C.c_int
    L.xcg_ctx_flags.argtypes = [vp, vp]
    L.xcg_ctx_flags.restype = C.c_int
    L.xcg_cache_size.argtypes = [vp]
    L.xcg_cache_size.restype = C.c_uint64
    L.xcg_cache_clear.argtypes = [vp]
    L.xcg_cache_clear.restype = C.c_int
    L.xcg_last_rounds.argtypes = [vp]
    L.xcg_last_rounds.restype = C.c_int
    L.xcg_ctx_destroy.argtypes = [vp]
    L.xcg_ctx_status.argtypes = [vp]
    L.xcg_ctx_status.restype = C.c_int
    L.xcg_encode_batch.argtypes = [vp, C.c_int, u8p, u64p, u32p, C.c_uint32, C.c_uint32, u8p, u64p, u64p, u32p, vp]
    L.xcg_encode_batch.restype = C.c_int
    L.xcg_encode_host.argtypes = [vp, C.c_int, u8p, C.c_uint64, u64p, u32p, C.c_uint32, u8p, C.c_uint64, u64p, u64p]
    L.xcg_encode_host.restype = C.c_int
    L.xcg_decode_batch.argtypes = [vp, u8p, u64p, u32p, C.c_uint32, C.c_uint32, u8p, C.c_uint64, u64p, u64p, vp, u64p,
                                   u64p, C.c_uint32, vp, u64p, vp]
    L.xcg_decode_batch.restype = C.c_int
    L.xcg_window_create.argtypes = [vp, C.POINTER(C.c_void_p)]
    L.xcg_window_create.restype = C.c_int
    L.xcg_window_destroy.argtypes = [vp]
    L.xcg_window_destroy.restype = None
    L.xcg_decode_set_window.argtypes = [vp, vp]
    L.xcg_decode_set_window.restype = C.c_int
    L.xcg_decode_call.argtypes = [vp, C.c_char_p, C.c_uint32, vp, C.c_uint64, vp, vp, vp, vp, C.c_uint32, vp, vp,
                                  C.c_uint32, vp]
    L.xcg_decode_call.restype = C.c_int
    L.xcg_pack_outputs.argtypes = [vp, u8p, u64p, u64p, C.c_uint32, u8p, u64p, u64p, vp]
    L.xcg_pack_outputs.restype = C.c_int
    L.xcg_window_hashes.argtypes = [vp, u8p, C.c_uint64, u64p, vp]
    L.xcg_window_hashes.restype = C.c_int
    L.xcg_segment_hashes.argtypes = [vp, u8p, C.c_uint64, u64p, vp]
    L.xcg_segment_hashes.restype = C.c_int
    L.xcg_pipe_create.argtypes = [vp, vp, C.c_char_p, C.POINTER(C.c_void_p)]
    L.xcg_pipe_create.restype = C.c_int
    L.xcg_pipe_destroy.argtypes = [vp]
    L.xcg_pipe_destroy.restype = None
    L.xcg_pipe_create_connect.argtypes = [vp, vp, C.c_char_p, C.POINTER(C.c_void_p)]
    L.xcg_pipe_create_connect.restype = C.c_int
    L.xcg_pipe_decoder_ctx.argtypes = [vp]
    L.xcg_pipe_decoder_ctx.restype = vp
    L.xcg_ctx_connect.argtypes = [vp, C.c_char_p, C.POINTER(C.c_void_p)]
    L.xcg_ctx_connect.restype = C.c_int
    L.xcg_ctx_register.argtypes = [vp, C.c_char_p]
    L.xcg_ctx_register.restype = C.c_int
    L.xcg_ctx_lookup.argtypes = [C.c_char_p]
    L.xcg_ctx_lookup.restype = vp
    L.xcg_connect_registry_clear.argtypes = []
    L.xcg_connect_registry_clear.restype = None
    L.xcg_pipe_encoder_consume.argtypes = [vp, C.c_char_p, C.c_uint64, C.POINTER(_PipeOut)]
    L.xcg_pipe_encoder_consume.restype = C.c_int
    L.xcg_pipe_encoder_consume_many.argtypes = [C.POINTER(C.c_void_p), C.POINTER(C.c_char_p), C.POINTER(C.c_uint64),
                                                C.c_uint32, C.POINTER(_PipeOut)]
    L.xcg_pipe_encoder_consume_many.restype = C.c_int
    L.xcg_pipe_decoder_consume.argtypes = [vp, C.c_char_p, C.c_uint64, C.POINTER(_PipeOut)]
    L.xcg_pipe_decoder_consume.restype = C.c_int
    L.xcg_pipe_pending_frames.argtypes = [vp]
    L.xcg_pipe_pending_frames.restype = C.c_uint32
    L.xcg_debug_set_stream_seed.argtypes = [C.c_int]
    L.xcg_debug_set_stream_seed.restype = C.c_int
    L.xcg_debug_stream_kernel_timing.argtypes = [C.c_int]
    L.xcg_debug_stream_kernel_timing.restype = C.c_int
    L.xcg_debug_stream_kernel_time.argtypes = [C.POINTER(C.c_double), C.POINTER(C.c_uint32)]
    L.xcg_debug_stream_kernel_time.restype = C.c_int
    L.xcg_debug_restart_counts.argtypes = [vp, C.POINTER(C.c_uint64), C.POINTER(C.c_uint64)]
    L.xcg_debug_restart_counts.restype = C.c_int
    L.xcg_debug_set_lds_filter_keys.argtypes = [C.c_uint32]
    L.xcg_debug_set_lds_filter_keys.restype = C.c_uint32
    L.xcg_debug_set_lds_prefilter_keys.argtypes = [C.c_uint32]
    L.xcg_debug_set_lds_prefilter_keys.restype = C.c_uint32
    L.xcg_debug_decode_kernel_timing.argtypes = [C.c_int]
    L.xcg_debug_decode_kernel_timing.restype = C.c_int
    L.xcg_debug_decode_kernel_time.argtypes = [C.POINTER(C.c_double), C.POINTER(C.c_double), C.POINTER(C.c_uint32)]
    L.xcg_debug_decode_kernel_time.restype = C.c_int
    L.xcg_debug_set_screen.argtypes = [C.c_int]
    L.xcg_debug_set_screen.restype = C.c_int
    L.xcg_debug_screen_counts.argtypes = [C.POINTER(C.c_uint64), C.POINTER(C.c_uint64)]
    L.xcg_debug_screen_counts.restype = C.c_int
    _lib = L
    return L


def _check(rc):
    if rc != 0:
        raise XCGError(f'xcgpu: {lib().xcg_strerror(rc).decode()} ({rc})')


def _stream_ptr(stream):
    import torch
    s = stream if stream is not None else torch.cuda.current_stream()
    return C.c_void_p(s.cuda_stream)


def stream_kernel_time():
    """(milliseconds, launches) of the stream-parse kernel since the last call,
    timed by HIP events on its launch stream while xcg_debug_stream_kernel_timing
    is on (bench.py's roofline for stream semantics)."""
    ms, k = C.c_double(), C.c_uint32()
    _check(lib().xcg_debug_stream_kernel_time(C.byref(ms), C.byref(k)))
    return float(ms.value), int(k.value)


def encode_bound(n: int) -> int:
    return 2 * int(n) + 16


class Disk:
    """One XCodecDisk shared by several pair contexts (xcg_disk_create): the
    local cache's front and each peer front XCodecCache::connect makes append
    to one FIFO ring (xcodec/xcodec_cache_disk.h:33-69)."""

    HOST, DEVICE = 1, 2          # XCG_DISK_HOST / XCG_DISK_DEVICE: force the blocks' tier

    def __init__(self, disk_bytes: int, tier: int = 0, path: str = None):
        """With `path`: the volume file there (xcg_disk_open: reopened when it
        holds one, else fresh)."""
        h = C.c_void_p()
        if path is not None:
            _check(lib().xcg_disk_open(path.encode(), int(disk_bytes), int(tier), C.byref(h)))
        else:
            _check(lib().xcg_disk_create_ex(int(disk_bytes), int(tier), C.byref(h)))
        self.h = h

    def save(self, path: str):
        """Write the volume as the reference's file stands now (xcg_disk_save)."""
        _check(lib().xcg_disk_save(self.h, path.encode()))

    def head(self):
        """The write head: (index block, next entry) -- XCodecDisk's
        current_index_block_ / index_block_next_."""
        b, n = C.c_uint64(), C.c_uint64()
        _check(lib().xcg_disk_head(self.h, C.byref(b), C.byref(n)))
        return int(b.value), int(n.value)

    def tier(self) -> int:
        """Where the data blocks live: 0 HBM, 1 pinned host memory (-1: no front yet)."""
        return int(lib().xcg_disk_tier(self.h))

    def stats(self):
        """(live index entries of every front, entries written, index blocks, fronts)."""
        st = (C.c_uint64 * 4)()
        _check(lib().xcg_disk_stats(self.h, st))
        return tuple(int(v) for v in st)

    def close(self):
        if getattr(self, 'h', None):
            lib().xcg_disk_destroy(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


class Context:
    """An XCodecEncoder + cache configuration bound to one GPU."""

    def __init__(self, device: int = 0, out_of_band: bool = False, null_cache: bool = False,
                 cache_segments: int = 1 << 19, memory_cache_limit: int = 0, disk_bytes: int = 0,
                 disk: Disk = None, uuid: str = None, xuid: int = None):
        """memory_cache_limit (bytes): the bounded, LRU-evicting cache
        XCodecMemoryCache(uuid, memory_cache_limit) (xcodec/xcodec_cache.h:277)
        instead of an unbounded one of cache_segments capacity.  With
        disk_bytes too: wanproxy.conf's XCodecCachePair of that memory cache
        and a disk of disk_bytes (xcodec/xcodec_cache.h:140-237); with `disk`
        instead, the pair's secondary is the next front of that shared disk
        (with `uuid`, that UUID's front: XCodecDisk::connect; with `xuid`, that
        front of the disk)."""
        import torch
        if not torch.cuda.is_available():
            raise XCGError('no GPU: the XCodec engine has no CPU path')
        self.device = device
        self.flags = (XCG_FLAG_OOB if out_of_band else 0) | (XCG_FLAG_NULLCACHE if null_cache else 0)
        h = C.c_void_p()
        if disk is not None and xuid is not None:
            _check(lib().xcg_ctx_create_pair_xuid(device, self.flags, int(memory_cache_limit), disk.h,
                                                  uuid.encode() if uuid else None, int(xuid), C.byref(h)))
        elif disk is not None and uuid is not None:
            _check(lib().xcg_ctx_create_pair_uuid(device, self.flags, int(memory_cache_limit), disk.h, uuid.encode(),
                                                  C.byref(h)))
        elif disk is not None:
            _check(lib().xcg_ctx_create_pair_on(device, self.flags, int(memory_cache_limit), disk.h, C.byref(h)))
        elif disk_bytes:
            _check(lib().xcg_ctx_create_pair(device, self.flags, int(memory_cache_limit), int(disk_bytes), C.byref(h)))
        elif memory_cache_limit:
            _check(lib().xcg_ctx_create_bounded(device, self.flags, int(memory_cache_limit), C.byref(h)))
        else:
            _check(lib().xcg_ctx_create_ex(device, self.flags, int(cache_segments), C.byref(h)))
        self.h = h

    # The persistent cache (XCG_SEM_STREAM): XCodecMemoryCache of the encoder.
    def cache_size(self) -> int:
        return int(lib().xcg_cache_size(self.h))

    def cache_lookup(self, h: int):
        """XCodecCache::lookup of one hash: its 2048 bytes, or None (a hit
        refreshes a bounded cache's LRU order)."""
        buf = (C.c_uint8 * 2048)()
        rc = lib().xcg_cache_lookup_host(self.h, C.c_uint64(h), buf)
        if rc == XCG_ENOENT:
            return None
        _check(rc)
        return bytes(buf)

    def cache_enter(self, h: int, seg: bytes):
        """enter (or replace the bytes of) one segment -- XCodecPipePair's <LEARN>."""
        assert len(seg) == 2048
        _check(lib().xcg_cache_enter_host(self.h, C.c_uint64(h), (C.c_uint8 * 2048).from_buffer_copy(seg)))

    def pair_stats(self):
        """(primary entries, this front's disk index entries, disk entries
        written by every front, disk index blocks) of a pair context."""
        st = (C.c_uint64 * 4)()
        _check(lib().xcg_pair_stats(self.h, st))
        return tuple(int(v) for v in st)

    def xuid(self) -> int:
        """The disk front (xuid) of a pair context."""
        x = lib().xcg_pair_xuid(self.h)
        _check(min(x, 0))
        return x

    def restart_counts(self):
        """(chunks resumed from their rows, chunks that rejoined their old parse)
        in this context's bounded / pair re-parse passes so far."""
        a, b = C.c_uint64(), C.c_uint64()
        _check(lib().xcg_debug_restart_counts(self.h, C.byref(a), C.byref(b)))
        return int(a.value), int(b.value)

    def cache_clear(self):
        _check(lib().xcg_cache_clear(self.h))

    def last_rounds(self) -> int:
        return int(lib().xcg_last_rounds(self.h))

    def close(self):
        if getattr(self, 'h', None):
            lib().xcg_ctx_destroy(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def status(self):
        _check(lib().xcg_ctx_status(self.h))

    # ------------------------------------------------------------- device API
    def encode_batch_device(self, d_in, d_off, d_len, n, max_len, d_out, d_out_off, d_out_len,
                            d_stats=None, stream=None, semantics=XCG_SEM_INDEPENDENT):
        """Raw launch on device tensors (all torch tensors on this device)."""
        _check(lib().xcg_encode_batch(
            self.h, semantics, C.c_void_p(d_in.data_ptr()), C.c_void_p(d_off.data_ptr()),
            C.c_void_p(d_len.data_ptr()), int(n), int(max_len), C.c_void_p(d_out.data_ptr()),
            C.c_void_p(d_out_off.data_ptr()), C.c_void_p(d_out_len.data_ptr()),
            C.c_void_p(d_stats.data_ptr()) if d_stats is not None else None, _stream_ptr(stream)))

    def encode_chunks(self, data, offs, lens, with_stats=False, semantics=XCG_SEM_INDEPENDENT):
        """Encode chunks of host `data` (bytes / np.uint8) on the GPU; returns a
        list of encoded bytes objects (and per-chunk stats if asked)."""
        import torch
        dev = torch.device('cuda', self.device)
        a = np.frombuffer(data, dtype=np.uint8) if not isinstance(data, np.ndarray) else data
        offs = np.ascontiguousarray(offs, dtype=np.uint64)
        lens = np.ascontiguousarray(lens, dtype=np.uint32)
        n = int(offs.size)
        if n == 0:
            return ([], np.zeros((0, 4), np.uint32)) if with_stats else []
        bounds = 2 * lens.astype(np.uint64) + 16
        oo = np.zeros(n, dtype=np.uint64)
        oo[1:] = np.cumsum(bounds)[:-1]
        d_in = torch.from_numpy(a.copy() if a.size else np.zeros(1, np.uint8)).to(dev)
        d_off = torch.from_numpy(offs.view(np.int64)).to(dev)
        d_len = torch.from_numpy(lens.view(np.int32)).to(dev)
        d_oo = torch.from_numpy(oo.view(np.int64)).to(dev)
        d_out = torch.zeros(int(bounds.sum()), dtype=torch.uint8, device=dev)
        d_ol = torch.zeros(n, dtype=torch.int64, device=dev)
        d_st = torch.zeros(4 * n, dtype=torch.int32, device=dev)
        self.encode_batch_device(d_in, d_off, d_len, n, int(lens.max()), d_out, d_oo, d_ol, d_st,
                                 semantics=semantics)
        torch.cuda.synchronize(dev)
        self.status()
        out = d_out.cpu().numpy()
        ol = d_ol.cpu().numpy().astype(np.uint64)
        res = [out[int(oo[i]):int(oo[i] + ol[i])].tobytes() for i in range(n)]
        if with_stats:
            return res, d_st.cpu().numpy().view(np.uint32).reshape(n, 4)
        return res

    def decode_chunks(self, encs, window: 'Window' = None):
        """Decode encoded chunks (one stream, this context's cache) on the GPU,
        with `window` as the decoder's BACKREF window (default: the context's).
        Returns (outs, status, consumed, unknown) -- see xcg_decode_batch."""
        import torch
        dev = torch.device('cuda', self.device)
        n = len(encs)
        lens = np.array([len(e) for e in encs], dtype=np.uint32)
        offs = np.zeros(n, dtype=np.uint64)
        if n > 1:
            offs[1:] = np.cumsum(lens.astype(np.uint64))[:-1]
        blob = np.frombuffer(b''.join(encs) or b'\0', dtype=np.uint8)
        d_in = torch.from_numpy(blob.copy()).to(dev)
        d_off = torch.from_numpy(offs.view(np.int64)).to(dev)
        d_len = torch.from_numpy(lens.view(np.int32)).to(dev)
        d_oo = torch.zeros(n, dtype=torch.int64, device=dev)
        d_ol = torch.zeros(n, dtype=torch.int64, device=dev)
        d_st = torch.zeros(n, dtype=torch.int32, device=dev)
        d_cons = torch.zeros(n, dtype=torch.int64, device=dev)
        cap = int(lens.astype(np.uint64).sum()) * 205 + 4096   # a 10-byte REF expands to 2048
        unk = np.zeros(1 << 16, dtype=np.uint64)
        nunk = np.zeros(1, dtype=np.uint32)
        total = np.zeros(1, dtype=np.uint64)
        if window is not None:
            _check(lib().xcg_decode_set_window(self.h, window.h))
        try:
            for _ in range(2):
                d_out = torch.zeros(cap, dtype=torch.uint8, device=dev)
                rc = lib().xcg_decode_batch(
                    self.h, C.c_void_p(d_in.data_ptr()), C.c_void_p(d_off.data_ptr()), C.c_void_p(d_len.data_ptr()),
                    n, int(lens.max()) if n else 0, C.c_void_p(d_out.data_ptr()), cap, C.c_void_p(d_oo.data_ptr()),
                    C.c_void_p(d_ol.data_ptr()), C.c_void_p(d_st.data_ptr()), C.c_void_p(d_cons.data_ptr()),
                    unk.ctypes.data, unk.size, nunk.ctypes.data, total.ctypes.data, _stream_ptr(None))
                if rc != XCG_EOVERFLOW:
                    break
                cap = int(total[0])            # BACKREF-dense: 3 bytes -> 2048; nothing was committed
            _check(rc)
        finally:
            if window is not None:
                lib().xcg_decode_set_window(self.h, None)
        torch.cuda.synchronize(dev)
        oo = d_oo.cpu().numpy()
        ol = d_ol.cpu().numpy()
        st = d_st.cpu().numpy()
        cons = d_cons.cpu().numpy()
        out = d_out.cpu().numpy()
        outs = [out[int(oo[i]):int(oo[i]) + int(ol[i])].tobytes() if st[i] != 2 else b'' for i in range(n)]
        return outs, st, cons, [int(u) for u in unk[:int(nunk[0])]]

    def decode_call(self, data: bytes, out_cap: int = None):
        """One XCodecDecoder::decode(output, input, unknown) call from host memory
        (xcg_decode_call: one launch, one synchronisation on an unbounded cache).
        Returns (status, out, consumed, unknown, extract_hashes or None)."""
        n = len(data)
        if out_cap is None:
            out_cap = (n // 10 + 1) * 2048 + n
        out = np.zeros(max(1, out_cap), np.uint8)
        ol, cons = np.zeros(1, np.uint64), np.zeros(1, np.uint64)
        st = np.zeros(1, np.int32)
        unk = np.zeros(1 << 16, np.uint64)
        nunk, ne = np.zeros(1, np.uint32), np.zeros(1, np.uint32)
        ext = np.zeros(1024, np.uint64)
        _check(lib().xcg_decode_call(self.h, data, n, out.ctypes.data, out_cap, ol.ctypes.data, cons.ctypes.data,
                                     st.ctypes.data, unk.ctypes.data, unk.size, nunk.ctypes.data, ext.ctypes.data,
                                     ext.size, ne.ctypes.data))
        hashes = None if int(ne[0]) == 0xFFFFFFFF else [int(h) for h in ext[:int(ne[0])]]
        return (int(st[0]), out[:int(ol[0])].tobytes(), int(cons[0]), [int(u) for u in unk[:int(nunk[0])]], hashes)

    def window_hashes(self, data) -> np.ndarray:
        import torch
        dev = torch.device('cuda', self.device)
        a = np.frombuffer(data, dtype=np.uint8)
        n = max(0, a.size - SEG + 1)
        if n == 0:
            return np.zeros(0, np.uint64)
        d_x = torch.from_numpy(a.copy()).to(dev)
        d_h = torch.zeros(n, dtype=torch.int64, device=dev)
        _check(lib().xcg_window_hashes(self.h, C.c_void_p(d_x.data_ptr()), a.size, C.c_void_p(d_h.data_ptr()),
                                       _stream_ptr(None)))
        torch.cuda.synchronize(dev)
        return d_h.cpu().numpy().view(np.uint64)

    def segment_hashes_be(self, data) -> bytes:
        import torch
        dev = torch.device('cuda', self.device)
        a = np.frombuffer(data, dtype=np.uint8)
        n = a.size // SEG
        if n == 0:
            return b''
        d_x = torch.from_numpy(a.copy()).to(dev)
        d_h = torch.zeros(n, dtype=torch.int64, device=dev)
        _check(lib().xcg_segment_hashes(self.h, C.c_void_p(d_x.data_ptr()), a.size, C.c_void_p(d_h.data_ptr()),
                                        _stream_ptr(None)))
        torch.cuda.synchronize(dev)
        return d_h.cpu().numpy().tobytes()


class Window:
    """A decoder's BACKREF window (XCodecWindow, xcodec/xcodec_window.h)."""

    def __init__(self, ctx: Context):
        self.ctx = ctx
        h = C.c_void_p()
        _check(lib().xcg_window_create(ctx.h, C.byref(h)))
        self.h = h

    def close(self):
        if getattr(self, 'h', None):
            lib().xcg_window_destroy(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


class XCodecEncoder:
    """Mirror of XCodecEncoder(XCodecCache*) (xcodec/xcodec_encoder.h:40-43):
    successive encode() calls share the context's cache, exactly like tack's
    loop (programs/tack/tack.cc:301-321)."""

    def __init__(self, ctx: Context):
        self.ctx = ctx

    def encode(self, data: bytes) -> bytes:
        if not data:
            return b''
        return self.ctx.encode_chunks(data, np.array([0]), np.array([len(data)]), semantics=XCG_SEM_STREAM)[0]


class XCodecDecoder:
    """Mirror of XCodecDecoder(XCodecCache*) (xcodec/xcodec_decoder.h:35-45):
    decode(input) -> (ok, output, consumed, unknown_hashes), where `consumed`
    is how much of `input` decode() removed (a partial op stays) and
    `unknown_hashes` the sorted set an ASK would request."""

    def __init__(self, ctx: Context):
        self.ctx = ctx
        self.window = Window(ctx)      # XCodecDecoder::window_, one per decoder

    def decode(self, data: bytes):
        if not data:
            return True, b'', 0, []
        outs, st, cons, unk = self.ctx.decode_chunks([data], window=self.window)
        return int(st[0]) >= 0, outs[0], int(cons[0]), unk


class PipePair:
    """Mirror of XCodecPipePair (xcodec/xcodec_pipe_pair.h:41-212) over
    xcg_pipe_*: encoder_consume(data) -> bytes for the peer (b'' input = EOS);
    decoder_consume(data) -> (to_peer, to_local, local_eos, peer_eos).  `enc`
    is the codec's context (cache shared by its pipes), `dec` the context of the
    peer's cache; `uuid` the 36-byte UUID string sent in <HELLO>."""

    def __init__(self, enc: Context, dec: Context, uuid: bytes, connect: bool = False):
        """connect=True: `dec` is the codec's cache (codec_->cache()) and the
        decoder context is connected at the peer's <HELLO>
        (xcg_pipe_create_connect: XCodecCache::connect(uuid, parent))."""
        self.enc, self.dec = enc, dec
        h = C.c_void_p()
        fn = lib().xcg_pipe_create_connect if connect else lib().xcg_pipe_create
        _check(fn(enc.h, dec.h, uuid, C.byref(h)))
        self.h = h

    def decoder_ctx(self):
        """Handle (int) of the context this pipe decodes on, None before <HELLO>."""
        return lib().xcg_pipe_decoder_ctx(self.h)

    def close(self):
        if getattr(self, 'h', None):
            lib().xcg_pipe_destroy(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def encoder_consume(self, data: bytes) -> bytes:
        o = _PipeOut()
        _check(lib().xcg_pipe_encoder_consume(self.h, data, len(data), C.byref(o)))
        return o.peer()

    @staticmethod
    def encoder_consume_many(pipes, datas):
        n = len(pipes)
        hs = (C.c_void_p * n)(*[p.h.value for p in pipes])
        ds = (C.c_char_p * n)(*datas)
        ls = (C.c_uint64 * n)(*[len(d) for d in datas])
        outs = (_PipeOut * n)()
        _check(lib().xcg_pipe_encoder_consume_many(hs, ds, ls, n, outs))
        return [o.peer() for o in outs]

    def decoder_consume(self, data: bytes):
        o = _PipeOut()
        rc = lib().xcg_pipe_decoder_consume(self.h, data, len(data), C.byref(o))
        _check(rc)
        return o.peer(), o.local(), bool(o.local_eos), bool(o.peer_eos)

    def pending_frames(self) -> int:
        return int(lib().xcg_pipe_pending_frames(self.h))


def ctx_connect(parent: Context, uuid: bytes):
    """xcg_ctx_connect: handle (int) of the registry's context for `uuid`."""
    h = C.c_void_p()
    _check(lib().xcg_ctx_connect(parent.h, uuid, C.byref(h)))
    return h.value


def ctx_register(ctx: Context, uuid: bytes):
    _check(lib().xcg_ctx_register(ctx.h, uuid))


def ctx_lookup(uuid: bytes):
    return lib().xcg_ctx_lookup(uuid)


def connect_registry_clear():
    lib().xcg_connect_registry_clear()
