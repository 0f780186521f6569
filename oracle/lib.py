"""ctypes bindings for the test oracles.  TEST INFRASTRUCTURE ONLY.

`Oracle()` loads oracle/build/liboracle.so (the in-repo C restatement,
oracle/xcodec_oracle.c); `Oracle(ref=True)` loads oracle/_ref/libxcref.so (the
real reference hot path compiled from /root/reference by oracle/Makefile).
Both expose the same batch encode / decode / hash surface so tests can check
one against the other and both against the GPU engine.
"""
from __future__ import annotations

import ctypes as C
import os

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
SEG = 2048

MODE_INDEPENDENT, MODE_STREAM, MODE_NULL = 0, 1, 2

_u8p = C.POINTER(C.c_uint8)
_u32p = C.POINTER(C.c_uint32)
_u64p = C.POINTER(C.c_uint64)


def _p(a, t):
    return a.ctypes.data_as(t)


def build():
    import subprocess
    subprocess.run(['make', '-s', '-C', HERE], check=True)


class Oracle:
    def __init__(self, ref: bool = False, dropin: bool = False):
        # dropin: the reference's own driver and Buffer / cache classes, with
        # XCodecEncoder / XCodecDecoder provided by integration/ over the GPU
        # engine (oracle/Makefile libxcdropin.so) -- reference-shaped calls.
        self.ref = ref or dropin
        ref = self.ref
        if dropin:
            import torch  # noqa: F401  (one HIP runtime shared with libxcgpu.so)
            # (XCGPU_DROPIN_LIB: a diagnostics build of the same harness, e.g.
            # _ref/libxcdropin_at.so with the adapter's phase timers)
            path = os.environ.get('XCGPU_DROPIN_LIB') or os.path.join(HERE, '_ref/libxcdropin.so')
        else:
            path = os.path.join(HERE, '_ref/libxcref.so' if ref else 'build/liboracle.so')
        if not os.path.exists(path):
            raise FileNotFoundError(path)
        L = self.lib = C.CDLL(path)
        pre = ('xdi_' if dropin else 'xcr_') if ref else 'xco_'
        self._pre = pre
        self._hash = getattr(L, pre + 'hash')
        self._hash.restype = C.c_uint64
        self._hash.argtypes = [_u8p]
        self._wh = getattr(L, pre + 'window_hashes')
        self._wh.argtypes = [_u8p, C.c_uint64, _u64p]
        self._cnew = getattr(L, pre + "cache_new")
        self._cnew.restype = C.c_void_p
        self._cnewl = getattr(L, pre + 'cache_new_limited')
        self._cnewl.restype = C.c_void_p
        self._cnewl.argtypes = [C.c_uint64]
        self._cfree = getattr(L, pre + 'cache_free')
        self._cfree.argtypes = [C.c_void_p]
        self._eb = getattr(L, pre + 'encode_batch')
        if ref:
            self._eb.argtypes = [C.c_void_p, _u8p, _u64p, _u32p, C.c_uint32, C.c_int, _u8p, _u64p, _u64p]
        else:
            self._eb.argtypes = [C.c_void_p, _u8p, _u64p, _u32p, C.c_uint32, C.c_int, C.c_int, _u8p, _u64p, _u64p]
        self._eb.restype = C.c_int
        self._dec = getattr(L, pre + 'decode') if ref else None
        self._cnew.restype = C.c_void_p
        if ref:
            self._dec.argtypes = [C.c_void_p, _u8p, C.c_uint64, _u8p, C.c_uint64, _u64p, _u64p, _u64p, _u64p, C.c_uint64]
            self._dec.restype = C.c_int
            self._dnew = getattr(L, pre + 'decoder_new')
            self._dnew.restype = C.c_void_p
            self._dnew.argtypes = [C.c_void_p]
            self._dfree = getattr(L, pre + 'decoder_free')
            self._dfree.argtypes = [C.c_void_p]
            self._ddec = getattr(L, pre + 'decoder_decode')
            self._ddec.argtypes = [C.c_void_p, _u8p, C.c_uint64, _u8p, C.c_uint64, _u64p, _u64p, _u64p, _u64p,
                                   C.c_uint64]
            self._ddec.restype = C.c_int
        else:
            L.xco_decoder_new.restype = C.c_void_p
            L.xco_decoder_new.argtypes = [C.c_void_p]
            L.xco_decoder_free.argtypes = [C.c_void_p]
            L.xco_decode.argtypes = [C.c_void_p, _u8p, C.c_uint64, _u8p, C.c_uint64, _u64p, _u64p, _u64p, _u64p, C.c_uint64]
            L.xco_decode.restype = C.c_int
            L.xco_cache_size.restype = C.c_uint64
            L.xco_cache_size.argtypes = [C.c_void_p]
            L.xco_cache_enter.argtypes = [C.c_void_p, C.c_uint64, _u8p]
            L.xco_cache_enter.restype = C.c_int
            L.xco_cache_export.argtypes = [C.c_void_p, _u64p, _u8p, C.c_uint64]
            L.xco_cache_export.restype = C.c_uint64

    # ------------------------------------------------------------------ hash
    def hash(self, w: bytes) -> int:
        a = np.frombuffer(w, dtype=np.uint8)
        assert a.size >= SEG
        return int(self._hash(_p(a, _u8p)))

    def window_hashes(self, x: bytes) -> np.ndarray:
        a = np.frombuffer(x, dtype=np.uint8)
        n = max(0, a.size - SEG + 1)
        out = np.zeros(n, dtype=np.uint64)
        if n:
            self._wh(_p(a, _u8p), a.size, _p(out, _u64p))
        return out

    # ----------------------------------------------------------------- cache
    def cache_new(self, limit_bytes: int = 0):
        """XCodecMemoryCache(uuid) or, with limit_bytes, the bounded LRU variant
        XCodecMemoryCache(uuid, limit_bytes) (xcodec/xcodec_cache.h:277-288)."""
        return self._cnewl(limit_bytes) if limit_bytes else self._cnew()

    def cache_new_pair(self, memory_limit_bytes: int, disk_bytes: int):
        """XCodecCachePair(XCodecMemoryCache(uuid, memory_limit_bytes), disk of
        disk_bytes) -- wanproxy.conf's cache (xcodec/xcodec_cache.h:140-237,
        xcodec/xcodec_cache_disk.cc).  The reference build runs the real pair
        over a restated disk level (oracle/ref_driver.cc RefDiskCache)."""
        f = getattr(self.lib, self._pre + 'cache_new_pair')
        f.restype = C.c_void_p
        f.argtypes = [C.c_uint64, C.c_uint64]
        c = f(memory_limit_bytes, disk_bytes)
        if not c:
            raise ValueError('disk too small for one index block')
        return c

    def cache_open_pair(self, memory_limit_bytes: int, disk_bytes: int, path: str, local_uuid: str):
        """wanproxy.conf's pair over the disk volume file at `path`
        (XCodecDisk::open, xcodec_cache_disk.cc:824-871): reopened when the file
        holds a volume (the constructor's reload, :107-237), else fresh with
        local_uuid registered.  Reference build only (the restated RefDisk)."""
        f = getattr(self.lib, self._pre + 'cache_open_pair')
        f.restype = C.c_void_p
        f.argtypes = [C.c_uint64, C.c_uint64, C.c_char_p, C.c_char_p]
        c = f(memory_limit_bytes, disk_bytes, path.encode(), local_uuid.encode())
        if not c:
            raise RuntimeError('could not open the volume')
        return c

    def cache_pair_front(self, pair, uuid: str, memory_limit_bytes: int):
        """A fresh pair over `uuid`'s front of the disk under `pair` (a
        restarted process's connect on a reopened volume)."""
        f = getattr(self.lib, self._pre + 'cache_pair_front')
        f.restype = C.c_void_p
        f.argtypes = [C.c_void_p, C.c_char_p, C.c_uint64]
        c = f(pair, uuid.encode(), memory_limit_bytes)
        if not c:
            raise RuntimeError('connect failed')
        return c

    def disk_save(self, pair, path: str):
        """Write the volume under `pair` as the reference's file stands now."""
        f = getattr(self.lib, self._pre + 'disk_save')
        f.argtypes = [C.c_void_p, C.c_char_p]
        if f(pair, path.encode()) != 0:
            raise RuntimeError('could not write the volume')

    def pair_stats(self, c, disk_live=False):
        """(disk index entries, disk entries written) of a pair cache; with
        disk_live, also the index entries of every front on its disk."""
        st = np.zeros(4, np.uint64)
        if self.ref:
            f = getattr(self.lib, self._pre + 'pair_stats')
            f.argtypes = [C.c_void_p, _u64p]
            f(c, _p(st, _u64p))
            return (int(st[0]), int(st[1]), int(st[2])) if disk_live else (int(st[0]), int(st[1]))
        self.lib.xco_pair_stats.argtypes = [C.c_void_p, _u64p]
        self.lib.xco_pair_stats(c, _p(st, _u64p))
        return int(st[1]), int(st[2])

    def cache_free(self, c):
        self._cfree(c)

    def cache_connect(self, parent, uuid: str):
        """XCodecCache::connect(uuid, parent) (xcodec/xcodec_cache.h:101-111): what
        XCodecPipePair's decoding side makes on <HELLO> (xcodec_pipe_pair.cc:203).
        Reference / drop-in builds; the cache lives for the process."""
        f = getattr(self.lib, self._pre + 'cache_connect')
        f.restype = C.c_void_p
        f.argtypes = [C.c_void_p, C.c_char_p]
        c = f(parent, uuid.encode())
        if not c:
            raise RuntimeError('connect failed')
        return c

    def cache_learn(self, cache, seg: bytes):
        """XCodecPipePair's <LEARN> of one segment (xcodec_pipe_pair.cc:296-327)."""
        f = getattr(self.lib, self._pre + 'cache_learn')
        f.argtypes = [C.c_void_p, C.c_char_p]
        assert len(seg) == SEG
        f(cache, seg)

    # ---------------------------------------------------------------- encode
    def encode_batch(self, data, offs, lens, mode=MODE_INDEPENDENT, oob=False, cache=None):
        """Encode chunks data[offs[i]:offs[i]+lens[i]]; returns list of bytes."""
        a = np.frombuffer(data, dtype=np.uint8) if not isinstance(data, np.ndarray) else data
        offs = np.ascontiguousarray(offs, dtype=np.uint64)
        lens = np.ascontiguousarray(lens, dtype=np.uint32)
        n = offs.size
        bounds = 2 * lens.astype(np.uint64) + 16
        oo = np.zeros(n, dtype=np.uint64)
        if n > 1:
            oo[1:] = np.cumsum(bounds)[:-1]
        out = np.zeros(int(bounds.sum()) + 1, dtype=np.uint8)
        ol = np.zeros(n, dtype=np.uint64)
        if self.ref:
            assert oob == (mode == MODE_NULL), 'reference OOB mode is the null cache'
            rc = self._eb(cache, _p(a, _u8p), _p(offs, _u64p), _p(lens, _u32p), n, mode,
                          _p(out, _u8p), _p(oo, _u64p), _p(ol, _u64p))
        else:
            rc = self._eb(cache, _p(a, _u8p), _p(offs, _u64p), _p(lens, _u32p), n, mode, int(oob),
                          _p(out, _u8p), _p(oo, _u64p), _p(ol, _u64p))
        if rc != 0:
            raise RuntimeError('oracle encode failed')
        return [out[int(oo[i]):int(oo[i] + ol[i])].tobytes() for i in range(n)]

    def encode_stream(self, data: bytes, chunk=65536, mode=MODE_STREAM, oob=False, cache=None) -> bytes:
        from wanproxy_amd.synth import chunks_of
        offs, lens = chunks_of(data, chunk)
        return b''.join(self.encode_batch(data, offs, lens, mode=mode, oob=oob, cache=cache))

    # ------------------------------------------------- encode with a refmap
    def encoder_new(self, cache):
        """A persistent XCodecEncoder on `cache` (reference / drop-in builds)."""
        f = getattr(self.lib, self._pre + 'encoder_new')
        f.restype = C.c_void_p
        f.argtypes = [C.c_void_p]
        return f(cache)

    def encoder_free(self, enc):
        f = getattr(self.lib, self._pre + 'encoder_free')
        f.argtypes = [C.c_void_p]
        f(enc)

    def encode_refmap(self, enc, data: bytes):
        """One encode(output, input, &refmap) call: (output, {hash: segment})."""
        f = getattr(self.lib, self._pre + 'encode_refmap')
        f.argtypes = [C.c_void_p, _u8p, C.c_uint64, _u8p, C.c_uint64, _u64p, _u64p, _u8p, C.c_uint64, _u64p]
        f.restype = C.c_int
        a = np.frombuffer(data, dtype=np.uint8)
        out = np.zeros(2 * a.size + 16, dtype=np.uint8)
        ol = np.zeros(1, dtype=np.uint64)
        mx = a.size // SEG + 1
        hs = np.zeros(mx, dtype=np.uint64)
        segs = np.zeros(mx * SEG, dtype=np.uint8)
        nref = np.zeros(1, dtype=np.uint64)
        if f(enc, _p(a, _u8p), a.size, _p(out, _u8p), out.size, _p(ol, _u64p), _p(hs, _u64p), _p(segs, _u8p), mx,
             _p(nref, _u64p)) != 0:
            raise RuntimeError('encode overflow')
        refs = {int(hs[k]): segs[k * SEG:(k + 1) * SEG].tobytes() for k in range(int(nref[0]))}
        return out[:int(ol[0])].tobytes(), refs

    # ---------------------------------------------------------------- decode
    def decoder_new(self, cache):
        """A persistent XCodecDecoder on `cache` (its BACKREF window lives
        across decode() calls)."""
        return self._dnew(cache) if self.ref else self.lib.xco_decoder_new(cache)

    def decoder_free(self, d):
        if self.ref:
            self._dfree(d)
        else:
            self.lib.xco_decoder_free(d)

    def decode(self, enc: bytes, cache, out_cap=None, decoder=None):
        """One XCodecDecoder::decode over `enc`.  Returns (ok, out, consumed, unknown)."""
        a = np.frombuffer(enc, dtype=np.uint8)
        cap = out_cap or (a.size // 3 + 1) * SEG + a.size   # a 3-byte BACKREF expands to 2048
        out = np.zeros(cap, dtype=np.uint8)
        ol = np.zeros(1, dtype=np.uint64)
        cons = np.zeros(1, dtype=np.uint64)
        unk = np.zeros(4096, dtype=np.uint64)
        nunk = np.zeros(1, dtype=np.uint64)
        if self.ref and decoder is not None:
            rc = self._ddec(decoder, _p(a, _u8p), a.size, _p(out, _u8p), cap, _p(ol, _u64p), _p(cons, _u64p),
                            _p(unk, _u64p), _p(nunk, _u64p), unk.size)
        elif self.ref:
            rc = self._dec(cache, _p(a, _u8p), a.size, _p(out, _u8p), cap, _p(ol, _u64p), _p(cons, _u64p),
                           _p(unk, _u64p), _p(nunk, _u64p), unk.size)
        else:
            d = decoder if decoder is not None else self.lib.xco_decoder_new(cache)
            rc = self.lib.xco_decode(d, _p(a, _u8p), a.size, _p(out, _u8p), cap, _p(ol, _u64p), _p(cons, _u64p),
                                     _p(unk, _u64p), _p(nunk, _u64p), unk.size)
            if decoder is None:
                self.lib.xco_decoder_free(d)
        if rc < 0:
            raise RuntimeError('decode overflow')
        return bool(rc), out[:int(ol[0])].tobytes(), int(cons[0]), [int(u) for u in unk[:int(nunk[0])]]
