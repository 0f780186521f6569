"""zlib stage checkers -- TEST INFRASTRUCTURE ONLY.

`DeflatePipeRef` drives the system zlib (1.2.11 in this image and on the GPU
box; the pinned version of the dependency wanproxy's zlib stage links) in the
exact call pattern of the reference's DeflatePipe::consume
(zlib/deflate_pipe.cc:57-115), through oracle/deflate_pipe_ref.c: every Buffer
segment through deflate(Z_NO_FLUSH), then one deflate(Z_SYNC_FLUSH) into the
pipe's 64 KiB buffer; an empty consume is EOS, deflate(Z_FINISH).
`InflatePipeRef` is the matching InflatePipe::consume (zlib/inflate_pipe.cc:
54-139): inflate(Z_NO_FLUSH) per segment, then Z_SYNC_FLUSH / Z_FINISH.

`ZOracle` loads oracle/build/libzoracle.so, the C restatement of zlib's
deflate in the GPU's formulation (oracle/zlib_oracle.c), pinned to
DeflatePipeRef by tests/test_zlib_oracle.py.
"""
from __future__ import annotations

import ctypes as C
import os
import zlib

HERE = os.path.dirname(os.path.abspath(__file__))
ZLIB_VERSION = '1.2.11'


class DeflatePipeRef:
    """DeflatePipe(level) over the system zlib in the pipe's exact call pattern
    (oracle/deflate_pipe_ref.c restates deflate_pipe.cc:57-115: segments of at
    most 2048 bytes through deflate(Z_NO_FLUSH), then ONE deflate(Z_SYNC_FLUSH)
    into the 64 KiB buffer; a full buffer ends the consume with output still
    pending in zlib and, when a block flush filled it, no sync marker)."""

    def __init__(self, level: int = 6):
        lib = ZOracle.lib()
        self.s = lib.dpr_create(level)
        if not self.s:
            raise ValueError(f'deflateInit({level}) failed')

    def consume(self, data: bytes, segments=None) -> bytes:
        """One consume(): the bytes of one Buffer, cut into `segments` lengths
        (default: 2048-byte segments, BUFFER_SEGMENT_SIZE); b'' = EOS.  Returns
        what the pipe produces."""
        lib = ZOracle.lib()
        cap = 2 * len(data) + 4 * 65536 + 1024
        buf = C.create_string_buffer(cap)
        if segments is None:
            seg, nseg = None, 0
        else:
            arr = (C.c_uint32 * max(1, len(segments)))(*segments)
            seg, nseg = arr, len(segments)
        n = lib.dpr_consume(self.s, data, len(data), seg, nseg, buf, cap)
        if n < 0:
            raise RuntimeError('dpr_consume failed')
        return buf.raw[:n]

    def close(self):
        if getattr(self, 's', None):
            ZOracle.lib().dpr_free(self.s)
            self.s = None

    def __del__(self):
        self.close()


class DeflatePipeUnbounded:
    """zlib driven with unbounded output per call (Python's zlib module): the
    stream a DeflatePipe would emit if its flush call never ran out of room.
    Kept to show where DeflatePipeRef's 64 KiB buffer changes the bytes."""

    def __init__(self, level: int = 6):
        self.z = zlib.compressobj(level, zlib.DEFLATED, 15, 8, zlib.Z_DEFAULT_STRATEGY)
        self.done = False

    def consume(self, data: bytes) -> bytes:
        if self.done:
            return b''
        if not data:
            self.done = True
            return self.z.flush(zlib.Z_FINISH)
        return self.z.compress(data) + self.z.flush(zlib.Z_SYNC_FLUSH)


class InflatePipeRef:
    def __init__(self):
        self.z = zlib.decompressobj(15)

    def consume(self, data: bytes) -> bytes:
        return self.z.decompress(data)


class ZOracle:
    """C restatement: one object per stream (DeflatePipe)."""
    _lib = None

    @classmethod
    def lib(cls):
        if cls._lib is None:
            path = os.path.join(HERE, 'build', 'libzoracle.so')
            lib = C.CDLL(path)
            lib.zr_create.restype = C.c_void_p
            lib.zr_create.argtypes = [C.c_int]
            lib.zr_free.argtypes = [C.c_void_p]
            lib.zr_consume.restype = C.c_int64
            lib.zr_consume.argtypes = [C.c_void_p, C.c_char_p, C.c_uint64, C.c_char_p, C.c_uint64]
            lib.zr_bound.restype = C.c_uint64
            lib.zr_bound.argtypes = [C.c_uint64]
            lib.dpr_create.restype = C.c_void_p
            lib.dpr_create.argtypes = [C.c_int]
            lib.dpr_free.argtypes = [C.c_void_p]
            lib.dpr_consume.restype = C.c_int64
            lib.dpr_consume.argtypes = [C.c_void_p, C.c_char_p, C.c_uint64, C.c_void_p, C.c_uint32,
                                        C.c_char_p, C.c_uint64]
            cls._lib = lib
        return cls._lib

    def __init__(self, level: int = 6):
        self.s = self.lib().zr_create(level)
        if not self.s:
            raise ValueError(f'level {level} not restated (1-9 only)')

    def consume(self, data: bytes) -> bytes:
        lib = self.lib()
        cap = lib.zr_bound(len(data))
        buf = C.create_string_buffer(cap)
        n = lib.zr_consume(self.s, data, len(data), buf, cap)
        if n < 0:
            raise RuntimeError('zr_consume: output bound exceeded')
        return buf.raw[:n]

    def close(self):
        if self.s:
            self.lib().zr_free(self.s)
            self.s = None

    def __del__(self):
        self.close()


class ReferencePipes:
    """wanproxy's DeflatePipe / InflatePipe classes themselves, through
    oracle/zpipe_driver.cc: `ref` = the reference's zlib/deflate_pipe.cc and
    zlib/inflate_pipe.cc compiled from /root/reference over the system zlib
    (oracle/_ref/libzpref.so); `dropin` = integration/zlib_pipes_xcgpu.cc, the
    engine-backed bodies of the same classes (oracle/_ref/libzpdropin.so)."""
    _libs = {}

    def __init__(self, which: str = 'ref'):
        if which not in self._libs:
            name = {'ref': 'libzpref.so', 'dropin': 'libzpdropin.so'}[which]
            L = C.CDLL(os.path.join(HERE, '_ref', name))
            L.zp_new.restype = C.c_void_p
            L.zp_new.argtypes = [C.c_int, C.c_int]
            L.zp_free.argtypes = [C.c_void_p, C.c_int]
            L.zp_consume.restype = C.c_int64
            L.zp_consume.argtypes = [C.c_void_p, C.c_int, C.c_char_p, C.c_uint64, C.c_void_p, C.c_uint32, C.c_char_p,
                                     C.c_uint64, C.POINTER(C.c_int)]
            self._libs[which] = L
        self.L = self._libs[which]

    def pipe(self, kind: str, level: int = 6) -> 'ReferencePipe':
        return ReferencePipe(self.L, 0 if kind == 'deflate' else 1, level)


class ReferencePipe:
    def __init__(self, L, kind: int, level: int):
        self.L, self.kind = L, kind
        self.h = L.zp_new(kind, level)

    def consume(self, data: bytes, segments=None):
        """-> (produced bytes, status: 0 produce, 1 produce_eos, -1 produce_error)"""
        arr = (C.c_uint32 * max(1, len(segments)))(*segments) if segments else None
        cap = 8 * len(data) + 4 * 65536 + 4096
        buf = C.create_string_buffer(cap)
        st = C.c_int(0)
        n = self.L.zp_consume(self.h, self.kind, data, len(data), arr, len(segments) if segments else 0, buf, cap,
                              C.byref(st))
        if n < 0:
            raise RuntimeError('zp_consume: output room')
        return buf.raw[:n], st.value

    def close(self):
        if getattr(self, 'h', None):
            self.L.zp_free(self.h, self.kind)
            self.h = None

    def __del__(self):
        self.close()
