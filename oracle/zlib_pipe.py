"""zlib stage checkers -- TEST INFRASTRUCTURE ONLY.

`DeflatePipeRef` drives the system zlib (1.2.11 in this image and on the GPU
box; the pinned version of the dependency wanproxy's zlib stage links) in the
exact call pattern of the reference's DeflatePipe::consume
(zlib/deflate_pipe.cc:57-115): every input segment through deflate(Z_NO_FLUSH),
then deflate(Z_SYNC_FLUSH); an empty consume is EOS, deflate(Z_FINISH).
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
    def __init__(self, level: int = 6):
        # deflateInit(&stream_, level): windowBits 15, memLevel 8, default strategy
        self.z = zlib.compressobj(level, zlib.DEFLATED, 15, 8, zlib.Z_DEFAULT_STRATEGY)
        self.done = False

    def consume(self, data: bytes, segments=None) -> bytes:
        """One consume(): the bytes of one Buffer (cut into `segments` lengths,
        default one segment); b'' = EOS.  Returns what the pipe produces."""
        if self.done:
            return b''
        if not data:
            self.done = True
            return self.z.flush(zlib.Z_FINISH)
        out = []
        if segments is None:
            segments = [len(data)]
        i = 0
        for n in segments:
            out.append(self.z.compress(data[i:i + n]))
            i += n
        assert i == len(data)
        out.append(self.z.flush(zlib.Z_SYNC_FLUSH))
        return b''.join(out)


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
            cls._lib = lib
        return cls._lib

    def __init__(self, level: int = 6):
        self.s = self.lib().zr_create(level)
        if not self.s:
            raise ValueError(f'level {level} not restated (4-9 only)')

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
