"""Synthetic XCodec workloads (the survey's deterministic generator).

BASELINE.md "Generator for kat_a/b/c" defines a splitmix64 stream of 2048-byte
blocks, each either a fresh block (256 little-endian draws, optionally with
bytes forced to the XCodec magic 0xF1) or, with probability dup%, a copy of an
earlier fresh block.  This module reproduces that stream bit-exactly, but draws
the block bodies vectorised with numpy: splitmix64's n-th output is a pure
function of seed + n * gamma, so only the per-block control draws are walked
sequentially.  Used by tests/ and bench.py to build inputs.
"""
from __future__ import annotations

import numpy as np

GAMMA = 0x9E3779B97F4A7C15
M64 = (1 << 64) - 1
SEG = 2048


def _mix(z: np.ndarray) -> np.ndarray:
    z = z.astype(np.uint64, copy=True)
    z ^= z >> np.uint64(30)
    z *= np.uint64(0xBF58476D1CE4E5B9)
    z ^= z >> np.uint64(27)
    z *= np.uint64(0x94D049BB133111EB)
    z ^= z >> np.uint64(31)
    return z


def _draw(seed: int, idx: np.ndarray) -> np.ndarray:
    """Values of the idx-th (0-based) next() call of SM(seed)."""
    x = (np.uint64(seed & M64) + (idx.astype(np.uint64) + np.uint64(1)) * np.uint64(GAMMA))
    return _mix(x)


def _draw1(seed: int, i: int) -> int:
    return int(_draw(seed, np.array([i], dtype=np.uint64))[0])


_CTL = {}


def _control(seed: int, nblocks: int, dup_pct: int, magic_pct: int):
    """The generator's sequential control walk over the first `nblocks` blocks:
    (draw index of the first body draw of each fresh block, fresh-block id of
    each block).  Cached per (seed, dup, magic) and extended on demand."""
    key = (seed, dup_pct, magic_pct)
    st = _CTL.get(key)
    if st is None:
        st = _CTL[key] = {'pos': 0, 'fresh': [], 'order': []}
    fresh_starts, order = st['fresh'], st['order']
    if len(order) < nblocks:
        per_fresh = 256 + (SEG if magic_pct else 0)
        pos = st['pos']
        cache_base, cache = -1, None

        def ctl(i: int) -> int:
            nonlocal cache_base, cache
            if cache is None or not (cache_base <= i < cache_base + len(cache)):
                cache_base = i
                cache = _draw(seed, np.arange(i, i + 4096, dtype=np.uint64)).tolist()
            return cache[i - cache_base]

        for _ in range(nblocks - len(order)):
            if fresh_starts and dup_pct > 0:
                r = ctl(pos); pos += 1
                if r % 100 < dup_pct:
                    order.append(ctl(pos) % len(fresh_starts)); pos += 1
                    continue
            elif fresh_starts:
                pos += 1          # `r.next() % 100 < 0` still consumes a draw
            fresh_starts.append(pos)
            order.append(len(fresh_starts) - 1)
            pos += per_fresh
        st['pos'] = pos
    return fresh_starts, order


_SYNTH = None


def _csynth():
    """csrc/xcg_synth.c (built by build.py / __graft_entry__.build()), or None."""
    global _SYNTH
    if _SYNTH is None:
        import ctypes as C
        import os
        p = os.path.join(os.path.dirname(os.path.abspath(__file__)), 'libxcsynth.so')
        _SYNTH = False
        if os.path.exists(p):
            L = C.CDLL(p)
            L.xcs_stream_range.argtypes = [C.c_uint64, C.c_uint32, C.c_uint32, C.c_uint64, C.c_uint64, C.c_void_p]
            L.xcs_stream_range.restype = C.c_int
            _SYNTH = L
    return _SYNTH or None


def stream_range(seed: int, dup_pct: int, magic_pct: int, lo: int, hi: int, use_c: bool = True) -> np.ndarray:
    """Bytes [lo, hi) of the generator's stream (any stream of >= hi bytes has
    this prefix), built so memory stays ~ (hi - lo): a rank's shard of a long
    stream without materialising the rest.  Uses the C build of
    the same generator when present (8 GiB streams), else numpy."""
    if hi <= lo:
        return np.zeros(0, np.uint8)
    L = _csynth() if use_c else None
    if L is not None:
        out = np.empty(hi - lo, np.uint8)
        if L.xcs_stream_range(seed & M64, dup_pct, magic_pct, lo, hi, out.ctypes.data) != 0:
            raise MemoryError('xcs_stream_range')
        return out
    b0, b1 = lo // SEG, (hi + SEG - 1) // SEG
    fresh_starts, order = _control(seed, b1, dup_pct, magic_pct)
    starts = np.asarray(fresh_starts, dtype=np.uint64)
    ords = np.asarray(order[b0:b1], dtype=np.int64)
    out = np.empty((b1 - b0) * SEG, np.uint8)
    PIECE = 16384
    for a in range(0, b1 - b0, PIECE):
        st = starts[ords[a:a + PIECE]]
        body_idx = st[:, None] + np.arange(256, dtype=np.uint64)[None, :]
        blk = _draw(seed, body_idx).astype('<u8').view(np.uint8).reshape(st.size, SEG)
        if magic_pct:
            midx = st[:, None] + np.uint64(256) + np.arange(SEG, dtype=np.uint64)[None, :]
            blk[(_draw(seed, midx) % np.uint64(100)) < np.uint64(magic_pct)] = 0xF1
        out[a * SEG:(a + st.size) * SEG] = blk.reshape(-1)
    return out[lo - b0 * SEG:hi - b0 * SEG]


def stream(seed: int, nbytes: int, dup_pct: int, magic_pct: int = 0) -> bytes:
    """Bit-exact port of BASELINE.md's `stream(seed, nbytes, dup, magic)`."""
    return stream_range(seed, dup_pct, magic_pct, 0, nbytes).tobytes()


def dense(seed: int, nbytes: int, distinct: int, shift_every: int = 64) -> bytes:
    """REF-dense input (not a BASELINE.md dataset): 2048-byte blocks drawn
    uniformly from a pool of `distinct` random segments, with a short random
    literal (1..300 bytes) after every `shift_every`-th block on average so the
    alignment moves.  Every block after a pool entry's first use can be a REF:
    per entity thousands of cache references in one batch (the pair replay's
    long runs)."""
    rng = np.random.default_rng(seed)
    pool = rng.integers(0, 256, (distinct, SEG), dtype=np.uint8)
    nblk = nbytes // SEG + 1
    data = pool[rng.integers(0, distinct, nblk)].reshape(-1)
    nins = max(1, nblk // shift_every)
    at = np.sort(rng.integers(0, nblk, nins)) * SEG
    lens = rng.integers(1, 301, nins)
    data = np.insert(data, np.repeat(at, lens), rng.integers(0, 256, int(lens.sum()), dtype=np.uint8))
    return data[:nbytes].tobytes()


def stream_ref(seed: int, nbytes: int, dup_pct: int, magic_pct: int = 0) -> bytes:
    """The BASELINE.md generator verbatim in pure Python (slow; for tests)."""
    class SM:
        def __init__(s, seed):
            s.x = seed & M64

        def next(s):
            s.x = (s.x + GAMMA) & M64
            z = s.x
            z = ((z ^ (z >> 30)) * 0xBF58476D1CE4E5B9) & M64
            z = ((z ^ (z >> 27)) * 0x94D049BB133111EB) & M64
            return z ^ (z >> 31)

    def block(r):
        return b''.join(r.next().to_bytes(8, 'little') for _ in range(256))

    r = SM(seed)
    out = bytearray()
    blocks = []
    while len(out) < nbytes:
        if blocks and r.next() % 100 < dup_pct:
            b = blocks[r.next() % len(blocks)]
        else:
            b = bytearray(block(r))
            if magic_pct:
                for i in range(SEG):
                    if r.next() % 100 < magic_pct:
                        b[i] = 0xF1
            b = bytes(b)
            blocks.append(b)
        out += b
    return bytes(out[:nbytes])


def kat_col() -> bytes:
    """BASELINE.md "kat_col construction": X || Y || Z || Y || X with H(X)==H(Y)."""
    import random
    r = random.Random(42)
    X = bytearray(r.getrandbits(8) | 1 for _ in range(SEG))
    for i in range(SEG):
        if X[i] > 250:
            X[i] = 201
        if X[i] < 6:
            X[i] = 7
    Y = bytearray(X)
    k = 100
    Y[k] += 2
    Y[k + 1] -= 4
    Y[k + 2] += 2
    Z = bytes(r.getrandbits(8) for _ in range(3000))
    return bytes(X) + bytes(Y) + Z + bytes(Y) + bytes(X)


def kat_blocks() -> bytes:
    """BASELINE.md additional KAT: 128 draws of 16 random 8 KiB blocks."""
    import random
    random.seed(1)
    blk = [bytes(random.getrandbits(8) for _ in range(8192)) for _ in range(16)]
    return b''.join(random.choice(blk) for _ in range(128))


KATS = {
    'kat_a': lambda: stream(0x5eed, 1048576, 50, 0),
    'kat_b': lambda: stream(0xb0b, 1048576, 50, 2),
    'kat_c': lambda: stream(0xc0de, 300001, 0, 0),
    'kat_z': lambda: bytes(65536),
    'kat_col': kat_col,
    'kat_blocks': kat_blocks,
}


def chunks_of(data: bytes, size: int):
    """Offsets/lengths of tack's read() loop over a regular file (<= size each)."""
    n = len(data)
    offs = np.arange(0, n, size, dtype=np.uint64)
    lens = np.minimum(size, n - offs.astype(np.int64)).astype(np.uint32)
    return offs, lens
