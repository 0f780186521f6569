"""A worst case for the stream encoder's Jacobi rounds: a
declaration-dependence chain.  Chunk 0 = E_0; chunk k = z_k + E_{k-1} + E_k
(one byte, then the previous chunk's fresh block, then a fresh block).  In the
sequential encoder (xcodec_encoder.cc:183-248) chunk k finds E_{k-1} at offset
1 -- a REF, because chunk k-1 declared it -- and then declares E_k at offset
2049.  Had E_{k-1} not been declared, chunk k would instead declare its 2048-byte
tiling and never E_k, so chunk k+1 would miss too: every chunk's parse hangs
on the one before it, and neither a round-0 parse nor the tiling seed guesses
any of it."""
import numpy as np

SEG = 2048


def chain(n: int, seed: int = 7):
    r = np.random.default_rng(seed)
    E = [r.integers(0, 256, SEG, dtype=np.uint8).tobytes() for _ in range(n)]
    z = r.integers(0, 256, n, dtype=np.uint8).tobytes()
    parts = [E[0]] + [z[k:k + 1] + E[k - 1] + E[k] for k in range(1, n)]
    lens = np.array([len(p) for p in parts], np.uint32)
    offs = np.zeros(n, np.uint64)
    offs[1:] = np.cumsum(lens.astype(np.uint64))[:-1]
    return b''.join(parts), offs, lens
