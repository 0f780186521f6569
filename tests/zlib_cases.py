"""Deterministic inputs for the zlib-stage tests (CPU oracle and GPU parity).

Each case is (level, [call bytes...]); the last call of a stream may be b''
(EOS -> deflate(Z_FINISH), zlib/deflate_pipe.cc:72-75).  The generators aim
at deflate's edge cases: long runs (258-byte matches, nice-length breaks),
skewed alphabets (Huffman length overflow in gen_bitlen), incompressible
bytes (stored blocks), copies at distances near MAX_DIST / TOO_FAR, calls
whose ends fall where the window slides (strstart 65274 / 65275) and tiny
calls (pending hash insertions across calls)."""
from __future__ import annotations

import random


def gen_bytes(rng: random.Random, n: int) -> bytes:
    mode = rng.random()
    out = bytearray()
    while len(out) < n:
        k = rng.random()
        if mode < 0.2:
            nsym = rng.randint(2, 255)
            w = [2 ** rng.randint(0, 14) for _ in range(nsym)]
            out += bytes(rng.choices(range(nsym), weights=w, k=rng.randint(1, 3000)))
        elif k < 0.15:
            out += bytes([rng.randrange(256)]) * rng.randint(1, 2000)
        elif k < 0.35:
            out += rng.randbytes(rng.randint(1, 4000))
        elif k < 0.7 and len(out) > 10:
            a = rng.randrange(len(out))
            if rng.random() < 0.3 and len(out) > 33000:
                a = len(out) - rng.choice([32506, 32505, 32507, 4096, 4097, 32768])
            for j in range(rng.randint(3, 600)):
                out.append(out[a + j] if a + j < len(out) else 0)
        else:
            out += bytes(rng.choice(b'ab\x00\xff ') for _ in range(rng.randint(1, 3000)))
    return bytes(out[:n])


SIZE_PATTERNS = [
    [1, 2, 1, 5], [65274, 300], [32506, 32768, 261], [65536] * 3, [100000, 7],
    [262, 258, 3, 65000, 65536, 33000], [65275], [65274 + 258, 1], [131072],
]


def cases(seed: int, n: int, max_extra: int = 150000):
    rng = random.Random(seed)
    out = []
    for _ in range(n):
        level = rng.choice([4, 5, 6, 6, 7, 8, 9])
        sizes = list(rng.choice(SIZE_PATTERNS))
        sizes += [rng.randint(1, max_extra) for _ in range(rng.randint(0, 3))]
        calls = [gen_bytes(rng, s) for s in sizes]
        if rng.random() < 0.8:
            calls.append(b'')
        out.append((level, calls))
    return out


def fast_cases(seed: int, n: int, max_extra: int = 150000):
    """As cases(), at the deflate_fast levels 1-3."""
    rng = random.Random(seed)
    return [(rng.choice([1, 2, 3]), calls) for _, calls in cases(seed, n, max_extra)]


def stored_cases(seed: int, n: int):
    """Level 0 (deflate_stored): consumes around its 32 KiB / 64 KiB thresholds."""
    rng = random.Random(seed)
    out = []
    for _ in range(n):
        sizes = [rng.choice([1, 7, 2048, 32763, 32768, 40000, 65530, 65536, 70000, 140000, rng.randint(1, 200000)])
                 for _ in range(rng.randint(1, 6))]
        calls = [gen_bytes(rng, s) for s in sizes]
        if rng.random() < 0.8:
            calls.append(b'')
        out.append((0, calls))
    return out


def stop_cases(seed: int, levels=(1, 3, 4, 6, 9), offsets=range(-3, 270, 9)):
    """Streams whose first consume is 4 * 16383 + j incompressible bytes: the
    fourth block flush falls at loop top 65532 + j - ... of the call, inside
    the Z_SYNC_FLUSH call's last MIN_LOOKAHEAD positions for most j, where the
    pipe's 64 KiB buffer (deflate_pipe.cc:34,101-105) is full -- the consume
    stops there and the rest of its positions are parsed with the next one's
    bytes.  Then a short consume, another such consume and EOS."""
    rng = random.Random(seed)
    out = []
    for level in levels:
        for j in offsets:
            out.append((level, [rng.randbytes(4 * 16383 + j), rng.randbytes(rng.randint(1, 70000)),
                                rng.randbytes(4 * 16383 + j), b'']))
    return out


def wan_stream(seed: int, ncalls: int, call_bytes: int) -> list:
    """XCodec-output-like traffic: frames of mostly incompressible bytes with
    escapes, references (F1 02 + 8 bytes) and repeated literal runs."""
    rng = random.Random(seed)
    calls = []
    for _ in range(ncalls):
        b = bytearray()
        while len(b) < call_bytes:
            k = rng.random()
            if k < 0.4:
                b += rng.randbytes(rng.randint(16, 2048))
            elif k < 0.7:
                b += b'\xf1\x02' + rng.randbytes(8)
            else:
                b += bytes(rng.choice(b'GET /index.html HTTP/1.1\r\nHost: example\r\n\r\n') for _ in range(rng.randint(8, 512)))
        calls.append(bytes(b[:call_bytes]))
    return calls
