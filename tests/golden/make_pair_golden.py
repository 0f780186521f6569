#!/usr/bin/env python3
"""Regenerate tests/golden/pair.json from the REAL reference XCodecCachePair
(xcodec/xcodec_cache.h:140-237) of a bounded XCodecMemoryCache primary
(:245-365, xcodec/xcodec_lru.h) and a disk secondary -- wanproxy.conf's cache
(programs/wanproxy/wanproxy.conf:8-26).  The disk level is oracle/ref_driver.cc
RefDiskCache, a restatement of XCodecDisk / XCodecDiskCache
(xcodec/xcodec_cache_disk.{h,cc}), which cannot be compiled here (libuuid's
header is absent); the pair, encoder, decoder, LRU and Buffer code are the
reference's own.

Run in the build container only (needs oracle/_ref/libxcref.so).  Inputs are
regenerated deterministically by `inputs()`; per (input, chunk, memory limit,
disk size) the JSON holds the per-encode() lengths + SHA-256 prefixes of one
XCodecEncoder on one pair (tack's loop), the disk counters after the stream
(index entries, entries written), and what one persistent reference
XCodecDecoder on a pair of the same geometry returns for each frame.
"""
from __future__ import annotations

import hashlib
import importlib.util
import json
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, ROOT)

from wanproxy_amd import synth  # noqa: E402

_spec = importlib.util.spec_from_file_location('make_lru_golden', os.path.join(HERE, 'make_lru_golden.py'))
_mlg = importlib.util.module_from_spec(_spec)
_spec.loader.exec_module(_mlg)

SEG = 2048
KiB, MiB = 1024, 1 << 20

INPUTS = {
    # repeats reach far back: past the primary, served by the disk (promotions)
    'pair_far': ('recency', 0x9A1, 3 << 20, 55, 1200),
    # hot set reused over a disk that laps: primary hits re-enter lost hashes (touch)
    'pair_hot': ('hot', 0x9A2, 3 << 20, 70, 400),
    'pair_uniform': ('stream', 0x9A3, 4 << 20, 40, 1),
    'pair_col': ('kat', 'kat_col'),
}


def hot_stream(seed: int, nbytes: int, dup: int, span: int) -> bytes:
    """Block-aligned 2 KiB blocks (no odd fragments, so declarations stay on
    block boundaries): `dup` % repeat one of the last `span` distinct blocks,
    the most recent ones most often -- a hot set a small primary keeps while a
    small disk laps past it."""
    import numpy as np
    rng = np.random.default_rng(seed)
    blocks: list[bytes] = []
    out = bytearray()
    while len(out) < nbytes:
        if blocks and rng.random() < dup / 100.0:
            back = int(min(len(blocks), span) * rng.random() ** 3)
            out += blocks[len(blocks) - 1 - back]
        else:
            b = rng.integers(0, 256, size=SEG, dtype=np.uint8).tobytes()
            blocks.append(b)
            out += b
    return bytes(out[:nbytes])


def inputs(name: str) -> bytes:
    spec = INPUTS[name]
    if spec[0] == 'recency':
        return _mlg.recency_stream(*spec[1:])
    if spec[0] == 'hot':
        return hot_stream(*spec[1:])
    if spec[0] == 'stream':
        return synth.stream(*spec[1:])
    return synth.KATS[spec[1]]()


def disk_bytes(index_blocks: int) -> int:
    """A volume with exactly `index_blocks` index blocks (xcodec_cache_disk.cc:110-111)."""
    return (18 + 205 * index_blocks) * SEG


CASES = [  # (input, chunk size, memory_cache_limit_bytes, disk bytes)
    ('pair_far', 65536, 256 * SEG, disk_bytes(8)),
    ('pair_far', 65536, 64 * SEG, disk_bytes(2)),
    ('pair_far', 131072, 200 * SEG, disk_bytes(30)),
    ('pair_far', 4096, 300 * SEG, disk_bytes(4)),
    ('pair_hot', 65536, 200 * SEG, disk_bytes(1)),
    ('pair_hot', 65536, 400 * SEG, disk_bytes(2)),
    ('pair_hot', 32768, 100 * SEG, disk_bytes(3)),
    ('pair_uniform', 65536, 300 * SEG, disk_bytes(6)),
    ('pair_uniform', 131072, 1000 * SEG, disk_bytes(40)),
    ('pair_uniform', 65536, 1, disk_bytes(3)),
    ('pair_col', 65536, 3 * SEG, disk_bytes(1)),
    ('pair_col', 4096, 2 * SEG, disk_bytes(1)),
]


def sha(b: bytes) -> str:
    return hashlib.sha256(b).hexdigest()


def main():
    from oracle.lib import MODE_STREAM, Oracle
    ref = Oracle(ref=True)
    out = {'generator': 'tests/golden/make_pair_golden.py', 'inputs': {}, 'cases': []}
    for name in INPUTS:
        d = inputs(name)
        out['inputs'][name] = {'len': len(d), 'sha256': sha(d)}
    for name, chunk, limit, disk in CASES:
        d = inputs(name)
        offs, lens = synth.chunks_of(d, chunk)
        cache = ref.cache_new_pair(limit, disk)
        encs = ref.encode_batch(d, offs, lens, mode=MODE_STREAM, cache=cache)
        entries, written = ref.pair_stats(cache)
        ref.cache_free(cache)
        dcache = ref.cache_new_pair(limit, disk)
        dec = ref.decoder_new(dcache)
        calls = []
        for e in encs:
            ok, o, cons, unk = ref.decode(e, dcache, decoder=dec)
            calls.append({'ok': ok, 'consumed': cons, 'nunknown': len(unk), 'out_len': len(o), 'out_sha256': sha(o)})
            if not ok or unk:
                break
        ref.decoder_free(dec)
        ref.cache_free(dcache)
        out['cases'].append({'input': name, 'chunk': chunk, 'limit': limit, 'disk': disk, 'lens': [len(e) for e in encs],
                             'chunk_sha256': [sha(e)[:32] for e in encs], 'sha256': sha(b''.join(encs)),
                             'disk_entries': entries, 'disk_written': written, 'dec': calls})
        print(name, chunk, limit // SEG, 'segs', (disk // SEG - 18) // 205, 'index blocks:', len(encs), 'chunks',
              sum(map(len, encs)), 'bytes, disk', entries, '/', written, 'dec calls', len(calls),
              'blocked' if calls[-1]['nunknown'] else '')
    with open(os.path.join(HERE, 'pair.json'), 'w') as f:
        json.dump(out, f, indent=1)


if __name__ == '__main__':
    main()
