#!/usr/bin/env python3
"""Regenerate tests/golden/golden.json from the REAL reference.

Run in the build container only (needs /root/reference and oracle/_ref/libxcref.so,
built by `make -C oracle`).  The GPU box never runs this script; it only reads
the committed JSON.  Inputs are NOT stored: they are regenerated bit-exactly by
wanproxy_amd.synth (pinned by the input SHA-256s below).  Expected outputs are
stored as SHA-256 + length (and as raw hex for the few short ones).

Contents
  hash_kats        256 single-character KATs, parsed from the reference test
                   xcodec/test/xcodec-hash1/xcodec-hash1.cc:34-291 (data only)
  baseline         SHA-256s published in BASELINE.md (survey runs of `tack`)
  cases            reference encodings (XCodecEncoder over the reference
                   XCodecMemoryCache / a null OOB cache) of synthetic inputs at
                   several chunkings and in three cache modes
"""
from __future__ import annotations

import hashlib
import json
import os
import re
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)

from oracle.lib import Oracle, MODE_INDEPENDENT, MODE_STREAM, MODE_NULL  # noqa: E402
from wanproxy_amd import synth  # noqa: E402

REF = '/root/reference'


def sha(b: bytes) -> str:
    return hashlib.sha256(b).hexdigest()


def hash_kats():
    src = open(os.path.join(REF, 'xcodec/test/xcodec-hash1/xcodec-hash1.cc')).read()
    body = src[src.index('char_kats[] = {'):]
    body = body[:body.index('};')]
    vals = [int(v, 16) for v in re.findall(r'0x([0-9a-fA-F]{16})ull', body)]
    assert len(vals) == 256, len(vals)
    return ['%016x' % v for v in vals]


BASELINE = {
    # name: (input sha, .xc bytes, .xc sha, .oob bytes, .oob sha)   -- BASELINE.md "KAT" table
    'kat_a': ('5b8dd221efd6c2380e8c199c710473b4b41044a3fe7efb6b1d80fe0ad8c05be2', 521240,
              '34532f4b4d56219ffb9d9f0c108d10c79e4f276e36dee3a29c9fc918228af116', 5120,
              '442597b5fbdea4961019f6f13d230732871699b41552bd47bf1e612fd571c857'),
    'kat_b': ('6bc2835f54c93c94bec43ef53e3b3714bb4b3dfb448065556c9564fe9c9c8990', 543680,
              '066d9d68cbc91608d237ea431c9adafe00c85af7fba9232eac1492bd548e6b56', 5120,
              '072fb47e754c26d1107d17ceb49c842f8d45f3a9e3b5f2375cd18dd2427fc868'),
    'kat_c': ('fda3f4080d011fd40a4e10890d9e4687cf65d638e13bce25fed34ebe9e247df5', 300296,
              'ff0ab15246fec3c4c12a5fd93a7e5c06306e25919145d5b24534745bf23b514f', 2456,
              '489083797a74a26ac03096e256d66bae60b16d8d55a0e1758dfeeed049ea6252'),
    'kat_z': ('de2f256064a0af797747c2b97505dc0b9f3df0de4f489eac731c23ae9ca9cc31', 2360,
              '37743e3adb3a5b8929ed5123706ef26ff6a4e68853c4a94ddd9861489145b32e', 320,
              'd03c3767ec78def9d7eff26bb1c77792133ffc2412dddc029d2aa7c7c0baf7cb'),
    'kat_col': ('16926f2183e0fae9ffb49131820952eee1a930be5e6bb892bd5ab35db39acba1', 9171,
                'ed7c8fd845d328ad6fb0a779a99b32bc3ddff1b48f992a61498de8e337c367af', None, None),
    'kat_blocks': ('5a3342d5bf2e2a94e189f4260255fd2f164d10c2ed3b0bf630fcbed0e26307f1', 135680,
                   '2fc77468752bbbcad2a9a4500018b405dc5dd98d88a944219a7d35bab7eda224', None, None),
}

# Inputs for `cases`: (name, generator spec).  Specs are evaluated by inputs().
INPUTS = {
    'kat_a': ('kat', 'kat_a'),
    'kat_b': ('kat', 'kat_b'),
    'kat_c': ('kat', 'kat_c'),
    'kat_z': ('kat', 'kat_z'),
    'kat_col': ('kat', 'kat_col'),
    'kat_blocks': ('kat', 'kat_blocks'),
    'c2_small': ('stream', 0xC2, 64 * 65536, 50, 0),           # C2 generator, 64 chunks
    'c4_small': ('stream', 0xC4, 256 * 4096, 4, 0),            # C4 generator, 256 packets
    'magic_heavy': ('stream', 0xF1F1, 262144, 30, 40),         # many 0xF1 bytes
    'runs': ('runs',),                                          # byte runs of varying length
    'periodic': ('periodic',),                                  # 1000-byte period text-like
    'all_f1': ('const', 0xF1, 70000),
    'ragged': ('ragged',),                                      # random chunk lengths 0..9000
}


def inputs(name):
    spec = INPUTS[name]
    if spec[0] == 'kat':
        return synth.KATS[spec[1]]()
    if spec[0] == 'stream':
        return synth.stream(*spec[1:])
    if spec[0] == 'const':
        return bytes([spec[1]]) * spec[2]
    if spec[0] == 'runs':
        rng = np.random.default_rng(12345)
        out = bytearray()
        while len(out) < 200000:
            out += bytes([int(rng.integers(0, 256))]) * int(rng.integers(1, 6000))
        return bytes(out[:200000])
    if spec[0] == 'periodic':
        rng = np.random.default_rng(777)
        pat = rng.integers(32, 127, size=1000, dtype=np.uint8).tobytes()
        return (pat * 200)[:180000]
    if spec[0] == 'ragged':
        return synth.stream(0x7a66, 400000, 35, 1)
    raise KeyError(name)


def chunking(name, data, chunk):
    if name == 'ragged' and chunk == 'ragged':
        rng = np.random.default_rng(99)
        lens = []
        tot = 0
        while tot < len(data):
            l = int(rng.choice([0, 1, 7, 2047, 2048, 2049, 4095, 4096, 4097, int(rng.integers(0, 9000))]))
            l = min(l, len(data) - tot)
            lens.append(l)
            tot += l
        lens = np.array(lens, dtype=np.uint32)
        offs = np.zeros(lens.size, dtype=np.uint64)
        offs[1:] = np.cumsum(lens.astype(np.uint64))[:-1]
        return offs, lens
    return synth.chunks_of(data, chunk)


CASES = [
    # (input, chunk size, mode)
    *[(k, 65536, m) for k in BASELINE for m in ('stream', 'null', 'independent')],
    ('kat_a', 4096, 'stream'), ('kat_a', 131072, 'stream'), ('kat_b', 4096, 'stream'),
    ('kat_b', 131072, 'stream'), ('kat_a', 524288, 'stream'),
    ('c2_small', 65536, 'independent'), ('c2_small', 65536, 'stream'), ('c2_small', 65536, 'null'),
    ('c4_small', 4096, 'independent'), ('c4_small', 4096, 'stream'),
    ('magic_heavy', 65536, 'independent'), ('magic_heavy', 65536, 'stream'), ('magic_heavy', 8192, 'stream'),
    ('runs', 65536, 'independent'), ('runs', 65536, 'stream'), ('runs', 3000, 'stream'),
    ('periodic', 65536, 'independent'), ('periodic', 65536, 'stream'),
    ('all_f1', 65536, 'independent'), ('all_f1', 65536, 'stream'),
    ('ragged', 'ragged', 'independent'), ('ragged', 'ragged', 'stream'),
]

MODES = {'independent': MODE_INDEPENDENT, 'stream': MODE_STREAM, 'null': MODE_NULL}


def main():
    ref = Oracle(ref=True)
    out = {'hash_kats': hash_kats(), 'baseline': {}, 'inputs': {}, 'cases': []}
    # Cross-check the parsed KATs against the compiled reference.
    for i, h in enumerate(out['hash_kats']):
        assert ref.hash(bytes([i]) * 2048) == int(h, 16)
    for k, v in BASELINE.items():
        out['baseline'][k] = dict(zip(('input', 'xc_len', 'xc', 'oob_len', 'oob'), v))
    for name in INPUTS:
        d = inputs(name)
        out['inputs'][name] = {'len': len(d), 'sha256': sha(d)}
    for name, chunk, mode in CASES:
        d = inputs(name)
        offs, lens = chunking(name, d, chunk)
        outs = ref.encode_batch(d, offs, lens, mode=MODES[mode], oob=(mode == 'null'))
        whole = b''.join(outs)
        case = {'input': name, 'chunk': chunk, 'mode': mode, 'nchunks': int(lens.size),
                'lens': [len(o) for o in outs], 'chunk_sha256': [sha(o)[:32] for o in outs],
                'sha256': sha(whole), 'len': len(whole)}
        if len(whole) <= 4096:
            case['hex'] = whole.hex()
        if name in BASELINE and chunk == 65536 and mode in ('stream', 'null'):
            b = BASELINE[name]
            exp = (b[1], b[2]) if mode == 'stream' else (b[3], b[4])
            if exp[0] is not None:
                assert (len(whole), sha(whole)) == exp, (name, mode)
        out['cases'].append(case)
    path = os.path.join(os.path.dirname(os.path.abspath(__file__)), 'golden.json')
    with open(path, 'w') as f:
        json.dump(out, f, indent=0, sort_keys=True)
    print('wrote', path, os.path.getsize(path), 'bytes;', len(out['cases']), 'cases')


if __name__ == '__main__':
    main()
