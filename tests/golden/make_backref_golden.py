#!/usr/bin/env python3
"""Regenerate tests/golden/backref.json from the REAL reference decoder.

Run in the build container only (needs oracle/_ref/libxcref.so from
`make -C oracle`).  Streams are regenerated on any machine, bit-exactly, by
tests/backref_streams.py over wanproxy_amd.synth data encoded by the C oracle
(pinned by `stream_sha256`); the JSON holds what one persistent reference
XCodecDecoder returns for each decode() call: ok, consumed, unknown count and
the SHA-256 + length of the output.
"""
from __future__ import annotations

import hashlib
import json
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.dirname(HERE))

from oracle.lib import Oracle  # noqa: E402
from wanproxy_amd import synth  # noqa: E402
from backref_streams import count_backrefs, stream_with_backrefs  # noqa: E402

CASES = [  # name, seed, dup %, nbytes, chunk, BACKREF rate, share of random indices
    ('br_64k', 11, 50, 1 << 20, 65536, 0.3, 0.0),
    ('br_4k', 12, 85, 1 << 19, 4096, 0.5, 0.0),
    ('br_bad', 13, 40, 1 << 20, 32768, 0.3, 0.08),
    ('br_dense', 14, 95, 1 << 18, 8192, 1.0, 0.0),
]


def sha(b: bytes) -> str:
    return hashlib.sha256(b).hexdigest()


def main():
    enc_oracle = Oracle()
    ref = Oracle(ref=True)
    out = {'generator': 'tests/golden/make_backref_golden.py', 'cases': []}
    for name, seed, dup, nbytes, chunk, rate, bad in CASES:
        data = synth.stream(seed, nbytes, dup, 0)
        encs = stream_with_backrefs(enc_oracle, data, chunk, seed, rate, bad)
        cache = ref.cache_new()
        dec = ref.decoder_new(cache)
        calls = []
        for e in encs:
            ok, o, cons, unk = ref.decode(e, cache, decoder=dec)
            calls.append({'ok': ok, 'consumed': cons, 'nunknown': len(unk), 'out_len': len(o), 'out_sha256': sha(o)})
            if not ok:
                break
        ref.decoder_free(dec)
        ref.cache_free(cache)
        out['cases'].append({'name': name, 'seed': seed, 'dup': dup, 'nbytes': nbytes, 'chunk': chunk,
                             'rate': rate, 'bad': bad, 'backrefs': sum(count_backrefs(e) for e in encs),
                             'stream_sha256': sha(b''.join(encs)), 'calls': calls})
        print(name, len(encs), 'calls', len(calls), 'ok' if all(c['ok'] for c in calls) else 'stops')
    with open(os.path.join(HERE, 'backref.json'), 'w') as f:
        json.dump(out, f, indent=1)


if __name__ == '__main__':
    main()
