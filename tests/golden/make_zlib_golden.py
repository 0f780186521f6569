#!/usr/bin/env python3
"""Regenerate tests/golden/zlib.json: outputs of the system zlib 1.2.11 (the
version wanproxy's zlib stage links in this image) driven in the reference
DeflatePipe's call pattern (zlib/deflate_pipe.cc:57-115, oracle/zlib_pipe.py),
on the deterministic cases of tests/zlib_cases.py: `streams` (levels 4-9,
deflate_slow), `fast` (levels 1-3, deflate_fast) and `stops` (incompressible
consumes sized so that a block flush falls in the Z_SYNC_FLUSH call's last
MIN_LOOKAHEAD positions: the pipe's 64 KiB buffer fills there, the consume
ends and the remaining positions wait for the next one) and `stored` (level 0,
deflate_stored: block sizes follow the 2048-byte Buffer segments and the
pipe's buffer).  Per call: input
length, output length, SHA-256 of the output, and the output hex for short
ones."""
import hashlib
import json
import os
import sys
import zlib

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(os.path.dirname(HERE)))
sys.path.insert(0, os.path.dirname(HERE))

from oracle.zlib_pipe import DeflatePipeRef, ZLIB_VERSION  # noqa: E402
from zlib_cases import cases, fast_cases, stop_cases, stored_cases  # noqa: E402


def main():
    assert zlib.ZLIB_RUNTIME_VERSION == ZLIB_VERSION, zlib.ZLIB_RUNTIME_VERSION
    out = {'zlib': zlib.ZLIB_RUNTIME_VERSION,
           'generator': 'tests/zlib_cases.py cases(seed=7, n=24), fast_cases(seed=8, n=12), stop_cases(seed=9), '
                        'stored_cases(seed=10, n=10)'}
    for key, streams in (('streams', cases(7, 24)), ('fast', fast_cases(8, 12)), ('stops', stop_cases(9)),
                         ('stored', stored_cases(10, 10))):
        out[key] = []
        for level, calls in streams:
            ref = DeflatePipeRef(level)
            rec = {'level': level, 'calls': []}
            for c in calls:
                o = ref.consume(c)
                e = {'in_len': len(c), 'in_sha256': hashlib.sha256(c).hexdigest(), 'out_len': len(o),
                     'out_sha256': hashlib.sha256(o).hexdigest()}
                if len(o) <= 64:
                    e['out_hex'] = o.hex()
                rec['calls'].append(e)
            out[key].append(rec)
    with open(os.path.join(HERE, 'zlib.json'), 'w') as f:
        json.dump(out, f, indent=1)


if __name__ == '__main__':
    main()
