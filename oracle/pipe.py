"""Restatement of XCodecPipePair's encoder framing.  TEST INFRASTRUCTURE ONLY.

XCodecPipePair::encoder_consume (xcodec/xcodec_pipe_pair.cc:549-642): the first
call emits <HELLO> 0xFF len uuid (:557-573); a non-empty buffer is cut into
pieces of XCODEC_PIPE_MAX_FRAME / 2 = 512 KiB (:585-600), each one
XCodecEncoder::encode() call on the codec's cache, framed as <FRAME> 0x02
BE32(len) data (:620-628); an empty buffer emits <EOS> 0xFC (:632-636).  The
frame payloads come from the oracle encoder (oracle.lib), itself pinned to the
reference; the framing bytes are these few lines.  The reference pipe pair
itself is not built here: its <HELLO> needs libuuid's header.
"""
from __future__ import annotations

import numpy as np

MAX_FRAME = 1024 * 1024


def encoder_stream(oracle, cache, uuid: bytes, consumes) -> bytes:
    out = bytearray()
    for k, buf in enumerate(consumes):
        if k == 0:
            out += bytes([0xFF, len(uuid)]) + uuid
        if not buf:
            out += b'\xfc'
            continue
        for a in range(0, len(buf), MAX_FRAME // 2):
            piece = buf[a:a + MAX_FRAME // 2]
            enc = oracle.encode_batch(piece, np.array([0], np.uint64), np.array([len(piece)], np.uint32),
                                      mode=1, cache=cache)[0]
            out += b'\x02' + len(enc).to_bytes(4, 'big') + enc
    return bytes(out)
