"""The CPU oracle is pinned against the reference before anything trusts it.

Mirrors the reference's own tests: xcodec/test/xcodec-hash1 (256 hash KATs)
and xcodec/test/xcodec-encode-decode1 (256 single-byte 512 KiB runs: encode,
reduction in size, decode, byte-equal round trip), plus the reference-produced
goldens of BASELINE.md and tests/golden/golden.json.
"""
import numpy as np
import pytest

from golden_cases import MODES, chunks, data, sha
from oracle.lib import MODE_STREAM


def test_hash_kats(golden, oracle):
    # xcodec/test/xcodec-hash1/xcodec-hash1.cc:293-314
    for i, h in enumerate(golden['hash_kats']):
        assert oracle.hash(bytes([i]) * 2048) == int(h, 16), i


def test_inputs_pinned(golden):
    for name, meta in golden['inputs'].items():
        d = data(name)
        assert len(d) == meta['len'] and sha(d) == meta['sha256'], name


def test_baseline_shas(golden, oracle):
    # BASELINE.md "KAT": reference tack -c / tack -N -c outputs.
    for name, b in golden['baseline'].items():
        d = data(name)
        assert sha(d) == b['input']
        enc = oracle.encode_stream(d)
        assert (len(enc), sha(enc)) == (b['xc_len'], b['xc']), name
        if b['oob']:
            enc = oracle.encode_stream(d, mode=2, oob=True)
            assert (len(enc), sha(enc)) == (b['oob_len'], b['oob']), name


def test_golden_cases(golden, oracle):
    for case in golden['cases']:
        d, (offs, lens) = chunks(case)
        outs = oracle.encode_batch(d, offs, lens, mode=MODES[case['mode']], oob=case['mode'] == 'null')
        assert [len(o) for o in outs] == case['lens'], (case['input'], case['chunk'], case['mode'])
        assert [sha(o)[:32] for o in outs] == case['chunk_sha256'], (case['input'], case['chunk'], case['mode'])
        if 'hex' in case:
            assert b''.join(outs).hex() == case['hex']


def test_window_hashes_closed_form(oracle):
    # Every window hash equals the non-rolling XCodecHash::hash of that window.
    rng = np.random.default_rng(5)
    x = rng.integers(0, 256, size=9000, dtype=np.uint8)
    x[1000:3500] = 0xF1
    x[4000:4100] = 0
    wh = oracle.window_hashes(x.tobytes())
    for s in list(range(0, 300)) + list(range(6500, 6953)):
        assert int(wh[s]) == oracle.hash(x[s:s + 2048].tobytes())


def test_window_hashes_vs_reference(oracle, ref_oracle):
    rng = np.random.default_rng(6)
    x = rng.integers(0, 256, size=70000, dtype=np.uint8).tobytes()
    assert np.array_equal(oracle.window_hashes(x), ref_oracle.window_hashes(x))


@pytest.mark.parametrize('ch', [0, 1, 0x7f, 0xf1, 0xff])
def test_char_run_round_trip(oracle, ch):
    # xcodec/test/xcodec-encode-decode1/xcodec-encode-decode1.cc:41-104
    run = bytes([ch]) * (2048 << 8)
    cache = oracle.cache_new()
    try:
        enc = oracle.encode_batch(run, np.array([0]), np.array([len(run)]), mode=MODE_STREAM, cache=cache)[0]
        assert len(enc) < len(run)
        assert enc[:2] == b'\xf1\x01' and len(enc) == 2050 + 255 * 10
        ok, out, consumed, unk = oracle.decode(enc, cache)
        assert ok and not unk and consumed == len(enc) and out == run
    finally:
        oracle.cache_free(cache)


def test_decode_round_trip_fresh_cache(golden, oracle, ref_oracle):
    # tack -c | tack -d with separate caches (programs/tack/tack.cc:298-359).
    for name in ('kat_a', 'kat_b', 'kat_c', 'kat_z', 'kat_col', 'magic_heavy', 'runs', 'periodic', 'all_f1'):
        d = data(name)
        enc = oracle.encode_stream(d)
        for o in (oracle, ref_oracle):
            c = o.cache_new()
            ok, out, consumed, unk = o.decode(enc, c)
            o.cache_free(c)
            assert ok and not unk and consumed == len(enc) and out == d, (name, o.ref)


def test_decode_partial_and_unknown(oracle, ref_oracle):
    d = data('kat_a')
    enc = oracle.encode_stream(d)
    # Truncated mid-EXTRACT: both stop before the op and keep it unconsumed.
    cut = enc.index(b'\xf1\x01', 5000) + 100
    res = []
    for o in (oracle, ref_oracle):
        c = o.cache_new()
        res.append(o.decode(enc[:cut], c))
        o.cache_free(c)
    assert res[0] == res[1] and res[0][2] < cut
    # Unknown REF: strip the stream's EXTRACTs' cache by decoding from the
    # middle -- the first REF to an unknown hash blocks with an ASK list.
    start = enc.index(b'\xf1\x02')
    res = []
    for o in (oracle, ref_oracle):
        c = o.cache_new()
        ok, out, consumed, unk = o.decode(enc[start:], c)
        res.append((ok, out, consumed, sorted(unk)))   # std::set<uint64_t> order
        o.cache_free(c)
    assert res[0] == res[1] and res[0][0] and res[0][3]


def test_pipe_framing_oracle(oracle):
    """oracle/pipe.py: <HELLO>, 512 KiB <FRAME>s whose payloads decode back, <EOS>."""
    from golden_cases import data
    from oracle.pipe import encoder_stream
    uuid = b'0d1f4c8e-95a3-4b2d-8f6e-3c7a9b1d2e4f'
    d = data('kat_a')
    cache = oracle.cache_new()
    try:
        wire = encoder_stream(oracle, cache, uuid, [d, b''])
    finally:
        oracle.cache_free(cache)
    assert wire[:2] == bytes([0xFF, 36]) and wire[2:38] == uuid and wire[-1:] == b'\xfc'
    i, frames = 38, []
    while wire[i] == 0x02:
        n = int.from_bytes(wire[i + 1:i + 5], 'big')
        frames.append(wire[i + 5:i + 5 + n])
        i += 5 + n
    assert i == len(wire) - 1 and len(frames) == 2
    dcache = oracle.cache_new()
    try:
        out = b''.join(oracle.decode(f, dcache)[1] for f in frames)
    finally:
        oracle.cache_free(dcache)
    assert out == d
