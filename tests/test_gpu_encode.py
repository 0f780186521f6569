"""GPU parity: libxcgpu.so vs the oracle / reference goldens (run on MI355X).

Mirrors xcodec/test/xcodec-hash1 (hash KATs) and the reference's encode path
over the golden cases of tests/golden/golden.json (independent-chunk mode:
one fresh XCodecMemoryCache per encode() call)."""
import numpy as np
import pytest

from golden_cases import chunks, data, sha

pytestmark = pytest.mark.gpu


@pytest.fixture(scope='module')
def ctx():
    from wanproxy_amd.xcgpu import Context
    c = Context(0)
    yield c
    c.close()


@pytest.fixture(scope='module')
def ctx_null():
    from wanproxy_amd.xcgpu import Context
    c = Context(0, out_of_band=True, null_cache=True)
    yield c
    c.close()


def test_window_hash_kats(ctx, golden):
    # xcodec/test/xcodec-hash1/xcodec-hash1.cc:293-314 via the window kernel
    buf = b''.join(bytes([i]) * 2048 for i in range(256))
    wh = ctx.window_hashes(buf)
    for i, h in enumerate(golden['hash_kats']):
        assert int(wh[2048 * i]) == int(h, 16), i
    seg = ctx.segment_hashes_be(buf)
    for i, h in enumerate(golden['hash_kats']):
        assert seg[8 * i:8 * i + 8] == bytes.fromhex(h), i


@pytest.mark.parametrize('name', ['kat_a', 'kat_c', 'kat_col', 'magic_heavy', 'runs', 'all_f1'])
def test_window_hashes_every_offset(ctx, oracle, name):
    d = data(name)[:300000]
    assert np.array_equal(ctx.window_hashes(d), oracle.window_hashes(d))


def test_window_hashes_unaligned(ctx, oracle):
    rng = np.random.default_rng(3)
    d = rng.integers(0, 256, size=20000, dtype=np.uint8).tobytes()
    for cut in (1, 7, 15, 4097):
        assert np.array_equal(ctx.window_hashes(d[cut:]), oracle.window_hashes(d[cut:]))


def test_golden_independent(ctx, golden):
    n = 0
    for case in golden['cases']:
        if case['mode'] != 'independent':
            continue
        d, (offs, lens) = chunks(case)
        outs = ctx.encode_chunks(d, offs, lens)
        assert [len(o) for o in outs] == case['lens'], (case['input'], case['chunk'])
        assert [sha(o)[:32] for o in outs] == case['chunk_sha256'], (case['input'], case['chunk'])
        n += 1
    assert n >= 10


def test_golden_null_cache(ctx_null, golden):
    for case in golden['cases']:
        if case['mode'] != 'null':
            continue
        d, (offs, lens) = chunks(case)
        outs = ctx_null.encode_chunks(d, offs, lens)
        whole = b''.join(outs)
        assert (len(whole), sha(whole)) == (case['len'], case['sha256']), case['input']


def test_random_vs_oracle(ctx, oracle):
    # Fuzz: many chunk shapes and contents; oracle = CPU restatement pinned above.
    rng = np.random.default_rng(2024)
    parts, lens = [], []
    for i in range(300):
        kind = i % 6
        L = int(rng.choice([0, 1, 100, 2047, 2048, 2049, 3000, 4096, 6000, 16384, 65536, 65535, 70000, 131072]))
        if kind == 0:
            b = rng.integers(0, 256, size=L, dtype=np.uint8)
        elif kind == 1:   # repeated 2 KiB blocks at random offsets
            blk = rng.integers(0, 256, size=2048 + 37, dtype=np.uint8)
            b = np.resize(blk, L)
        elif kind == 2:   # small alphabet (many equal windows / collisions)
            b = rng.integers(0, 3, size=L, dtype=np.uint8) * 0x50
        elif kind == 3:   # magic heavy
            b = np.where(rng.random(L) < 0.3, 0xF1, rng.integers(0, 256, size=L)).astype(np.uint8)
        elif kind == 4:   # runs
            b = np.repeat(rng.integers(0, 256, size=max(1, L // 500 + 1)).astype(np.uint8), 500)[:L]
        else:             # duplicated random blocks, unaligned copies
            src = rng.integers(0, 256, size=6000, dtype=np.uint8)
            b = np.concatenate([src[rng.integers(0, 3000):][:3000] for _ in range(L // 3000 + 1)])[:L]
        parts.append(b.astype(np.uint8))
        lens.append(L)
    # pack with odd padding so chunk starts are unaligned
    offs, blob, pos = [], [], 0
    for b in parts:
        pad = int(rng.integers(0, 17))
        blob.append(np.zeros(pad, np.uint8)); pos += pad
        offs.append(pos); blob.append(b); pos += b.size
    allb = np.concatenate(blob)
    offs = np.array(offs, dtype=np.uint64)
    lens = np.array(lens, dtype=np.uint32)
    got = ctx.encode_chunks(allb, offs, lens)
    exp = oracle.encode_batch(allb, offs, lens, mode=0)
    bad = [i for i in range(len(got)) if got[i] != exp[i]]
    assert not bad, (bad[:10], [len(got[i]) for i in bad[:5]], [len(exp[i]) for i in bad[:5]])


def test_stats_and_roundtrip(ctx, oracle):
    d = data('c2_small')
    from wanproxy_amd.synth import chunks_of
    offs, lens = chunks_of(d, 65536)
    outs, st = ctx.encode_chunks(d, offs, lens, with_stats=True)
    assert st[:, 0].sum() > 0
    for i in range(0, len(outs), 7):
        c = oracle.cache_new()
        ok, dec, consumed, unk = oracle.decode(outs[i], c)
        oracle.cache_free(c)
        assert ok and not unk and dec == d[int(offs[i]):int(offs[i] + lens[i])]


def test_overlong_chunk_is_refused():
    """A chunk longer than the launch's max_chunk_len is refused loudly (the
    records sized for the bound would overflow), not encoded wrongly."""
    import torch
    from wanproxy_amd.xcgpu import XCG_SEM_INDEPENDENT, XCG_SEM_STREAM, Context, XCGError
    dev = torch.device('cuda', 0)
    n, L = 2, 200000
    d_in = torch.randint(0, 256, (n * L,), dtype=torch.uint8, device=dev)
    d_off = torch.tensor([0, L], dtype=torch.int64, device=dev)
    d_len = torch.tensor([L, 1000], dtype=torch.int32, device=dev)
    d_oo = torch.tensor([0, 2 * L + 16], dtype=torch.int64, device=dev)
    d_out = torch.zeros(4 * L + 64, dtype=torch.uint8, device=dev)
    d_ol = torch.zeros(n, dtype=torch.int64, device=dev)
    for sem in (XCG_SEM_INDEPENDENT, XCG_SEM_STREAM):
        ctx = Context(0, cache_segments=1 << 12)
        ctx.encode_batch_device(d_in, d_off, d_len, n, 65536, d_out, d_oo, d_ol, semantics=sem)
        with pytest.raises(XCGError):
            ctx.status()
        ctx.close()


def test_independent_fuzz(oracle):
    # Random chunk lengths up to 512 KiB (both kernel variants), in-band,
    # out-of-band and null-cache declarations, three data shapes.
    from wanproxy_amd import synth
    from wanproxy_amd.xcgpu import Context
    rng = np.random.default_rng(4242)
    for case in range(9):
        nbytes = int(rng.integers(1 << 19, 4 << 20))
        kind = case % 3
        if kind == 0:
            d = synth.stream(int(rng.integers(1 << 30)), nbytes, int(rng.integers(0, 95)), int(rng.integers(0, 5)))
        elif kind == 1:
            pat = rng.integers(0, 256, int(rng.integers(1, 5000)), dtype=np.uint8).tobytes()
            d = (pat * (nbytes // len(pat) + 1))[:nbytes]
        else:
            d = bytes(rng.choice([0, 0xF1, 9], size=nbytes, p=[0.4, 0.4, 0.2]).astype(np.uint8))
        lens, tot = [], 0
        big = case >= 6
        while tot < nbytes:
            n = int(rng.integers(0, 524288 if big else 131072))
            n = min(n, nbytes - tot)
            lens.append(n)
            tot += n
        lens = np.array(lens, np.uint32)
        offs = np.zeros(lens.size, np.uint64)
        offs[1:] = np.cumsum(lens.astype(np.uint64))[:-1]
        mode = case % 3                   # 0 in-band, 1 out-of-band, 2 null cache
        ctx = Context(0, out_of_band=mode != 0, null_cache=mode == 2)   # (TackNullCache is out-of-band)
        got = ctx.encode_chunks(d, offs, lens)
        ctx.close()
        exp = oracle.encode_batch(d, offs, lens, mode=2 if mode == 2 else 0, oob=mode != 0)
        bad = [k for k in range(len(exp)) if got[k] != exp[k]]
        assert not bad, (case, kind, mode, bad[:5])


def _dm_key(block):
    """The independent kernel's direct-mapped probe key of a 2048-byte window:
    -(X2 + CLO) mod 2^32, X2 = sum (2048 - k) x_k (roll_probe_dm, xcg_encode.hip)."""
    w = np.arange(2048, 0, -1, dtype=np.uint64)
    x2 = int((w * block.astype(np.uint64)).sum()) & 0xFFFFFFFF
    return (-(x2 + 0x80200400)) & 0xFFFFFFFF


def _block_in_slot(rng, slot):
    """A random 2 KiB block whose key lands in direct-mapped slot `slot`
    (bits 2..12 of the key): bytes 2016 and 2047 (weights 32 and 1) absorb
    the difference."""
    b = rng.integers(0, 256, 2048, dtype=np.uint8)
    b[2016] = 0
    b[2047] = 0
    r = (_dm_key(b) - 4 * slot) % 8192          # raising X2 by r lowers the key by r
    b[2016] = r >> 5
    b[2047] = r & 31
    assert (_dm_key(b) >> 2) & 2047 == slot
    return b


@pytest.mark.parametrize('ncoll', [2, 5, 9, 30])
def test_direct_mapped_slot_collisions(ctx, oracle, ncoll):
    """Chunks whose declarations share direct-mapped key slots (1 slot + up
    to 32 overflow keys per chunk: the N1 / N8 / N32 compare variants), then
    repeat those blocks -- aligned, unaligned and cut -- so the REFs must be
    found through the overflow keys."""
    rng = np.random.default_rng(0xD1 + ncoll)
    chunks_, lens = [], []
    for c in range(6):
        slot = int(rng.integers(0, 2048))
        coll = [_block_in_slot(rng, slot) for _ in range(ncoll)]
        fresh = [rng.integers(0, 256, 2048, dtype=np.uint8) for _ in range(max(0, 40 - ncoll))]
        blocks = coll + fresh
        parts = list(blocks)
        for k in range(22):   # repeats of colliding and fresh blocks, some shifted by a few bytes
            src = blocks[int(rng.integers(0, len(blocks)))] if k % 2 else coll[int(rng.integers(0, ncoll))]
            if k % 3 == 2:
                parts.append(rng.integers(0, 256, int(rng.integers(1, 40)), dtype=np.uint8))
            parts.append(src)
        b = np.concatenate(parts)[:131072 - int(rng.integers(0, 3000)) * (c % 2)]
        chunks_.append(b)
        lens.append(b.size)
    offs = np.zeros(len(lens), np.uint64)
    offs[1:] = np.cumsum(np.array(lens, np.uint64))[:-1]
    allb = np.concatenate(chunks_)
    lens = np.array(lens, np.uint32)
    got = ctx.encode_chunks(allb, offs, lens)
    ctx.status()
    exp = oracle.encode_batch(allb, offs, lens, mode=0)
    bad = [i for i in range(len(got)) if got[i] != exp[i]]
    assert not bad, bad
    # the repeats really were found (REFs in the oracle's output)
    assert sum(e.count(b'\xf1\x02') for e in exp) >= 6 * 10
