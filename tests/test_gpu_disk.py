"""The disk level's storage (XCodecDisk, xcodec/xcodec_cache_disk.{h,cc}):
one set of data blocks shared by every front on a disk (the reference's one
volume file), and the spill tier below HBM (the blocks in pinned host memory
behind the same device addresses).  Output parity is the pair's (the real
XCodecCachePair over the RefDisk restatement, oracle/ref_driver.cc)."""
import importlib.util
import os

import pytest

pytestmark = pytest.mark.gpu

HERE = os.path.dirname(os.path.abspath(__file__))
_spec = importlib.util.spec_from_file_location('make_pair_golden', os.path.join(HERE, 'golden/make_pair_golden.py'))
mpg = importlib.util.module_from_spec(_spec)
_spec.loader.exec_module(mpg)
SEG = 2048


def _ops(b):
    """The op list of an encoded stream: ('X', input offset) / ('R', offset, hash)."""
    i, pos, out = 0, 0, []
    while i < len(b):
        if b[i] != 0xF1:
            j = b.find(b'\xf1', i)
            j = len(b) if j < 0 else j
            pos += j - i
            i = j
            continue
        op = b[i + 1]
        if op == 0:
            i, pos = i + 2, pos + 1
        elif op == 1:
            out.append(('X', pos))
            i, pos = i + 2 + SEG, pos + SEG
        else:
            out.append(('R', pos, b[i + 2:i + 10].hex()))
            i, pos = i + 10, pos + SEG
    return out


def _first_diff(got, exp):
    for c, (a, b) in enumerate(zip(got, exp)):
        if a != b:
            oa, ob = _ops(a), _ops(b)
            j = next((t for t in range(min(len(oa), len(ob))) if oa[t] != ob[t]), min(len(oa), len(ob)))
            return f'chunk {c}: op {j}: engine {oa[j:j + 3]} reference {ob[j:j + 3]} ({len(oa)} / {len(ob)} ops)'
    return f'{len(got)} / {len(exp)} chunks'


def _uuid(k):
    return '%08x-0000-4000-8000-%012x' % (0xD15C, k)


@pytest.mark.parametrize('tier', [0, 1])
def test_shared_disk_tiers_vs_reference(ref_oracle, tier):
    """Two fronts on one disk encoding in alternation, with the blocks in HBM
    (tier 0) or spilled to pinned host memory (tier 1): every chunk and every
    front's disk counters equal the reference's local + connected pair."""
    from oracle.lib import MODE_STREAM
    from wanproxy_amd import synth
    from wanproxy_amd.xcgpu import XCG_SEM_STREAM, Context, Disk
    limit, disk = 100 * SEG, mpg.disk_bytes(2)
    da = synth.stream(0xA12 + tier, 2 << 20, 30, 0)
    db = synth.stream(0xB23 + tier, 2 << 20, 30, 0)
    oa, la = synth.chunks_of(da, 65536)
    ob, lb = synth.chunks_of(db, 65536)
    pa = ref_oracle.cache_new_pair(limit, disk)
    pb = ref_oracle.cache_connect(pa, _uuid(tier))
    exp = []
    for k in range(0, len(oa), 4):
        exp.append(ref_oracle.encode_batch(da, oa[k:k + 4], la[k:k + 4], mode=MODE_STREAM, cache=pa))
        exp.append(ref_oracle.encode_batch(db, ob[k:k + 4], lb[k:k + 4], mode=MODE_STREAM, cache=pb))
    est = [ref_oracle.pair_stats(pa, disk_live=True), ref_oracle.pair_stats(pb, disk_live=True)]
    K = Disk(disk, tier=Disk.HOST if tier else Disk.DEVICE)
    assert K.tier() == -1
    ca = Context(0, memory_cache_limit=limit, disk=K)
    cb = Context(0, memory_cache_limit=limit, disk=K)
    if tier and K.tier() != tier:
        ca.close()
        cb.close()
        K.close()
        pytest.skip('host-located virtual memory is not available in this HIP runtime (the disk stayed in HBM)')
    assert K.tier() == tier
    got = []
    for k in range(0, len(oa), 4):
        got.append(ca.encode_chunks(da, oa[k:k + 4], la[k:k + 4], semantics=XCG_SEM_STREAM))
        got.append(cb.encode_chunks(db, ob[k:k + 4], lb[k:k + 4], semantics=XCG_SEM_STREAM))
    sa, sb, ks = ca.pair_stats(), cb.pair_stats(), K.stats()
    ca.close()
    cb.close()
    K.close()
    for k, (a, b) in enumerate(zip(exp, got)):
        assert a == b, k
    assert (sa[1], sa[2], ks[0]) == est[0]
    assert (sb[1], sb[2], ks[0]) == est[1]
    assert ks[1] > 3 * 2 * 204, 'the shared disk never lapped'


def test_fronts_share_one_disk_of_hbm():
    """wanproxy.conf's 1 GiB disk with three fronts on it (the local cache and
    two connected peers): the device holds one disk's blocks, not three."""
    import torch
    from wanproxy_amd.xcgpu import XCG_SEM_STREAM, Context, Disk
    from wanproxy_amd import synth
    torch.cuda.synchronize()
    free0, _ = torch.cuda.mem_get_info(0)
    K = Disk(1 << 30, tier=Disk.DEVICE)
    ctxs = [Context(0, memory_cache_limit=128 << 20, disk=K) for _ in range(3)]
    d = synth.stream(0xD15, 1 << 20, 20, 0)
    offs, lens = synth.chunks_of(d, 65536)
    for c in ctxs:                                   # (allocates each front's tables and scratch)
        c.encode_chunks(d, offs, lens, semantics=XCG_SEM_STREAM)
    torch.cuda.synchronize()
    free1, _ = torch.cuda.mem_get_info(0)
    used = free0 - free1
    assert K.tier() == 0
    for c in ctxs:
        c.close()
    K.close()
    # one disk (1 GiB) + three primaries (128 MiB) + per-front tables and
    # scratch (~0.2 GiB each); three copies of the disk would be >= 3 GiB
    assert used < 2.2 * (1 << 30), used


def _vol_case(rng_seed, parts, chunk=65536, size=3 << 20):
    from wanproxy_amd import synth
    d = synth.stream(rng_seed, size * parts, 25, 0)
    offs, lens = synth.chunks_of(d, chunk)
    k = len(offs) // parts
    return d, [(offs[i * k:(i + 1) * k], lens[i * k:(i + 1) * k]) for i in range(parts)]


@pytest.mark.parametrize('nb', [3, 12])
def test_volume_reopen_vs_reference(ref_oracle, tmp_path, nb):
    """A process encodes on wanproxy.conf's pair over a volume file, saves it,
    a second process reopens it (a fresh memory cache over the reloaded disk:
    XCodecDisk::XCodecDisk, xcodec_cache_disk.cc:107-237) and encodes on; a
    connected peer's front finds its entries again by UUID.  Every chunk equals
    the reference's pair over the restated disk saved and reopened the same way
    (oracle/ref_driver.cc RefDisk::save / load); the reopened encoder REFs
    segments only the first process declared."""
    from oracle.lib import MODE_STREAM
    from wanproxy_amd.xcgpu import XCG_SEM_STREAM, Context, Disk
    limit, disk = 40 * SEG, mpg.disk_bytes(nb)
    local, peer = _uuid(0x100 + nb), _uuid(0x200 + nb)
    d, parts = _vol_case(0x7E1 + nb, 3)
    e, eparts = _vol_case(0x8E1 + nb, 2)
    # the reference: run 1 (local + peer), save, run 2 on the reopened volume
    vref = str(tmp_path / 'ref.vol')
    pa = ref_oracle.cache_open_pair(limit, disk, vref, local)
    pb = ref_oracle.cache_pair_front(pa, peer, limit)
    # run 1: the peer, then the local cache (whose entries are then the newest)
    exp1 = [ref_oracle.encode_batch(e, o, l, mode=MODE_STREAM, cache=pb) for o, l in eparts[:1]]
    exp1 += [ref_oracle.encode_batch(d, o, l, mode=MODE_STREAM, cache=pa) for o, l in parts[:2]]
    ref_oracle.disk_save(pa, vref)
    pa2 = ref_oracle.cache_open_pair(limit, disk, vref, _uuid(0x999))
    pb2 = ref_oracle.cache_pair_front(pa2, peer, limit)
    # run 2: the local cache sends the last part again, then the peer goes on
    exp2 = [ref_oracle.encode_batch(d, o, l, mode=MODE_STREAM, cache=pa2) for o, l in parts[1:2]]
    exp2 += [ref_oracle.encode_batch(e, o, l, mode=MODE_STREAM, cache=pb2) for o, l in eparts[1:]]
    # the engine, the same calls
    vgpu = str(tmp_path / 'gpu.vol')
    K = Disk(disk, path=vgpu)
    ca = Context(0, memory_cache_limit=limit, disk=K, uuid=local)
    cb = Context(0, memory_cache_limit=limit, disk=K, uuid=peer)
    got1 = [cb.encode_chunks(e, o, l, semantics=XCG_SEM_STREAM) for o, l in eparts[:1]]
    got1 += [ca.encode_chunks(d, o, l, semantics=XCG_SEM_STREAM) for o, l in parts[:2]]
    K.save(vgpu)
    vgpu_saved = str(tmp_path / 'gpu_saved.vol')
    K.save(vgpu_saved)
    ca.close()
    cb.close()
    K.close()
    K2 = Disk(disk, path=vgpu)
    ca2 = Context(0, memory_cache_limit=limit, disk=K2, uuid=local)
    cb2 = Context(0, memory_cache_limit=limit, disk=K2, uuid=peer)
    got2 = [ca2.encode_chunks(d, o, l, semantics=XCG_SEM_STREAM) for o, l in parts[1:2]]
    got2 += [cb2.encode_chunks(e, o, l, semantics=XCG_SEM_STREAM) for o, l in eparts[1:]]
    st = (ca2.pair_stats(), cb2.pair_stats())
    ca2.close()
    cb2.close()
    K2.close()
    assert got1 == exp1
    # the engine's saved volume is the reference's file, byte for byte
    # (registry, index blocks with their counters and entries, data blocks)
    a, b = open(vref, 'rb').read(), open(vgpu_saved, 'rb').read()
    if a != b:
        k = next(i for i in range(min(len(a), len(b))) if a[i] != b[i]) if len(a) == len(b) else -1
        pytest.fail(f'saved volumes differ: sizes {len(a)} {len(b)}, first differing byte {k} (block {k // 2048})')
    assert got2 == exp2
    # the reopened volume made a difference: without it the same calls declare more
    pf = ref_oracle.cache_new_pair(limit, disk)
    fresh = [ref_oracle.encode_batch(d, o, l, mode=MODE_STREAM, cache=pf) for o, l in parts[1:2]]
    assert sum(map(len, sum(exp2[:1], []))) < sum(map(len, sum(fresh, [])))
    # and each front's index holds what the reference's holds
    assert (st[0][1], st[1][1]) == (ref_oracle.pair_stats(pa2)[0], ref_oracle.pair_stats(pb2)[0])


def test_host_tier_in_a_process_without_torch(ref_oracle, tmp_path):
    """The spill tier where it is meant to run: a process that links
    libxcgpu.so and never loads PyTorch (wanproxy with the drop-in), whose HIP
    runtime maps pinned host memory behind device addresses.  Two fronts on a
    host-tier disk (tests/native/disk_tier_driver.c) encode in alternation;
    every chunk and the counters equal the reference's local + connected pair.
    (In this pytest process PyTorch's bundled HIP runtime is loaded, which has
    no host-located virtual memory: test_shared_disk_tiers_vs_reference skips
    its tier-1 case here.)"""
    import struct
    import subprocess
    from oracle.lib import MODE_STREAM
    from wanproxy_amd import synth
    drv = os.path.join(HERE, 'native', 'disk_tier_driver')
    if not os.path.exists(drv):
        pytest.fail('tests/native/disk_tier_driver not built (__graft_entry__.build())')
    limit, disk = 100 * SEG, mpg.disk_bytes(2)
    da = synth.stream(0xA17, 2 << 20, 30, 0)
    db = synth.stream(0xB27, 2 << 20, 30, 0)
    pa_, pb_ = tmp_path / 'a.bin', tmp_path / 'b.bin'
    pa_.write_bytes(da)
    pb_.write_bytes(db)
    outp = tmp_path / 'out.bin'
    env = {k: v for k, v in os.environ.items() if k != 'LD_LIBRARY_PATH'}
    r = subprocess.run([drv, str(pa_), str(pb_), str(outp), str(limit), str(disk), '1'], capture_output=True,
                       text=True, timeout=120, env=env)
    if r.returncode != 0 and 'host' in r.stderr.lower():
        pytest.skip('this HIP runtime maps no host memory behind device addresses: ' + r.stderr.strip())
    assert r.returncode == 0, r.stderr
    blob = outp.read_bytes()
    oa, la = synth.chunks_of(da, 65536)
    ob, lb = synth.chunks_of(db, 65536)
    pa = ref_oracle.cache_new_pair(limit, disk)
    pb = ref_oracle.cache_connect(pa, _uuid(0x7157))
    exp = []
    for k in range(0, max(len(oa), len(ob)), 4):
        if k < len(oa):
            exp += ref_oracle.encode_batch(da, oa[k:k + 4], la[k:k + 4], mode=MODE_STREAM, cache=pa)
        if k < len(ob):
            exp += ref_oracle.encode_batch(db, ob[k:k + 4], lb[k:k + 4], mode=MODE_STREAM, cache=pb)
    got, pos = [], 0
    for _ in exp:
        (n,) = struct.unpack_from('<Q', blob, pos)
        got.append(blob[pos + 8:pos + 8 + n])
        pos += 8 + n
    st = struct.unpack_from('<12Qq', blob, pos)
    assert pos + 13 * 8 == len(blob)
    tier = st[12]
    if tier != 1:
        pytest.skip(f'the disk stayed in HBM (tier {tier}): this runtime maps no host memory behind device addresses')
    for k, (a, b) in enumerate(zip(exp, got)):
        assert a == b, k
    est = [ref_oracle.pair_stats(pa, disk_live=True), ref_oracle.pair_stats(pb, disk_live=True)]
    assert (st[1], st[2], st[8]) == est[0]
    assert (st[5], st[6], st[8]) == est[1]
    assert st[9] > 3 * 2 * 204, 'the shared disk never lapped'


def test_volume_saved_after_its_fronts_are_gone(ref_oracle, tmp_path):
    """Shutdown order: the contexts close first, then the disk is saved.  The
    data blocks come from the disk's own allocation, so the volume equals the
    one saved while the fronts were open (and the reference's), and a reopen
    REFs what the first run declared."""
    from oracle.lib import MODE_STREAM
    from wanproxy_amd.xcgpu import XCG_SEM_STREAM, Context, Disk
    limit, disk = 40 * SEG, mpg.disk_bytes(4)
    local = _uuid(0x5A7E)
    d, parts = _vol_case(0x5A7, 2)
    vref = str(tmp_path / 'ref.vol')
    pa = ref_oracle.cache_open_pair(limit, disk, vref, local)
    for o, l in parts[:1]:
        ref_oracle.encode_batch(d, o, l, mode=MODE_STREAM, cache=pa)
    ref_oracle.disk_save(pa, vref)
    K = Disk(disk)
    ca = Context(0, memory_cache_limit=limit, disk=K, uuid=local)
    for o, l in parts[:1]:
        ca.encode_chunks(d, o, l, semantics=XCG_SEM_STREAM)
    open_ = str(tmp_path / 'open.vol')
    K.save(open_)
    ca.close()
    closed = str(tmp_path / 'closed.vol')
    K.save(closed)
    K.close()
    a, b, c = (open(p, 'rb').read() for p in (vref, open_, closed))
    assert b == c, 'the volume saved after the front closed lost its data blocks'
    assert a == b
    # the second run sends the first run's last 16 chunks again (the newest
    # entries, still on the disk) and goes on
    tail = (parts[0][0][-16:], parts[0][1][-16:])
    K2 = Disk(disk, path=closed)
    c2 = Context(0, memory_cache_limit=limit, disk=K2, uuid=local)
    got = [c2.encode_chunks(d, *p, semantics=XCG_SEM_STREAM) for p in (tail, parts[1])]
    c2.close()
    K2.close()
    pa2 = ref_oracle.cache_open_pair(limit, disk, vref, _uuid(0x999))
    exp = [ref_oracle.encode_batch(d, *p, mode=MODE_STREAM, cache=pa2) for p in (tail, parts[1])]
    for g, e in zip(got, exp):
        assert g == e, _first_diff(g, e)
    pf = ref_oracle.cache_new_pair(limit, disk)
    fresh = ref_oracle.encode_batch(d, *tail, mode=MODE_STREAM, cache=pf)
    assert sum(map(len, got[0])) < sum(map(len, fresh)) - 100 * 2040, 'the reopened volume REFs nothing'


def test_volume_of_a_front_without_uuid(ref_oracle, tmp_path):
    """A front made without a UUID is XCodecDisk::local: on a fresh volume it
    registers a generated local UUID at xuid 0 (registry_load,
    xcodec_cache_disk.cc:575-596), so a saved and reopened volume keeps its
    entries, and a front made without a UUID on the reopened volume is xuid 0
    again (local()) and finds them -- as the reference's local front does."""
    from oracle.lib import MODE_STREAM
    from wanproxy_amd.xcgpu import XCG_SEM_STREAM, Context, Disk
    limit, disk = 40 * SEG, mpg.disk_bytes(5)
    d, parts = _vol_case(0x10C, 2)
    vgpu = str(tmp_path / 'gpu.vol')
    K = Disk(disk)
    c = Context(0, memory_cache_limit=limit, disk=K)
    assert c.xuid() == 0
    got1 = [c.encode_chunks(d, o, l, semantics=XCG_SEM_STREAM) for o, l in parts[:1]]
    c.close()
    K.save(vgpu)
    K.close()
    reg = open(vgpu, 'rb').read(36)
    assert reg[8:9] == b'-' and reg[14:15] == b'4', reg           # a version-4 UUID string at xuid 0
    K2 = Disk(disk, path=vgpu)
    assert K2.head()[1] == 0                                       # (a reload starts an index block)
    c2 = Context(0, memory_cache_limit=limit, disk=K2)
    assert c2.xuid() == 0
    tail = (parts[0][0][-16:], parts[0][1][-16:])
    got2 = [c2.encode_chunks(d, *p, semantics=XCG_SEM_STREAM) for p in (tail, parts[1])]
    c3 = Context(0, memory_cache_limit=limit, disk=K2)              # a second unnamed front: a new xuid
    assert c3.xuid() == 1
    c3.close()
    c2.close()
    K2.close()
    # the reference: the local front under the UUID the engine generated
    vref = str(tmp_path / 'ref.vol')
    pa = ref_oracle.cache_open_pair(limit, disk, vref, reg.decode())
    exp1 = [ref_oracle.encode_batch(d, o, l, mode=MODE_STREAM, cache=pa) for o, l in parts[:1]]
    ref_oracle.disk_save(pa, vref)
    assert open(vref, 'rb').read() == open(vgpu, 'rb').read()
    pa2 = ref_oracle.cache_open_pair(limit, disk, vref, _uuid(0x998))
    exp2 = [ref_oracle.encode_batch(d, *p, mode=MODE_STREAM, cache=pa2) for p in (tail, parts[1])]
    assert got1 == exp1
    for g, e in zip(got2, exp2):
        assert g == e, _first_diff(g, e)
    assert sum(map(len, got2[0])) < sum(tail[1]) * 3 // 4, 'the local front found nothing on the reopened volume'


def test_front_by_xuid(tmp_path):
    """xcg_ctx_create_pair_xuid binds the front a host XCodecDiskCache already
    is (the drop-in's disks): that xuid, whatever order fronts bind in; a UUID
    registered at another xuid, or a held xuid, is refused."""
    from wanproxy_amd.xcgpu import XCGError, Context, Disk
    limit, disk = 40 * SEG, mpg.disk_bytes(2)
    K = Disk(disk)
    c3 = Context(0, memory_cache_limit=limit, disk=K, uuid=_uuid(3), xuid=3)
    c0 = Context(0, memory_cache_limit=limit, disk=K, xuid=0)
    assert (c3.xuid(), c0.xuid()) == (3, 0)
    with pytest.raises(XCGError):
        Context(0, memory_cache_limit=limit, disk=K, uuid=_uuid(3), xuid=4)
    with pytest.raises(XCGError):
        Context(0, memory_cache_limit=limit, disk=K, uuid=_uuid(5), xuid=3)
    c1 = Context(0, memory_cache_limit=limit, disk=K, uuid=_uuid(7))   # connect: the lowest free xuid
    assert c1.xuid() == 1
    for c in (c3, c0, c1):
        c.close()
    K.close()
