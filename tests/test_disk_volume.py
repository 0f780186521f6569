"""The engine's XCodecDisk volume file on the host side (no GPU): a volume the
reference wrote (XCodecDisk over the restated disk, oracle/ref_driver.cc
RefDisk) is reopened by xcg_disk_open -- the reload of
xcodec/xcodec_cache_disk.cc:107-237 -- and saved again by xcg_disk_save before
any front binds it to a device: the file must be the reference's after the
same reopen (which writes only the registry entries of fronts it collects).  A missing path is a fresh volume; a
damaged file reopens without a crash."""
import importlib.util
import os

import pytest

HERE = os.path.dirname(os.path.abspath(__file__))
_spec = importlib.util.spec_from_file_location('make_pair_golden', os.path.join(HERE, 'golden/make_pair_golden.py'))
mpg = importlib.util.module_from_spec(_spec)
_spec.loader.exec_module(mpg)
SEG = 2048


def _uuid(k):
    return '%08x-0000-4000-8000-%012x' % (0xF11E, k)


@pytest.mark.parametrize('nb,parts,peer', [(3, 1, False), (3, 3, True), (12, 2, True)])
def test_reopen_and_save_is_the_reference_file(ref_oracle, tmp_path, nb, parts, peer):
    from oracle.lib import MODE_STREAM
    from wanproxy_amd import synth
    from wanproxy_amd.xcgpu import Disk
    limit, disk = 40 * SEG, mpg.disk_bytes(nb)
    d = synth.stream(0xF0 + 7 * nb + parts, 3 << 20, 25, 0)
    e = synth.stream(0xF1 + 7 * nb + parts, 1 << 20, 25, 0)
    offs, lens = synth.chunks_of(d, 65536)
    eo, el = synth.chunks_of(e, 65536)
    vref = str(tmp_path / 'ref.vol')
    pa = ref_oracle.cache_open_pair(limit, disk, vref, _uuid(nb))
    if peer:   # a connected peer's front registered and writing too
        pb = ref_oracle.cache_pair_front(pa, _uuid(0x100 + nb), limit)
        ref_oracle.encode_batch(e, eo, el, mode=MODE_STREAM, cache=pb)
    k = len(offs) // parts
    for i in range(parts):
        ref_oracle.encode_batch(d, offs[i * k:(i + 1) * k], lens[i * k:(i + 1) * k], mode=MODE_STREAM, cache=pa)
    ref_oracle.disk_save(pa, vref)
    # the reference reopens it (its reload writes the registry of fronts it
    # collects: registry_collect, xcodec_cache_disk.cc:496-528) and saves
    vref2 = str(tmp_path / 'ref_reopened.vol')
    pa2 = ref_oracle.cache_open_pair(limit, disk, vref, _uuid(nb))
    ref_oracle.disk_save(pa2, vref2)
    K = Disk(disk, path=vref)
    out = str(tmp_path / 'engine.vol')
    K.save(out)
    K.close()
    a, b = open(vref2, 'rb').read(), open(out, 'rb').read()
    assert len(a) == len(b) == disk
    if a != b:
        i = next(j for j in range(len(a)) if a[j] != b[j])
        pytest.fail(f'reopened volume saved differently: first byte {i} (block {i // SEG})')


def test_fresh_and_damaged_volumes(tmp_path):
    from wanproxy_amd.xcgpu import Disk
    disk = mpg.disk_bytes(3)
    # a missing path: a fresh volume (zero registry, no index block in use)
    K = Disk(disk, path=str(tmp_path / 'absent.vol'))
    K.save(str(tmp_path / 'fresh.vol'))
    K.close()
    fresh = open(tmp_path / 'fresh.vol', 'rb').read()
    assert len(fresh) == disk and fresh == bytes(disk)
    # damaged files reopen (their index entries fail the reload's checks or
    # read as empty) and save without a crash
    import numpy as np
    rng = np.random.default_rng(5)
    for name, blob in (('short', rng.integers(0, 256, disk // 3, dtype=np.uint8).tobytes()),
                       ('noise', rng.integers(0, 256, disk, dtype=np.uint8).tobytes())):
        p = tmp_path / (name + '.vol')
        p.write_bytes(blob)
        K = Disk(disk, path=str(p))
        K.save(str(tmp_path / (name + '.out')))
        K.close()
        assert os.path.getsize(tmp_path / (name + '.out')) == disk
