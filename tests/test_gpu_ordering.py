"""Calls of one context on different HIP streams are serialised as the
reference's calls on one cache are (one event thread): the context records
its completion marker behind its last call only when another stream or a host
wait needs it (xcg_api.hip ctx_flush_mark / ctx_order).  A second batch issued
on another stream right behind the first must see every segment the first one
committed, and a cache clear between repetitions orders against both.  (The
stream encode's own host waits -- on its verification flags -- already order
much of this, so the test guards the results, not the marker alone.)"""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def _dev_batch(dev, data, offs, lens):
    import torch
    bounds = 2 * lens.astype(np.uint64) + 16
    oo = np.zeros(len(offs), np.uint64)
    oo[1:] = np.cumsum(bounds)[:-1]
    return dict(
        d_in=torch.from_numpy(np.frombuffer(data, np.uint8).copy()).to(dev),
        d_off=torch.from_numpy((offs - offs[0]).astype(np.uint64).view(np.int64)).to(dev),
        d_len=torch.from_numpy(lens.astype(np.uint32).view(np.int32)).to(dev),
        d_oo=torch.from_numpy(oo.view(np.int64)).to(dev),
        d_out=torch.zeros(int(bounds.sum()), dtype=torch.uint8, device=dev),
        d_ol=torch.zeros(len(offs), dtype=torch.int64, device=dev), oo=oo, n=len(offs))


def _outs(b):
    ol = b['d_ol'].cpu().numpy()
    out = b['d_out'].cpu().numpy()
    return [out[int(o):int(o) + int(k)].tobytes() for o, k in zip(b['oo'], ol)]


@pytest.mark.parametrize('split', [8, 40])
def test_batches_on_two_streams_are_ordered(oracle, split):
    import torch
    from oracle.lib import MODE_STREAM
    from wanproxy_amd import synth
    from wanproxy_amd.xcgpu import XCG_SEM_STREAM, Context
    dev = torch.device('cuda', 0)
    d = synth.stream(0x0D + split, 64 * 65536, 50, 0)
    offs, lens = synth.chunks_of(d, 65536)
    exp = oracle.encode_batch(d, offs, lens, mode=MODE_STREAM)
    a = _dev_batch(dev, d[:split * 65536], offs[:split], lens[:split])
    b = _dev_batch(dev, d[split * 65536:], offs[split:], lens[split:])
    torch.cuda.synchronize()
    ctx = Context(0, cache_segments=1 << 14)
    s1, s2 = torch.cuda.Stream(dev), torch.cuda.Stream(dev)
    for rep in range(2):
        if rep:
            ctx.cache_clear()
        ctx.encode_batch_device(a['d_in'], a['d_off'], a['d_len'], a['n'], 65536, a['d_out'], a['d_oo'], a['d_ol'],
                                stream=s1, semantics=XCG_SEM_STREAM)
        ctx.encode_batch_device(b['d_in'], b['d_off'], b['d_len'], b['n'], 65536, b['d_out'], b['d_oo'], b['d_ol'],
                                stream=s2, semantics=XCG_SEM_STREAM)
        torch.cuda.synchronize()
        got = _outs(a) + _outs(b)
        bad = [i for i in range(len(exp)) if got[i] != exp[i]]
        assert not bad, (rep, bad[:8])
    # the second batch really referenced the first one's segments
    assert sum(e.count(b'\xf1\x02') for e in exp[split:]) > 0
    ctx.close()
