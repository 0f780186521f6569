"""The workload generator (BASELINE.md "Generator for kat_a/b/c"): the C build
(wanproxy_amd/csrc/xcg_synth.c), the numpy path and the verbatim pure-Python
generator agree, and any byte range equals that slice of the whole stream
(the multi-GPU shards of SURVEY.md 8e rely on it)."""
import numpy as np
import pytest

from wanproxy_amd import synth


@pytest.mark.parametrize('args', [(0x5eed, 1 << 20, 50, 0), (0xb0b, 1 << 20, 50, 2), (0xc0de, 300001, 0, 0),
                                  (0xC4, 200000, 4, 0)])
def test_generators_agree(args):
    seed, n, dup, magic = args
    want = synth.stream_ref(*args)
    assert synth.stream_range(seed, dup, magic, 0, n, use_c=False).tobytes() == want
    if synth._csynth() is None:
        pytest.skip('libxcsynth.so not built')
    assert synth.stream(*args) == want


@pytest.mark.parametrize('use_c', [True, False])
def test_ranges_are_slices(use_c):
    if use_c and synth._csynth() is None:
        pytest.skip('libxcsynth.so not built')
    full = synth.stream_range(0xC5, 20, 0, 0, 9 << 20, use_c=False).tobytes()
    for lo, hi in ((0, 1), (1, 4097), (2047, 2049), (12345, 99999), (3 << 20, 9 << 20), (5 << 20, 5 << 20)):
        assert synth.stream_range(0xC5, 20, 0, lo, hi, use_c=use_c).tobytes() == full[lo:hi]
    m = synth.stream_range(0xb0b, 50, 2, 0, 1 << 20, use_c=False)
    assert np.array_equal(synth.stream_range(0xb0b, 50, 2, 777, 1 << 20, use_c=use_c), m[777:])
