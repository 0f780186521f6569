import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)


def pytest_configure(config):
    config.addinivalue_line('markers', 'gpu: needs an MI355X (run on the GPU box)')
    config.addinivalue_line('markers', 'slow: long-running CPU test')


@pytest.fixture(scope='session', autouse=True)
def _built():
    """Make sure the oracle libraries exist (cheap no-op when up to date)."""
    from oracle import lib
    if not os.path.exists(os.path.join(ROOT, 'oracle/build/liboracle.so')):
        lib.build()


@pytest.fixture(scope='session')
def golden():
    import json
    with open(os.path.join(ROOT, 'tests/golden/golden.json')) as f:
        return json.load(f)


@pytest.fixture(scope='session')
def oracle():
    from oracle.lib import Oracle
    return Oracle()


@pytest.fixture(params=[0, 1], ids=['round0', 'seeded'])
def stream_seed(request):
    """Both ways the stream encoder starts its rounds (xcg_debug_set_stream_seed):
    a parse round against the cache alone, or the chunks' tiling seed."""
    from wanproxy_amd.xcgpu import lib
    old = lib().xcg_debug_set_stream_seed(request.param)
    yield request.param
    lib().xcg_debug_set_stream_seed(old)


@pytest.fixture(scope='session')
def ref_oracle():
    from oracle.lib import Oracle
    p = os.path.join(ROOT, 'oracle/_ref/libxcref.so')
    if not os.path.exists(p):
        pytest.skip('oracle/_ref/libxcref.so not built (needs /root/reference)')
    return Oracle(ref=True)
