"""bench.py's launch contract (no GPU): `--gpus N` without an outer launcher
starts N ranks itself; under torchrun the launcher's WORLD_SIZE must equal
--gpus."""
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from bench import launch_plan  # noqa: E402


def test_launch_plan():
    assert launch_plan(None, {}) == ('rank', 1)
    assert launch_plan(1, {}) == ('rank', 1)
    assert launch_plan(8, {}) == ('spawn', 8)
    assert launch_plan(4, {'WORLD_SIZE': '4'}) == ('rank', 4)
    assert launch_plan(None, {'WORLD_SIZE': '2'}) == ('rank', 2)
    with pytest.raises(ValueError):
        launch_plan(8, {'WORLD_SIZE': '2'})
    with pytest.raises(ValueError):
        launch_plan(1, {'WORLD_SIZE': '8'})
    with pytest.raises(ValueError):
        launch_plan(0, {})


def test_mismatched_world_exits_nonzero():
    env = dict(os.environ, WORLD_SIZE='2', RANK='0', LOCAL_RANK='0')
    r = subprocess.run([sys.executable, os.path.join(ROOT, 'bench.py'), '--gpus', '4'], env=env,
                       capture_output=True, text=True, timeout=60)
    assert r.returncode != 0 and 'WORLD_SIZE 2' in r.stderr
