"""Shared helpers to rebuild golden inputs/chunkings (see tests/golden/make_golden.py)."""
import hashlib
import importlib.util
import os

HERE = os.path.dirname(os.path.abspath(__file__))
_spec = importlib.util.spec_from_file_location('make_golden', os.path.join(HERE, 'golden/make_golden.py'))
mg = importlib.util.module_from_spec(_spec)
_spec.loader.exec_module(mg)

MODES = mg.MODES
_cache = {}


def data(name):
    if name not in _cache:
        _cache[name] = mg.inputs(name)
    return _cache[name]


def chunks(case):
    d = data(case['input'])
    return d, mg.chunking(case['input'], d, case['chunk'])


def sha(b):
    return hashlib.sha256(b).hexdigest()
