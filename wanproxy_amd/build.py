"""Build libxcgpu.so in-tree for gfx950 (hipcc; no JIT cache, so the .so
travels with the repository snapshot to the GPU box)."""
from __future__ import annotations

import os
import subprocess

HERE = os.path.dirname(os.path.abspath(__file__))
SRCS = ['csrc/xcg_api.hip', 'csrc/xcg_encode.hip', 'csrc/xcg_decode.hip', 'csrc/xcg_hash.hip', 'csrc/xcg_lru.hip',
        'csrc/xcg_pipe.cpp']
OUT = os.path.join(HERE, 'libxcgpu.so')
HIPCC = os.environ.get('HIPCC', '/opt/rocm/bin/hipcc')


def build_lib(force: bool = False, verbose: bool = False, out: str = OUT, defines=()) -> str:
    """Build the library (or, for diagnostics, a variant at `out` with extra
    -D `defines`, e.g. XCG_TIMING: per-wave timestamps in the stats words)."""
    out = os.path.abspath(out)
    srcs = [os.path.join(HERE, s) for s in SRCS]
    deps = srcs + [os.path.join(HERE, 'csrc/xcg_device.h'), os.path.join(HERE, 'csrc/xcg_cache.h'),
            os.path.join(HERE, 'csrc/xcg_args.h'), os.path.join(HERE, '..', 'include', 'xcgpu.h')]
    if not force and os.path.exists(out) and all(os.path.getmtime(out) >= os.path.getmtime(d) for d in deps):
        return out
    cmd = [HIPCC, '--offload-arch=gfx950', '-O3', '-std=c++17', '-shared', '-fPIC', '-Wall',
           '-o', out + '.tmp'] + ['-D' + d for d in defines] + srcs
    if verbose:
        print(' '.join(cmd))
    subprocess.run(cmd, check=True, cwd=HERE)
    os.replace(out + '.tmp', out)
    return out


if __name__ == '__main__':
    print(build_lib(force=True, verbose=True))
