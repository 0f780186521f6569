"""Build libxcgpu.so in-tree for gfx950 (hipcc; no JIT cache, so the .so
travels with the repository snapshot to the GPU box).

Each source compiles to its own object in parallel (objects are reused while
they are newer than the source and every header), then one link."""
from __future__ import annotations

import os
import subprocess
from concurrent.futures import ThreadPoolExecutor

HERE = os.path.dirname(os.path.abspath(__file__))
SRCS = ['csrc/xcg_api.hip', 'csrc/xcg_encode.hip', 'csrc/xcg_decode.hip', 'csrc/xcg_hash.hip', 'csrc/xcg_lru.hip',
        'csrc/xcg_pair.hip', 'csrc/xcg_pipe.cpp', 'csrc/xcg_deflate.hip', 'csrc/xcg_inflate.hip']
HDRS = ['csrc/xcg_device.h', 'csrc/xcg_cache.h', 'csrc/xcg_args.h', '../include/xcgpu.h']
OUT = os.path.join(HERE, 'libxcgpu.so')
HIPCC = os.environ.get('HIPCC', '/opt/rocm/bin/hipcc')
FLAGS = ['--offload-arch=gfx950', '-O3', '-std=c++17', '-fPIC', '-Wall'] + os.environ.get('XCG_EXTRA_FLAGS', '').split()


def _newer(out: str, deps) -> bool:
    return os.path.exists(out) and all(os.path.getmtime(out) >= os.path.getmtime(d) for d in deps)


def build_lib(force: bool = False, verbose: bool = False, out: str = OUT, defines=()) -> str:
    """Build the library (or, for diagnostics, a variant at `out` with extra
    -D `defines`, e.g. XCG_TIMING: per-wave timestamps in the stats words)."""
    out = os.path.abspath(out)
    srcs = [os.path.join(HERE, s) for s in SRCS]
    hdrs = [os.path.join(HERE, h) for h in HDRS]
    if not force and _newer(out, srcs + hdrs):
        return out
    tag = '' if not defines else '.' + '_'.join(defines)
    objdir = os.path.join(HERE, 'build')
    os.makedirs(objdir, exist_ok=True)
    dflags = ['-D' + d for d in defines]

    def compile_one(src):
        obj = os.path.join(objdir, os.path.basename(src) + tag + '.o')
        if not force and _newer(obj, [src] + hdrs):
            return obj
        cmd = [HIPCC] + FLAGS + dflags + ['-c', '-o', obj + '.tmp', src]
        if verbose:
            print(' '.join(cmd))
        subprocess.run(cmd, check=True, cwd=HERE)
        os.replace(obj + '.tmp', obj)
        return obj

    with ThreadPoolExecutor(min(len(srcs), os.cpu_count() or 1)) as ex:
        objs = list(ex.map(compile_one, srcs))
    cmd = [HIPCC, '--offload-arch=gfx950', '-shared', '-fPIC', '-o', out + '.tmp'] + objs
    if verbose:
        print(' '.join(cmd))
    subprocess.run(cmd, check=True, cwd=HERE)
    os.replace(out + '.tmp', out)
    return out


SYNTH_SRC = os.path.join(HERE, 'csrc/xcg_synth.c')
SYNTH_OUT = os.path.join(HERE, 'libxcsynth.so')


def build_synth(force: bool = False) -> str:
    """The workload generator (csrc/xcg_synth.c: bench / test inputs, no GPU)."""
    if force or not _newer(SYNTH_OUT, [SYNTH_SRC]):
        subprocess.run(['gcc', '-O2', '-shared', '-fPIC', '-o', SYNTH_OUT + '.tmp', SYNTH_SRC], check=True)
        os.replace(SYNTH_OUT + '.tmp', SYNTH_OUT)
    return SYNTH_OUT


NATIVE_SRC = os.path.join(HERE, '..', 'tests', 'native', 'disk_tier_driver.c')
NATIVE_OUT = os.path.join(HERE, '..', 'tests', 'native', 'disk_tier_driver')


def build_native_tests(force: bool = False) -> str:
    """C drivers of the ABI that GPU tests run in processes without PyTorch
    (tests/native: test infrastructure, linked against the in-tree library)."""
    if force or not _newer(NATIVE_OUT, [NATIVE_SRC, OUT]):
        subprocess.run(['gcc', '-O2', '-Wall', '-o', NATIVE_OUT + '.tmp', NATIVE_SRC, '-L' + HERE, '-l:libxcgpu.so',
                        '-Wl,-rpath,$ORIGIN/../../wanproxy_amd'], check=True)
        os.replace(NATIVE_OUT + '.tmp', NATIVE_OUT)
    return NATIVE_OUT


if __name__ == '__main__':
    print(build_lib(force=True, verbose=True))
    print(build_synth(force=True))
