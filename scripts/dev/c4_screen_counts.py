"""C4's quiet-chunk screen: chunks screened vs sent to the parse (GPU box).
Usage: python3 scripts/dev/c4_screen_counts.py"""
import ctypes as C
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(__file__), '..', '..'))
sys.path.insert(0, os.path.join(os.path.dirname(__file__), '..'))
import configs_bench as cb  # noqa: E402
from wanproxy_amd.xcgpu import lib as _lib  # noqa: E402

ap = cb.argparse.ArgumentParser()
args = ap.parse_args([])
for k, v in dict(scale=1.0, reps=1, batch_mib=512, c4_batch=65536, no_decode=True, device=0).items():
    setattr(args, k, v)
lib = _lib()
lib.xcg_debug_set_screen(2)
r = cb.run_c4(args)
seen, parsed = C.c_uint64(), C.c_uint64()
lib.xcg_debug_screen_counts(C.byref(seen), C.byref(parsed))
print({'rounds': r['rounds'], 'screened': seen.value, 'parsed': parsed.value})
