"""Dump GPU deflate outputs for the zlib golden cases (level 6) to gpurun_out/zdump.json."""
import json, os, sys
sys.path.insert(0, os.getcwd())
from tests.zlib_cases import cases
from wanproxy_amd.zpipe import DeflatePipes
lvl = int(sys.argv[1]) if len(sys.argv) > 1 else 6
streams = [calls for level, calls in cases(7, 24) if level == lvl]
ctx = DeflatePipes(lvl, len(streams))
outs = [[] for _ in streams]
for k in range(max(len(s) for s in streams)):
    items = [(i, s[k]) for i, s in enumerate(streams) if k < len(s)]
    for (i, _), g in zip(items, ctx.consume_many(items)):
        outs[i].append(g.hex())
os.makedirs('gpurun_out', exist_ok=True)
json.dump(outs, open('gpurun_out/zdump.json', 'w'))
print('ok', len(streams))
