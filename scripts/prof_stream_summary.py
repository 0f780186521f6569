#!/usr/bin/env python3
"""Per-dispatch summary of encode_stream_kernel from a scripts/profile_stream.sh
run (gpurun_out/profs): duration (kernel trace) and counters (PMC passes),
grouped by configuration in launch order.  HBM bytes follow
MI355X_MICROARCH.md "HBM": FETCH_SIZE / WRITE_SIZE are KiB; FETCH_SIZE is
doubled on gfx950 (it reads half the bytes of a wide coalesced stream).

usage: prof_stream_summary.py SRC OUT.json  name=count ...   (dispatches per config, in order)
"""
import collections
import csv
import glob
import json
import sys

src, dst = sys.argv[1], sys.argv[2]
groups = [(a.split('=')[0], int(a.split('=')[1])) for a in sys.argv[3:]]
K = 'encode_stream_kernel'


def rows(sub, name):
    f = glob.glob(f'{src}/{sub}/**/{name}', recursive=True)
    return list(csv.DictReader(open(f[0]))) if f else []


trace = [r for r in rows('trace', 'run_kernel_trace.csv') if K in r['Kernel_Name']]
trace.sort(key=lambda r: int(r['Start_Timestamp']))
disp = [{'kernel': r['Kernel_Name'], 'grid': int(r['Grid_Size_X']),
         'us': (int(r['End_Timestamp']) - int(r['Start_Timestamp'])) / 1e3} for r in trace]
for sub in ('fetch', 'write', 'sq', 'sq2'):
    per = collections.OrderedDict()
    for r in rows(sub, 'run_counter_collection.csv'):
        if K in r['Kernel_Name']:
            per.setdefault(int(r['Dispatch_Id']), {})[r['Counter_Name']] = float(r['Counter_Value'])
    for i, d in enumerate(sorted(per)):
        if i < len(disp):
            disp[i].update(per[d])
out, i = {}, 0
for name, cnt in groups:
    ds = disp[i:i + cnt]
    i += cnt
    agg = {'dispatches': len(ds), 'kernel': ds[0]['kernel'] if ds else None}
    for k in set().union(*[d.keys() for d in ds]) - {'kernel'}:
        vals = [d[k] for d in ds if k in d]
        agg[k + '_sum'] = round(sum(vals), 3)
    if 'FETCH_SIZE_sum' in agg and 'WRITE_SIZE_sum' in agg:
        agg['hbm_bytes'] = int(agg['FETCH_SIZE_sum'] * 1024 * 2 + agg['WRITE_SIZE_sum'] * 1024)
        agg['hbm_GBps'] = round(agg['hbm_bytes'] / (agg['us_sum'] * 1e3), 1)
    if 'SQ_WAVE_CYCLES_sum' in agg and 'SQ_WAIT_ANY_sum' in agg:
        agg['wait_any_frac'] = round(agg['SQ_WAIT_ANY_sum'] / agg['SQ_WAVE_CYCLES_sum'], 3)
    out[name] = agg
out['dispatches_total'] = len(disp)
json.dump(out, open(dst, 'w'), indent=1)
print(json.dumps(out, indent=1))
