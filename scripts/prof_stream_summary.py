#!/usr/bin/env python3
"""Summarise a scripts/profile_stream.sh run (gpurun_out/profs: one directory
per configuration) for profiles/: per configuration, every kernel's launches,
time (kernel trace) and counters (PMC passes, matched by dispatch id), the
kernels sorted by total time.  HBM bytes follow MI355X_MICROARCH.md "HBM":
FETCH_SIZE / WRITE_SIZE are KiB and FETCH_SIZE is doubled on gfx950 (it reads
half the bytes of a wide coalesced stream).  For c2s the stream-parse
launches are also listed one by one; `c2s_seeded` is the last of them (the
seeded parse the bench times).

usage: prof_stream_summary.py SRC OUT.json
"""
import collections
import csv
import glob
import json
import os
import sys

src, dst = sys.argv[1], sys.argv[2]
K = 'encode_stream_kernel'


def rows(d, sub, name):
    f = glob.glob(f'{d}/{sub}/**/{name}', recursive=True)
    return list(csv.DictReader(open(f[0]))) if f else []


def short(name):
    return name.split('(')[0].replace('void ', '').strip() or name[:80]


def hbm(agg):
    if 'FETCH_SIZE' in agg and 'WRITE_SIZE' in agg:
        agg['hbm_bytes'] = int(agg['FETCH_SIZE'] * 1024 * 2 + agg['WRITE_SIZE'] * 1024)
        if agg.get('us'):
            agg['hbm_GBps'] = round(agg['hbm_bytes'] / (agg['us'] * 1e3), 1)
    if 'SQ_WAVE_CYCLES' in agg and 'SQ_WAIT_ANY' in agg and agg['SQ_WAVE_CYCLES']:
        agg['wait_any_frac'] = round(agg['SQ_WAIT_ANY'] / agg['SQ_WAVE_CYCLES'], 3)
    # L2 hit rate (MI355X_MICROARCH.md "L2 per XCD": hit / (hit + miss))
    h, m = agg.get('TCC_HIT_sum'), agg.get('TCC_MISS_sum')
    if h is not None and m is not None and h + m:
        agg['l2_hit_rate'] = round(h / (h + m), 3)
        if agg.get('us'):
            agg['l2_req_G_per_s'] = round((h + m) / (agg['us'] * 1e3), 1)
    return agg


out = {}
for d in sorted(glob.glob(os.path.join(src, '*', ''))):
    cfg = os.path.basename(os.path.dirname(d))
    trace = sorted(rows(d, 'trace', 'run_kernel_trace.csv'), key=lambda r: int(r['Start_Timestamp']))
    if not trace:
        continue
    disp = [{'kernel': short(r['Kernel_Name']), 'grid': int(r['Grid_Size_X']),
             'us': (int(r['End_Timestamp']) - int(r['Start_Timestamp'])) / 1e3} for r in trace]
    # counters per dispatch, matched to the trace in launch order per kernel
    for sub in ('fetch', 'write', 'sq', 'sq2', 'l2', 'tcp'):
        per = collections.OrderedDict()
        for r in rows(d, sub, 'run_counter_collection.csv'):
            per.setdefault(int(r['Dispatch_Id']), [short(r['Kernel_Name']), {}])[1][r['Counter_Name']] = \
                float(r['Counter_Value'])
        byk = collections.defaultdict(list)
        for did in sorted(per):
            byk[per[did][0]].append(per[did][1])
        seen = collections.Counter()
        for x in disp:
            lst = byk.get(x['kernel'], [])
            i = seen[x['kernel']]
            seen[x['kernel']] += 1
            if i < len(lst):
                x.update(lst[i])
    kern = collections.OrderedDict()
    for x in disp:
        a = kern.setdefault(x['kernel'], {'launches': 0})
        a['launches'] += 1
        for k, v in x.items():
            if k not in ('kernel', 'grid'):
                a[k] = a.get(k, 0) + v
    for a in kern.values():
        a['us'] = round(a['us'], 2)
        a['avg_us'] = round(a['us'] / a['launches'], 2)
        hbm(a)
        if 'hbm_bytes' in a:
            a['hbm_bytes_per_launch'] = a['hbm_bytes'] // a['launches']
    total = sum(a['us'] for a in kern.values())
    out[cfg] = {'kernel_us_total': round(total, 1),
                'kernels': dict(sorted(kern.items(), key=lambda kv: -kv[1]['us']))}
    if cfg == 'c2s':
        sp = [hbm(dict(x)) for x in disp if K in x['kernel']]
        out[cfg]['stream_launches'] = sp
        if sp and 'hbm_bytes' in sp[-1]:
            out['c2s_seeded'] = {'dispatches': 1, 'us_sum': sp[-1]['us'], 'hbm_bytes': sp[-1]['hbm_bytes'],
                                 'hbm_GBps': sp[-1].get('hbm_GBps'), 'wait_any_frac': sp[-1].get('wait_any_frac')}
    if cfg != 'c2s':
        # every stream-parse launch of the configuration, one by one
        out[cfg]['stream_launches'] = [hbm(dict(x)) for x in disp if K in x['kernel']]
json.dump(out, open(dst, 'w'), indent=1)
print(json.dumps({c: {'total_us': v['kernel_us_total'], 'top': list(v['kernels'])[:6]} for c, v in out.items()
                  if 'kernels' in v}, indent=1))
