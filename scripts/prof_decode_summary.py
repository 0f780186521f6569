#!/usr/bin/env python3
"""Summarise scripts/profile_decode.sh (gpurun_out/profd) for profiles/: every
kernel of the decode calls (launches, time from the kernel trace, HBM bytes
from FETCH_SIZE x 2 + WRITE_SIZE in KiB, MI355X_MICROARCH.md "HBM"), and the
decode step per call (`decode_step`: the decode kernels' time and HBM bytes
divided by the number of calls).  The stream encode that made the input runs
first and is excluded by kernel name.

usage: prof_decode_summary.py SRC OUT.json [CALLS]"""
import collections
import csv
import glob
import json
import sys

src, dst = sys.argv[1], sys.argv[2]
calls = int(sys.argv[3]) if len(sys.argv) > 3 else 5
DECODE = ('decode_kernel', 'decode_refcheck_kernel', 'dec_precheck_kernel', 'decode_tend_kernel', 'decl_record_kernel',
          'window_update_kernel', 'decode_commit_kernel', 'exclusive_scan_kernel')


def rows(sub, name):
    f = glob.glob(f'{src}/{sub}/**/{name}', recursive=True)
    return list(csv.DictReader(open(f[0]))) if f else []


def short(n):
    return n.split('(')[0].replace('void ', '').strip()


def is_dec(k):
    return any(d in k for d in DECODE)


kern = collections.OrderedDict()
for r in rows('trace', 'run_kernel_trace.csv'):
    k = short(r['Kernel_Name'])
    a = kern.setdefault(k, {'launches': 0, 'us': 0.0})
    a['launches'] += 1
    a['us'] += (int(r['End_Timestamp']) - int(r['Start_Timestamp'])) / 1e3
for sub in ('fetch', 'write', 'l2'):
    for r in rows(sub, 'run_counter_collection.csv'):
        a = kern.setdefault(short(r['Kernel_Name']), {'launches': 0, 'us': 0.0})
        a[r['Counter_Name']] = a.get(r['Counter_Name'], 0.0) + float(r['Counter_Value'])
for a in kern.values():
    if 'FETCH_SIZE' in a and 'WRITE_SIZE' in a:
        a['hbm_bytes'] = int(a['FETCH_SIZE'] * 1024 * 2 + a['WRITE_SIZE'] * 1024)
    if a.get('TCC_HIT_sum') is not None and a.get('TCC_MISS_sum'):
        a['l2_hit_rate'] = round(a['TCC_HIT_sum'] / (a['TCC_HIT_sum'] + a['TCC_MISS_sum']), 3)
    a['us'] = round(a['us'], 2)
dec = {k: v for k, v in kern.items() if is_dec(k)}
step = {'calls': calls, 'kernels': sorted(dec),
        'us_per_call': round(sum(v['us'] for v in dec.values()) / calls, 2),
        'hbm_bytes_per_call': int(sum(v.get('hbm_bytes', 0) for v in dec.values()) / calls)}
out = {'decode_step': step, 'kernels': dict(sorted(kern.items(), key=lambda kv: -kv[1]['us']))}
json.dump(out, open(dst, 'w'), indent=1)
print(json.dumps(step))
