#!/usr/bin/env python3
"""Summarise a scripts/profile.sh run (gpurun_out/prof) for profiles/.

HBM traffic per launch follows MI355X_MICROARCH.md "HBM": FETCH_SIZE and
WRITE_SIZE are in KiB; on gfx950 FETCH_SIZE reads exactly half the bytes of a
wide coalesced stream, so it is doubled; WRITE_SIZE is taken as is.
"""
import collections
import csv
import json
import os
import sys

src = sys.argv[1] if len(sys.argv) > 1 else 'gpurun_out/prof'
kname = sys.argv[2] if len(sys.argv) > 2 else 'encode_independent'
out = {}
stats = list(csv.DictReader(open(os.path.join(src, 'trace/run_kernel_stats.csv'))))
for r in stats:
    if kname in r['Name']:
        out['kernel'] = r['Name']
        out['calls'] = int(r['Calls'])
        out['avg_ns'] = float(r['AverageNs'])
        out['min_ns'] = float(r['MinNs'])
        out['max_ns'] = float(r['MaxNs'])
for grp in ('fetch', 'write', 'sq', 'sq2'):
    p = os.path.join(src, grp, 'run_counter_collection.csv')
    if not os.path.exists(p):
        continue
    agg = collections.defaultdict(list)
    for r in csv.DictReader(open(p)):
        if kname in r['Kernel_Name']:
            agg[r['Counter_Name']].append(float(r['Counter_Value']))
    for k, v in agg.items():
        out[k] = sum(v) / len(v)
if 'FETCH_SIZE' in out and 'WRITE_SIZE' in out:
    out['hbm_read_bytes_corrected'] = out['FETCH_SIZE'] * 1024 * 2
    out['hbm_write_bytes'] = out['WRITE_SIZE'] * 1024
    out['hbm_traffic_bytes_per_launch'] = out['hbm_read_bytes_corrected'] + out['hbm_write_bytes']
    if 'avg_ns' in out:
        out['hbm_GBps'] = out['hbm_traffic_bytes_per_launch'] / out['avg_ns']
# the headline launch alone (the 4096-chunk batch: the largest grid in the trace);
# run_kernel_stats also counts the host-inclusive sub-batch launches
import glob  # noqa: E402
tr = glob.glob(os.path.join(src, 'trace', '**', 'run_kernel_trace.csv'), recursive=True)
if tr:
    rows = [r for r in csv.DictReader(open(tr[0])) if kname in r['Kernel_Name']]
    if rows:
        gmax = max(int(r['Grid_Size_X']) for r in rows)
        full = [(int(r['End_Timestamp']) - int(r['Start_Timestamp'])) for r in rows if int(r['Grid_Size_X']) == gmax]
        out['avg_ns_full_batch'] = sum(full) / len(full)
        out['calls_full_batch'] = len(full)
        out['grid_full_batch'] = gmax
        if 'hbm_traffic_bytes_per_launch' in out:
            out['hbm_GBps_full_batch'] = out['hbm_traffic_bytes_per_launch'] / out['avg_ns_full_batch']
        out['note'] = ('avg_ns / calls include the host-inclusive sub-batch launches; avg_ns_full_batch is the '
                       'headline launch alone (kernel trace, largest grid); PMC counters come from --no-extras runs '
                       '(headline launches only)')
print(json.dumps(out, indent=1))
