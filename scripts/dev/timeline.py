"""Per-launch timeline of the last repetition in a rocprofv3 kernel trace
(`--kernel-trace [--memory-copy-trace] --output-format csv`): start, duration
and idle gap before each dispatch, from the last launch of MARK on.
Usage: python3 scripts/dev/timeline.py TRACE_DIR [MARK]"""
import csv
import glob
import os
import sys

d = sys.argv[1]
mark = sys.argv[2] if len(sys.argv) > 2 else 'cache_wipe'
ev = []
for f in glob.glob(os.path.join(d, '*kernel_trace.csv')):
    ev += [(int(x['Start_Timestamp']), int(x['End_Timestamp']), x['Kernel_Name'][:60]) for x in csv.DictReader(open(f))]
for f in glob.glob(os.path.join(d, '*memory_copy_trace.csv')):
    ev += [(int(x['Start_Timestamp']), int(x['End_Timestamp']), 'copy ' + x['Direction']) for x in csv.DictReader(open(f))]
ev.sort()
starts = [i for i, e in enumerate(ev) if mark in e[2]]
s = starts[-2] if len(starts) > 1 and ev[starts[-1] - 1][2].find(mark) >= 0 else starts[-1]
t0 = prev = ev[s][0]
print(f"{'start_us':>9} {'dur_us':>8} {'gap_us':>8}  dispatch")
for e in ev[s:]:
    if e[0] - prev > 1_000_000:
        break
    print(f'{(e[0] - t0) / 1e3:9.1f} {(e[1] - e[0]) / 1e3:8.1f} {(e[0] - prev) / 1e3:8.1f}  {e[2]}')
    prev = e[1]
