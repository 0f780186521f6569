"""Print the kernel timeline of the last rep (from the last cache_wipe) of a
rocprofv3 kernel trace: start offset and duration in microseconds."""
import csv
import sys
rows = list(csv.DictReader(open(sys.argv[1])))
rows.sort(key=lambda r: int(r['Start_Timestamp']))
rows = [r for r in rows if 'rocclr_copyBuffer' not in r['Kernel_Name'] or
        int(r['End_Timestamp']) - int(r['Start_Timestamp']) < 100000]
mark = sys.argv[2] if len(sys.argv) > 2 else 'cache_wipe'
idx = [i for i, r in enumerate(rows) if mark in r['Kernel_Name']]
i0 = idx[-1]
t0 = int(rows[i0]['Start_Timestamp'])
for r in rows[i0:i0 + int(sys.argv[3]) if len(sys.argv) > 3 else i0 + 40]:
    s, e = int(r['Start_Timestamp']), int(r['End_Timestamp'])
    print(f"{(s - t0) / 1000:9.1f} {(e - s) / 1000:8.1f} {r['Kernel_Name'][:60]}")
