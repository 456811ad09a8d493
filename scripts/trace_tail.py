"""Print the last N kernels of a rocprofv3 kernel trace (start, end, duration in us, name)."""
import csv
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
rows.sort(key=lambda r: int(r['Start_Timestamp']))
seq = rows[-int(sys.argv[2] if len(sys.argv) > 2 else 30):]
t0 = int(seq[0]['Start_Timestamp'])
for r in seq:
    s = int(r['Start_Timestamp']) - t0
    e = int(r['End_Timestamp']) - t0
    print(f"{s / 1e3:9.1f} {e / 1e3:9.1f} {(e - s) / 1e3:7.1f}  {r['Kernel_Name'][:60]}")
