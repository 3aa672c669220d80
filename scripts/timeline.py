#!/usr/bin/env python3
"""Print one step's kernel timeline (gaps = device idle) from a rocprofv3 kernel trace CSV.
usage: timeline.py run_kernel_trace.csv FIRST_KERNEL_PREFIX [min_gap_us]"""
import csv
import sys

rows = sorted(csv.DictReader(open(sys.argv[1])), key=lambda r: int(r["Start_Timestamp"]))
first = sys.argv[2]
min_gap = float(sys.argv[3]) if len(sys.argv) > 3 else 0.0
idx = [i for i, r in enumerate(rows) if first in r["Kernel_Name"]]
s, e = (idx[-2], idx[-1]) if len(idx) > 1 else (idx[-1], len(rows))
t0 = prev = int(rows[s]["Start_Timestamp"])
busy = idle = 0
for r in rows[s:e]:
    st, en = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
    gap = st - prev
    busy += en - st
    idle += max(gap, 0)
    if gap / 1e3 >= min_gap or (en - st) / 1e3 >= 50:
        print(f"{(st - t0) / 1e3:9.1f} gap {gap / 1e3:8.1f} dur {(en - st) / 1e3:8.1f}  {r['Kernel_Name'][:60]}")
    prev = max(prev, en)
print(f"span {(prev - t0) / 1e3:.1f} us  busy {busy / 1e3:.1f}  idle {idle / 1e3:.1f}")
