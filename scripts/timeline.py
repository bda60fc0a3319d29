#!/usr/bin/env python3
"""Print the kernel timeline (start offset, duration, gap before) of the last
step(s) of a rocprofv3 kernel trace: shows where a step's wall time goes
between kernels.  usage: timeline.py run_kernel_trace.csv [first_kernel_regex] [n]"""
import csv
import re
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
pat = re.compile(sys.argv[2] if len(sys.argv) > 2 else "k_chunk_sizes")
n = int(sys.argv[3]) if len(sys.argv) > 3 else 40
idx = [i for i, r in enumerate(rows) if pat.search(r["Kernel_Name"])]
start = idx[-2] - 6 if len(idx) >= 2 else 0
t0 = int(rows[start]["Start_Timestamp"])
prev_end = t0
for r in rows[start:start + n]:
    s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
    name = r["Kernel_Name"].split("(")[0].replace("void ", "")[:70]
    print(f"{(s - t0) / 1e3:9.1f} us  dur {(e - s) / 1e3:8.1f}  gap {(s - prev_end) / 1e3:7.1f}  {name}")
    prev_end = max(prev_end, e)
