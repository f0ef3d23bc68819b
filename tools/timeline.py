#!/usr/bin/env python3
"""Print one bench step's kernel timeline from a rocprofv3 kernel trace
(gaps between kernels show host synchronisation).  usage: timeline.py CSV [STEP_FROM_END]"""
import csv
import re
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
back = int(sys.argv[2]) if len(sys.argv) > 2 else 2
rows.sort(key=lambda r: int(r['Start_Timestamp']))
idx = [i for i, r in enumerate(rows) if 'k_nverts' in r['Kernel_Name']]
i0 = idx[-back]
t0 = int(rows[i0]['Start_Timestamp'])
prev = t0
for r in rows[i0:]:
    s, e = int(r['Start_Timestamp']), int(r['End_Timestamp'])
    m = re.search(r'(k_\w+)', r['Kernel_Name'])
    n = m.group(1) if m else r['Kernel_Name'][:30]
    print(f"{(s - t0) / 1e3:9.1f}us gap {(s - prev) / 1e3:7.1f} dur {(e - s) / 1e3:8.1f} {n} grid={r['Grid_Size_X']} vgpr={r['VGPR_Count']}")
    prev = e
    if 'k_join' in n:
        break
