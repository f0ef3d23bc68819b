#!/usr/bin/env python3
"""Kernels around the last-but-one k_join of a rocprofv3 kernel trace (one
bench step's join phase and what follows it).
usage: steptrace.py CSV [KERNEL] [BEFORE] [AFTER]"""
import csv
import re
import sys

path = sys.argv[1]
anchor = sys.argv[2] if len(sys.argv) > 2 else "k_join"
before = int(sys.argv[3]) if len(sys.argv) > 3 else 20
after = int(sys.argv[4]) if len(sys.argv) > 4 else 40
rows = sorted(csv.DictReader(open(path)), key=lambda r: int(r["Start_Timestamp"]))
idx = [i for i, r in enumerate(rows) if anchor in r["Kernel_Name"]]
i = idx[-2] if len(idx) > 1 else idx[-1]
t0 = int(rows[i]["Start_Timestamp"])
prev = None
for r in rows[max(0, i - before):i + after]:
    s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
    name = " ".join(re.findall(r"(k_\w+|__amd\w+)", r["Kernel_Name"])[:2])
    gap = (s - prev) / 1000 if prev else 0.0
    print(f"{(s - t0) / 1000:10.1f} gap {gap:7.1f} dur {(e - s) / 1000:9.1f} {name}")
    prev = e
