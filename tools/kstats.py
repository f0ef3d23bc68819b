#!/usr/bin/env python3
"""Average kernel durations from rocprofv3 kernel_stats CSVs.
usage: kstats.py STATS.csv [STATS.csv ...] [-k name,name]"""
import csv
import re
import sys

args = sys.argv[1:]
names = None
if "-k" in args:
    i = args.index("-k")
    names = args[i + 1].split(",")
    args = args[:i] + args[i + 2:]
for path in args:
    print("==", path)
    for r in csv.DictReader(open(path)):
        m = re.findall(r"(k_\w+(?:<[^>]*>)?|__amd\w+)", r["Name"])
        name = m[0] if m else r["Name"][:40]
        if names and not any(name.startswith(n) for n in names):
            continue
        print(f"  {name:40s} calls {int(r['Calls']):5d} avg_us {float(r['AverageNs']) / 1000:9.1f} "
              f"total_ms {float(r['TotalDurationNs']) / 1e6:8.2f}")
