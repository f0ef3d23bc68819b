#!/usr/bin/env python3
"""Summarize rocprofv3 output of tools/profile.sh: per kernel, the dispatch
count, average duration (kernel trace) and the average of every collected
counter per dispatch.  FETCH_SIZE is reported raw and x2 (gfx950 counts half
the bytes of wide coalesced reads, MI355X_MICROARCH.md s HBM)."""
import csv
import glob
import os
import re
import sys
from collections import defaultdict


def short(name):
    m = re.search(r"(k_\w+)", name)
    return m.group(1) if m else name[:40]


def main(d):
    dur = defaultdict(list)
    for f in glob.glob(os.path.join(d, "**", "*kernel_trace.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            if os.path.basename(f).startswith("kt"):
                dur[short(r["Kernel_Name"])].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e6)
    ctr = defaultdict(lambda: defaultdict(list))
    for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            ctr[short(r["Kernel_Name"])][r["Counter_Name"]].append(float(r["Counter_Value"]))
    names = sorted(set(dur) | set(ctr), key=lambda k: -sum(dur.get(k, [0])))
    cols = sorted({c for k in ctr for c in ctr[k]})
    print("kernel,dispatches,avg_ms,total_ms," + ",".join(cols) + (",FETCH_SIZE_x2_bytes" if "FETCH_SIZE" in cols else ""))
    for k in names:
        ds = dur.get(k, [])
        row = [k, str(len(ds)), f"{(sum(ds) / len(ds)) if ds else 0:.4f}", f"{sum(ds):.3f}"]
        for c in cols:
            v = ctr[k].get(c, [])
            row.append(f"{sum(v) / len(v):.6g}" if v else "")
        if "FETCH_SIZE" in cols:
            v = ctr[k].get("FETCH_SIZE", [])
            row.append(f"{2 * 1024 * sum(v) / len(v):.6g}" if v else "")  # FETCH_SIZE is in KiB
        print(",".join(row))


if __name__ == "__main__":
    main(sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/prof")
