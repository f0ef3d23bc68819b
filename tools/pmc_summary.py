#!/usr/bin/env python3
"""Summarize rocprofv3 output of tools/profile.sh: per kernel, the dispatch
count, average duration (kernel trace) and the average of every collected
counter per dispatch.

HBM bytes per launch follow MI355X_MICROARCH.md s HBM: FETCH_SIZE and
WRITE_SIZE are KiB; on gfx950 FETCH_SIZE reports half the bytes of a wide
coalesced read, so hbm = 2 * 1024 * FETCH_SIZE + 1024 * WRITE_SIZE (an upper
bound where a kernel's reads are narrower than 16 B per lane).

usage: pmc_summary.py DIR [--json OUT --queries NQ --intents NI --source TAG]
"""
import argparse
import csv
import glob
import json
import os
import re
from collections import defaultdict


def short(name):
    """Kernel name with its template arguments (k_join<false, true>): the
    variants of one kernel are summarized apart."""
    m = re.search(r"(k_\w+(?:<[^>(]*>)?)", name)
    return m.group(1) if m else name[:40]


def collect(d, skip_first=0):
    """Per kernel: durations (ms) and counter values per dispatch, in dispatch
    order, without each kernel's first `skip_first` dispatches (the intents'
    covering / index build and the first search's capacity growth: what is
    left is one steady-state search per dispatch)."""
    dur = defaultdict(list)
    for f in glob.glob(os.path.join(d, "**", "*kernel_trace.csv"), recursive=True):
        if not os.path.basename(f).startswith("kt"):
            continue
        rows = sorted(csv.DictReader(open(f)), key=lambda r: int(r.get("Dispatch_Id") or r["Start_Timestamp"]))
        for r in rows:
            dur[short(r["Kernel_Name"])].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e6)
    ctr = defaultdict(lambda: defaultdict(list))
    for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
        rows = list(csv.DictReader(open(f)))
        if rows and "Dispatch_Id" in rows[0]:
            rows.sort(key=lambda r: int(r["Dispatch_Id"]))
        for r in rows:
            ctr[short(r["Kernel_Name"])][r["Counter_Name"]].append(float(r["Counter_Value"]))
    if skip_first:
        dur = defaultdict(list, {k: v[skip_first:] for k, v in dur.items()})
        for k in ctr:
            for c in ctr[k]:
                ctr[k][c] = ctr[k][c][skip_first:]
    return dur, ctr


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("dir", nargs="?", default="gpurun_out/prof")
    ap.add_argument("--json")
    ap.add_argument("--queries", type=int)
    ap.add_argument("--intents", type=int)
    ap.add_argument("--source", default="")
    ap.add_argument("--skip-first", type=int, default=0,
                    help="drop each kernel's first N dispatches (setup + the first search's capacity growth)")
    a = ap.parse_args()
    dur, ctr = collect(a.dir, a.skip_first)
    names = sorted(set(dur) | set(ctr), key=lambda k: -sum(dur.get(k, [0])))
    cols = sorted({c for k in ctr for c in ctr[k]})
    print("kernel,dispatches,avg_ms,total_ms," + ",".join(cols) + ",hbm_bytes_per_launch")
    out = {}
    for k in names:
        ds = dur.get(k, [])
        avg = lambda c: (sum(ctr[k][c]) / len(ctr[k][c])) if ctr[k].get(c) else None  # noqa: E731
        row = [k, str(len(ds)), f"{(sum(ds) / len(ds)) if ds else 0:.4f}", f"{sum(ds):.3f}"]
        row += [f"{avg(c):.6g}" if avg(c) is not None else "" for c in cols]
        f, w = avg("FETCH_SIZE"), avg("WRITE_SIZE")
        hbm = 2 * 1024 * f + 1024 * w if f is not None and w is not None else None
        row.append(f"{hbm:.6g}" if hbm is not None else "")
        print(",".join(row))
        out[k] = {"dispatches": len(ds), "avg_ms": (sum(ds) / len(ds)) if ds else None,
                  "fetch_kib": f, "write_kib": w, "hbm_bytes_per_launch": hbm}
    # a kernel launched as several template variants per search (k_join's
    # short and long variants): the base name carries the per-search sum of
    # the variants' per-launch averages
    groups = {}
    for k, v in out.items():
        if "<" in k and v["hbm_bytes_per_launch"] is not None:
            groups.setdefault(k.split("<")[0], []).append(v)
    for base, vs in groups.items():
        if len(vs) > 1 and base not in out:
            out[base] = {"dispatches": sum(v["dispatches"] for v in vs), "avg_ms": sum(v["avg_ms"] or 0 for v in vs),
                         "fetch_kib": sum(v["fetch_kib"] for v in vs), "write_kib": sum(v["write_kib"] for v in vs),
                         "hbm_bytes_per_launch": sum(v["hbm_bytes_per_launch"] for v in vs),
                         "note": "per search: the sum over the template variants, each launched once per search"}
    if a.json:
        with open(a.json, "w") as fh:
            json.dump({"source": a.source, "queries": a.queries, "intents": a.intents, "skip_first": a.skip_first,
                       "correction": "hbm = 2*1024*FETCH_SIZE + 1024*WRITE_SIZE (MI355X_MICROARCH.md s HBM)",
                       "kernels": {k: v for k, v in out.items() if v["hbm_bytes_per_launch"] is not None}},
                      fh, indent=1)


if __name__ == "__main__":
    main()
