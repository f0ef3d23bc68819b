#!/usr/bin/env python3
"""FP64 VALU throughput of the covering kernels from tools/profile.sh's
pmc_f64 pass: flops per launch = 64 x (2 FMA + ADD + MUL) wave instructions
(TOTAL_64_OPS without the MFMA and INT64 terms; an upper bound where lanes
are masked off), over the kernel's average duration from the kernel trace.
Peak: MI355X FP64 vector 78.6 TFLOP/s.
usage: fp64_summary.py DIR OUT.json [QUERIES INTENTS SKIP_FIRST SOURCE]"""
import json
import sys

sys.path.insert(0, __file__.rsplit("/", 1)[0])
from pmc_summary import collect  # noqa: E402

PEAK = 78.6
d, out = sys.argv[1], sys.argv[2]
nq = int(sys.argv[3]) if len(sys.argv) > 3 else None
ni = int(sys.argv[4]) if len(sys.argv) > 4 else None
skip = int(sys.argv[5]) if len(sys.argv) > 5 else 0
src = sys.argv[6] if len(sys.argv) > 6 else d
dur, ctr = collect(d, skip)
rows = {}
for k, c in ctr.items():
    if "SQ_INSTS_VALU_FMA_F64" not in c or k not in dur:
        continue
    avg = lambda n: sum(c[n]) / len(c[n]) if c.get(n) else 0.0  # noqa: E731
    fl = 64 * (2 * avg("SQ_INSTS_VALU_FMA_F64") + avg("SQ_INSTS_VALU_ADD_F64") + avg("SQ_INSTS_VALU_MUL_F64"))
    if fl <= 0:
        continue
    ms = sum(dur[k]) / len(dur[k])
    rows[k] = {"avg_ms": ms, "fp64_flops_per_launch": fl, "trans_f64_insts": avg("SQ_INSTS_VALU_TRANS_F64"),
               "tflops": fl / (ms * 1e-3) / 1e12, "frac_of_fp64_peak": fl / (ms * 1e-3) / 1e12 / PEAK}
res = {"source": src, "queries": nq, "intents": ni, "skip_first": skip, "peak_tflops": PEAK, "kernels": dict(sorted(rows.items(), key=lambda kv: -kv[1]["avg_ms"]))}
json.dump(res, open(out, "w"), indent=1)
for k, r in list(res["kernels"].items())[:12]:
    print(f"{k:20s} {r['avg_ms']:.4f} ms  {r['tflops']:.2f} TFLOP/s  {100 * r['frac_of_fp64_peak']:.1f}%")
