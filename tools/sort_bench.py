"""Sort-phase measurement: the hand-written radix sort (dssg_radix_sort_device)
on the index build's and the join's key shapes, HBM GB/s against the 24 B per
posting algorithmic model of SURVEY.md s8(d) (8 B key + 4 B payload, read and
written once), with torch.sort (rocPRIM) timed beside it on the same keys."""
import ctypes as C
import json
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from dss_amd import _lib  # noqa: E402

SHAPES = [  # (name, n, bits, key_bytes)
    ("index build (cell, entity), configs[1]", 6_694_323, 64, 8),
    ("index build, 62 live key bits", 6_694_323, 62, 8),
    ("join key grouping (group id, record), configs[1]", 11_627_810, 18, 4),
    ("50M-posting index (configs[4] scale)", 50_000_000, 64, 8),
    ("level-13 cell ids (29 varying bits), configs[2] postings", 64_212_362, 64, 8),
    ("level-13 cell ids (29 varying bits), configs[1] postings", 6_694_323, 64, 8),
]


def main():
    ctx = _lib.context()
    rows = []
    for name, n, bits, kb in SHAPES:
        g = torch.Generator(device="cuda").manual_seed(n)
        if "level-13" in name:  # face + 26-bit position + the level-13 sentinel bit
            k = (torch.randint(0, 1 << 29, (n,), dtype=torch.int64, device="cuda", generator=g) << 35) | (1 << 34)
        elif kb == 8:
            k = torch.randint(0, 2**62, (n,), dtype=torch.int64, device="cuda", generator=g)
            if bits < 64:
                k = k & ((1 << bits) - 1)
        else:
            k = torch.randint(0, 1 << bits, (n,), dtype=torch.int32, device="cuda", generator=g)
        v = torch.arange(n, dtype=torch.int32, device="cuda")
        ko, vo = torch.empty_like(k), torch.empty_like(v)
        torch.cuda.synchronize()  # the library sorts on its own stream
        ms = C.c_double(0)
        best = 1e9
        for _ in range(6):
            ctx.check(ctx.L.dssg_radix_sort_device(ctx.h, kb, n, bits, C.c_void_p(k.data_ptr()),
                                                   C.c_void_p(ko.data_ptr()), C.c_void_p(v.data_ptr()),
                                                   C.c_void_p(vo.data_ptr()), None, C.byref(ms)))
            best = min(best, ms.value)
        # torch.sort (rocPRIM segmented radix sort) on the same keys, stable
        kk = k if kb == 8 else k.to(torch.int64)
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        tbest = 1e9
        for _ in range(6):
            e0.record()
            torch.sort(kk, stable=True)
            e1.record()
            torch.cuda.synchronize()
            tbest = min(tbest, e0.elapsed_time(e1))
        ok = (bool(torch.equal(ko, torch.sort(k if kb == 8 else k, stable=True).values))
              if (bits >= 62 and "level-13" not in name) or kb == 4 else None)
        if "level-13" in name:  # signed int64 order differs from uint64 order on faces 4-5: compare as uint
            ku = k.cpu().numpy().view(np.uint64)
            ok = bool(np.array_equal(ko.cpu().numpy().view(np.uint64), np.sort(ku, kind="stable")))
        alg = 2 * (kb + 4) * n
        rows.append({"shape": name, "onesweep": os.environ.get("DSS_RADIX_ONESWEEP", "1") != "0", "n": n, "bits": bits, "key_bytes": kb, "ms": best, "alg_bytes": alg,
                     "GBs": alg / best / 1e6, "frac_of_8TBs": alg / best / 1e6 / 8000.0, "torch_sort_ms": tbest,
                     "sorted_equal_torch": ok})
        print(json.dumps(rows[-1]), flush=True)


if __name__ == "__main__":
    main()
