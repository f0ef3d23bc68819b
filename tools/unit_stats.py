"""Shape of a config's join work per touched cell (no time narrowing): per
cell P postings (intent cells) and R records (query cells); a unit is one
64-posting tile of a touched cell with all of the cell's R records.  Prints
how the units and their (posting x record) products split by size class.
usage (GPU box): python tools/unit_stats.py [config] [scale]"""
import json
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from dss_amd import geo, workload as W  # noqa: E402


def main():
    cfg = int(sys.argv[1]) if len(sys.argv) > 1 else 2
    scale = float(sys.argv[2]) if len(sys.argv) > 2 else 1.0
    _, q, qa, it, ia, now = W.config(cfg, scale=scale)
    gi = geo.cover_batch(it.kind, it.voff, it.lat, it.lng, it.radius_m)
    gq = geo.cover_batch(q.kind, q.voff, q.lat, q.lng, q.radius_m)
    ic, pc = np.unique(gi.cells, return_counts=True)
    qc, rc = np.unique(gq.cells, return_counts=True)
    common, ii, qi = np.intersect1d(ic, qc, assume_unique=True, return_indices=True)
    P, R = pc[ii].astype(np.int64), rc[qi].astype(np.int64)
    tiles = (P + 63) // 64
    out = {"config": cfg, "scale": scale, "intent_cells": int(len(gi.cells)), "query_cells": int(len(gq.cells)),
           "cells_with_postings": int(len(ic)), "touched_cells": int(len(common)), "units": int(tiles.sum()),
           "posting_lanes": int(P.sum()), "unit_records_upper": int((tiles * R).sum()),
           "lane_tests_upper": int((P * R).sum())}
    # classes by the cell's postings
    for lo, hi in [(1, 8), (8, 32), (32, 64), (64, 256), (256, 1024), (1024, 1 << 40)]:
        m = (P >= lo) & (P < hi)
        out[f"P[{lo},{hi})"] = {"cells": int(m.sum()), "units": int(tiles[m].sum()), "mean_R": float(R[m].mean()) if m.any() else 0,
                                "lane_tests_upper": int((P[m] * R[m]).sum()), "posting_lanes": int(P[m].sum())}
    for lo, hi in [(1, 2), (2, 4), (4, 16), (16, 64), (64, 1 << 40)]:
        m = (R >= lo) & (R < hi)
        out[f"R[{lo},{hi})"] = {"cells": int(m.sum()), "units": int(tiles[m].sum()), "mean_P": float(P[m].mean()) if m.any() else 0}
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
