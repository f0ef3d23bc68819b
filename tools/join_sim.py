"""Time-dimension shape of a config's join (analysis only, not product code):
per touched cell, its postings sorted by m = min(t0, t1) in 64-posting tiles
and its records (query cells) sorted by quantised start, as k_units /
k_unit_ranges / k_join form them; counts per scheme:
  now      narrow records narrowed to tlo in [m_first - dqmax, m_last + dcap],
           wide records (window > 2^32 us) all loaded, records staged when
           they meet the tile's hull [m_first, max t1];
  classes  the same with each dense cell's postings split into K duration
           classes (tiles per class, dcap per class).
Prints loaded / staged records and lane tests per scheme for the cells with
>= DENSE postings.  usage (GPU box): python tools/join_sim.py [config] [scale] [K]"""
import json
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from dss_amd import geo, workload as W  # noqa: E402

WIDE = 1 << 32
DENSE = 1024


def tiles_of(m, t1, order, tp=64):
    """tile (start index, end index) ranges over `order` (indices sorted by m)."""
    n = len(order)
    return [(a, min(n, a + tp)) for a in range(0, n, tp)]


def main():
    cfg = int(sys.argv[1]) if len(sys.argv) > 1 else 2
    scale = float(sys.argv[2]) if len(sys.argv) > 2 else 1.0
    K = int(sys.argv[3]) if len(sys.argv) > 3 else 4
    _, q, qa, it, ia, now = W.config(cfg, scale=scale)
    gi = geo.cover_batch(it.kind, it.voff, it.lat, it.lng, it.radius_m)
    gq = geo.cover_batch(q.kind, q.voff, q.lat, q.lng, q.radius_m)
    ient = np.repeat(np.arange(it.n), np.diff(gi.offs))
    qent = np.repeat(np.arange(q.n), np.diff(gq.offs))
    qtlo = np.maximum(qa.t0, now)
    qthi = qa.t1
    iord = np.argsort(gi.cells, kind="stable")
    qord = np.argsort(gq.cells, kind="stable")
    ic, istart, icnt = np.unique(gi.cells[iord], return_index=True, return_counts=True)
    qc, qstart, qcnt = np.unique(gq.cells[qord], return_index=True, return_counts=True)
    common, ii, qi = np.intersect1d(ic, qc, assume_unique=True, return_indices=True)
    dense = icnt[ii] >= DENSE
    i_t0, i_t1 = ia.t0, ia.t1
    dur_all = (np.maximum(i_t0, i_t1) - np.minimum(i_t0, i_t1)).astype(np.float64)
    dcap = float(np.max(dur_all))
    nw = ~((qthi >= qtlo) & ((qthi.astype(np.float64) - qtlo.astype(np.float64)) > WIDE))
    dqmax = float(np.max(np.where(nw & (qthi >= qtlo), qthi.astype(np.float64) - qtlo.astype(np.float64), 0)))
    edges = np.quantile(dur_all, np.linspace(0, 1, K + 1))
    res = {"now": [0, 0, 0, 0], "classes": [0, 0, 0, 0]}  # loaded, staged, lane tests, tiles
    for c in np.nonzero(dense)[0]:
        pe = ient[iord[istart[ii[c]]: istart[ii[c]] + icnt[ii[c]]]]
        qe = qent[qord[qstart[qi[c]]: qstart[qi[c]] + qcnt[qi[c]]]]
        t0, t1 = i_t0[pe].astype(np.float64), i_t1[pe].astype(np.float64)
        m = np.minimum(t0, t1)
        mx = np.maximum(t0, t1)
        rlo, rhi = qtlo[qe].astype(np.float64), qthi[qe].astype(np.float64)
        wide = (rhi >= rlo) & ((rhi - rlo) > WIDE)
        nlo = np.sort(rlo[~wide])
        w_lo, w_hi = rlo[wide], rhi[wide]
        for scheme in ("now", "classes"):
            groups = [np.arange(len(pe))]
            caps = [dcap]
            if scheme == "classes":
                d = mx - m
                cl = np.clip(np.searchsorted(edges, d, side="right") - 1, 0, K - 1)
                groups = [np.nonzero(cl == k)[0] for k in range(K)]
                caps = [float(edges[k + 1]) for k in range(K)]
            for g, cap in zip(groups, caps):
                if len(g) == 0:
                    continue
                g = g[np.argsort(m[g], kind="stable")]
                for a in range(0, len(g), 64):
                    tl = g[a: a + 64]
                    mf, ml, hmax = m[tl[0]], m[tl[-1]], mx[tl].max()
                    lo = np.searchsorted(nlo, mf - dqmax, side="left")
                    hi = np.searchsorted(nlo, ml + cap, side="right")
                    cand = nlo[lo:hi]
                    # (narrow records carry their own thi; approximate the hull test by tlo <= hmax)
                    st_n = int(np.count_nonzero(cand <= hmax))
                    st_w = int(np.count_nonzero((w_lo <= hmax) & (w_hi >= mf)))
                    r = res[scheme]
                    r[0] += (hi - lo) + len(w_lo)
                    r[1] += st_n + st_w
                    r[2] += (st_n + st_w) * len(tl)
                    r[3] += 1
    out = {"config": cfg, "scale": scale, "K": K, "dense_cells": int(dense.sum()), "dcap_min": dcap / 6e7,
           "dqmax_min": dqmax / 6e7, "class_edges_min": [float(e) / 6e7 for e in edges]}
    for k, v in res.items():
        out[k] = {"loaded_records": int(v[0]), "staged_records": int(v[1]), "lane_tests": int(v[2]), "tiles": int(v[3])}
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
