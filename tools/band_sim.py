"""Altitude-banded tiles, simulated (analysis only, not product code).

The counting build (profiles/r06a) shows that on configs[2] the altitude
predicate rejects 38 % of k_join's lane tests (58 % of those that pass the
time test).  Today a quad's postings are tiled 64 at a time in m = min(t0, t1)
order, so a tile spans every altitude and a record can only be skipped by the
tile's time hull.  Here each dense quad's regular postings are split into B
altitude bands (global alt_lo quantiles), each band tiled in m order, and a
record is staged for a tile only if it meets both the tile's time hull and
its altitude hull [min alt_lo, max alt_hi].

Counts per scheme: loaded records (the unit's record range), staged records,
lane tests (staged x tile postings) and tiles, over the quads with >= DENSE
postings and over all quads.  usage (GPU box, for the covering):
    python tools/band_sim.py [config] [scale] [B list] [dense list]"""
import json
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from dss_amd import geo, workload as W  # noqa: E402

WIDE = 1 << 32


def main():
    cfg = int(sys.argv[1]) if len(sys.argv) > 1 else 2
    scale = float(sys.argv[2]) if len(sys.argv) > 2 else 1.0
    bands = [int(x) for x in (sys.argv[3] if len(sys.argv) > 3 else "1,2,4").split(",")]
    denses = [int(x) for x in (sys.argv[4] if len(sys.argv) > 4 else "512,2048").split(",")]
    qs, qa, it, ia, now, _ = W.config_split(cfg, 0, scale)
    gi = geo.cover_batch(it.kind, it.voff, it.lat, it.lng, it.radius_m)
    gq = geo.cover_batch(qs.kind, qs.voff, qs.lat, qs.lng, qs.radius_m)
    # one posting per (entity, quad), one record per (query, quad)
    def groups(offs, cells):
        ent = np.repeat(np.arange(len(offs) - 1), np.diff(offs))
        key = (ent.astype(np.uint64) << np.uint64(32)) | (cells >> np.uint64(37))
        u = np.unique(key)
        return (u >> np.uint64(32)).astype(np.int64), (u & np.uint64(0xFFFFFFFF)).astype(np.int64)
    pe, pq = groups(gi.offs, gi.cells)
    re_, rq = groups(gq.offs, gq.cells)
    t0, t1 = ia.t0.astype(np.float64), ia.t1.astype(np.float64)
    m_all, x_all = np.minimum(t0, t1), np.maximum(t0, t1)
    qtlo = np.maximum(qa.t0, now).astype(np.float64)
    qthi = qa.t1.astype(np.float64)
    dcap = float(np.max(x_all - m_all))
    wide_all = (qthi >= qtlo) & ((qthi - qtlo) > WIDE)
    dqmax = float(np.max(np.where(~wide_all & (qthi >= qtlo), qthi - qtlo, 0)))
    thr = np.quantile(ia.alt_lo, np.linspace(0, 1, 9)[1:-1])  # octile edges of alt_lo
    po = np.lexsort((m_all[pe], pq))
    pe, pq = pe[po], pq[po]
    ro = np.lexsort((qtlo[re_], rq))
    re_, rq = re_[ro], rq[ro]
    uq, ps, pc = np.unique(pq, return_index=True, return_counts=True)
    ur, rs, rc = np.unique(rq, return_index=True, return_counts=True)
    common, ia_, ib_ = np.intersect1d(uq, ur, assume_unique=True, return_indices=True)
    schemes = [(b, d) for b in bands for d in (denses if b > 1 else [0])]
    res = {f"B{b}_dense{d}": [0, 0, 0, 0] for b, d in schemes}
    hot = {f"B{b}_dense{d}": [0, 0, 0, 0] for b, d in schemes}
    for k in range(len(common)):
        if k % 20000 == 0:
            print(f"[band_sim] quad {k} of {len(common)}", file=sys.stderr, flush=True)
        e = pe[ps[ia_[k]]: ps[ia_[k]] + pc[ia_[k]]]
        q = re_[rs[ib_[k]]: rs[ib_[k]] + rc[ib_[k]]]
        m, x, alo, ahi = m_all[e], x_all[e], ia.alt_lo[e], ia.alt_hi[e]
        rlo, rhi, ralo, rahi = qtlo[q], qthi[q], qa.alt_lo[q], qa.alt_hi[q]
        wd = wide_all[q]
        nlo, nhi, nalo, nahi = rlo[~wd], rhi[~wd], ralo[~wd], rahi[~wd]
        wlo, whi, walo, wahi = rlo[wd], rhi[wd], ralo[wd], rahi[wd]
        for b, d in schemes:
            nb = b if len(e) >= d else 1
            band = np.searchsorted(thr[(8 // nb) - 1::8 // nb][: nb - 1], alo, side="right") if nb > 1 else \
                np.zeros(len(e), np.int64)
            acc = [0, 0, 0, 0]
            for bb in range(nb):
                g = np.nonzero(band == bb)[0]  # (m order kept)
                for a in range(0, len(g), 64):
                    tl = g[a: a + 64]
                    mf, ml, hmax = m[tl[0]], m[tl[-1]], x[tl].max()
                    hlo, hhi = (alo[tl].min(), ahi[tl].max()) if nb > 1 else (-np.inf, np.inf)
                    lo = np.searchsorted(nlo, mf - dqmax, side="left")
                    hi = np.searchsorted(nlo, ml + dcap, side="right")
                    sl = slice(lo, hi)
                    st = np.count_nonzero((nlo[sl] <= hmax) & (nhi[sl] >= mf) & (nahi[sl] >= hlo) & (nalo[sl] <= hhi))
                    st += np.count_nonzero((wlo <= hmax) & (whi >= mf) & (wahi >= hlo) & (walo <= hhi))
                    acc[0] += (hi - lo) + len(wlo)
                    acc[1] += st
                    acc[2] += st * len(tl)
                    acc[3] += 1
            key = f"B{b}_dense{d}"
            for i in range(4):
                res[key][i] += acc[i]
                if len(e) >= max(d, 512):
                    hot[key][i] += acc[i]
    out = {"config": cfg, "scale": scale, "quads_met": int(len(common)), "dcap_min": dcap / 6e7,
           "dqmax_min": dqmax / 6e7, "alt_lo_octiles": [float(t) for t in thr]}
    for name, r in (("all", res), ("quads_ge_512_postings", hot)):
        out[name] = {k: {"loaded": int(v[0]), "staged": int(v[1]), "lane_tests": int(v[2]), "tiles": int(v[3])} for k, v in r.items()}
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
