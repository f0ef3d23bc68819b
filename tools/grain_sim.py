"""Posting grain of the join (analysis only, not product code): how many
(query, entity) meetings, postings, records and tiled-join lane tests a
config produces when postings and query records are kept per level-L cell
group (L = 13: one level-13 cell; 12: quads of 2 x 2; 11: 4 x 4; 10: 8 x 8)
instead of per level-13 cell.  Coverings from the CPU oracle, so it runs on
any host.

  meetings  python tools/grain_sim.py meetings CFG SCALE LEVEL
            spatial (query, entity) meetings per group, those passing the
            time / altitude filter, those whose cell masks intersect, the
            meetings per distinct pair and the share where neither side is
            in its first group (the DISTINCT checks that need signatures);
  tiles     python tools/grain_sim.py tiles CFG SCALE
            the band join's shape at L = 13 and 12: postings, records, 64-
            posting tiles, tiles with a record, staged records (records whose
            window meets a tile's time hull) and lane tests (staged x tile
            size).

DESIGN.md s5 quotes its configs[2] / configs[3] numbers (round 5)."""
import sys

import numpy as np

sys.path.insert(0, __import__("os").path.dirname(__import__("os").path.dirname(__import__("os").path.abspath(__file__))))
from dss_amd import workload as W  # noqa: E402
from oracle import oracle as O  # noqa: E402


def covered(cfg, scale):
    q, qa, it, ia, now, _ = W.config_split(cfg, 0, scale, 1.0)
    io, ic, _, _ = O.cover_batch(it.kind, it.voff, it.lat, it.lng, it.radius_m, nthreads=8)
    qo, qc, _, _ = O.cover_batch(q.kind, q.voff, q.lat, q.lng, q.radius_m, nthreads=8)
    ie = np.repeat(np.arange(it.n), np.diff(io))
    qe = np.repeat(np.arange(q.n), np.diff(qo))
    return q, qa, it, ia, now, ic, qc, ie, qe


def meetings(cfg, scale, lv):
    import pandas as pd
    q, qa, it, ia, now, ic, qc, ie, qe = covered(cfg, scale)
    tlo, thi = np.maximum(qa.t0, now), qa.t1
    sh = 35 + 2 * (13 - lv)
    blk = lambda c: (c >> np.uint64(sh)).astype(np.int64)  # noqa: E731
    child = lambda c: ((c >> np.uint64(35)) & np.uint64((1 << (2 * (13 - lv))) - 1)).astype(np.int64)  # noqa: E731
    I = pd.DataFrame({"e": ie, "c": ic.view(np.int64), "b": blk(ic), "ch": child(ic)})
    Q = pd.DataFrame({"q": qe, "c": qc.view(np.int64), "b": blk(qc), "ch": child(qc)})

    def groups(df, key):
        df = df.assign(bit=np.left_shift(np.uint64(1), df.ch.values.astype(np.uint64)))
        g = df.groupby([key, "b"], sort=False)["bit"].agg(lambda s: np.bitwise_or.reduce(s.values)).reset_index()
        g["rank"] = g.groupby(key).cumcount()
        return g.rename(columns={"bit": "mask"})

    def passing(df):
        e, qq = df.e.values, df.q.values
        return (ia.t1[e] >= tlo[qq]) & (ia.t0[e] <= thi[qq]) & (ia.alt_hi[e] >= qa.alt_lo[qq]) & \
            (ia.alt_lo[e] <= qa.alt_hi[qq])

    IB, QB = groups(I, "e"), groups(Q, "q")
    M = I[["e", "c"]].merge(Q[["q", "c"]], on="c")
    Mf = M[passing(M)]
    pairs = len(Mf[["q", "e"]].drop_duplicates())
    B = IB.merge(QB, on="b", suffixes=("_e", "_q"))
    Bf = B[passing(B)]
    Ba = Bf[(Bf.mask_e.values.astype(np.uint64) & Bf.mask_q.values.astype(np.uint64)) != 0]
    both = (Ba.rank_e.values > 0) & (Ba.rank_q.values > 0)
    print(f"configs[{cfg}] scale {scale} level {lv}: postings/entity {len(IB) / it.n:.3f} (cells {len(I) / it.n:.3f}), "
          f"records/query {len(QB) / q.n:.3f}")
    print(f"  cell grain : spatial meetings {len(M)}, passing {len(Mf)}, pairs {pairs}, meetings/pair "
          f"{len(Mf) / max(1, pairs):.3f}")
    print(f"  level {lv}   : spatial meetings {len(B)} ({len(B) / max(1, len(M)):.3f}x), passing {len(Bf)}, masks meet "
          f"{len(Ba)}, meetings/pair {len(Ba) / max(1, pairs):.3f}, both non-first {both.mean():.3f}")


def tiles(cfg, scale):
    q, qa, it, ia, now, ic, qc, ie, qe = covered(cfg, scale)
    tlo, thi = np.maximum(qa.t0, now), qa.t1
    for lv in (13, 12):
        sh = 35 + 2 * (13 - lv)
        pe = np.unique(((ic >> np.uint64(sh)) << np.uint64(24)) | ie.astype(np.uint64))
        pk, pent = pe >> np.uint64(24), (pe & np.uint64((1 << 24) - 1)).astype(np.int64)
        re_ = np.unique(((qc >> np.uint64(sh)) << np.uint64(24)) | qe.astype(np.uint64))
        rk, rq = re_ >> np.uint64(24), (re_ & np.uint64((1 << 24) - 1)).astype(np.int64)
        m = np.minimum(ia.t0[pent], ia.t1[pent])
        mx = np.maximum(ia.t0[pent], ia.t1[pent])
        o = np.lexsort((m, pk))
        pk, m, mx = pk[o], m[o], mx[o]
        _, pstart, pcnt = np.unique(pk, return_index=True, return_counts=True)
        tid = np.repeat(pstart, pcnt) + ((np.arange(len(pk)) - np.repeat(pstart, pcnt)) // 64) * 64
        tstarts = np.unique(tid)
        t0min, t1max = m[tstarts], np.maximum.reduceat(mx, tstarts)
        tnp = np.diff(np.append(tstarts, len(pk)))
        tkey = pk[tstarts]
        o1 = np.lexsort((tlo[rq], rk))
        o2 = np.lexsort((thi[rq], rk))
        a1, a2 = tlo[rq][o1], thi[rq][o2]
        rkeys, rstart, rcnt = np.unique(rk[o1], return_index=True, return_counts=True)
        cnt = np.zeros(len(tstarts), np.int64)
        order = np.argsort(tkey, kind="stable")
        ukeys, ustart, ucnt = np.unique(tkey[order], return_index=True, return_counts=True)
        for key, a, c in zip(ukeys, ustart, ucnt):
            j = np.searchsorted(rkeys, key)
            if j >= len(rkeys) or rkeys[j] != key:
                continue
            A, Bv = a1[rstart[j]:rstart[j] + rcnt[j]], a2[rstart[j]:rstart[j] + rcnt[j]]
            tt = order[a:a + c]
            cnt[tt] = np.searchsorted(A, t1max[tt], side="right") - np.searchsorted(Bv, t0min[tt], side="left")
        cnt = np.maximum(cnt, 0)
        print(f"configs[{cfg}] scale {scale} level {lv}: postings {len(pk)} records {len(rk)} tiles {len(tstarts)} "
              f"tiles with records {(cnt > 0).sum()} staged records {cnt.sum()} lane tests {(cnt * tnp).sum()}")


if __name__ == "__main__":
    if sys.argv[1] == "meetings":
        meetings(int(sys.argv[2]), float(sys.argv[3]), int(sys.argv[4]))
    else:
        tiles(int(sys.argv[2]), float(sys.argv[3]))
