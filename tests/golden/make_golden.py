#!/usr/bin/env python3
"""Generate the committed golden fixtures (tests/golden/*.npz).

Inputs are seeded synthetic footprints (dss_amd.workload) plus every geometry
the reference's own tests and prober fixtures use; expected outputs come from
the CPU oracle (oracle/), whose covering restatement is pinned by the
reference's 20-cell KAT (pkg/models/geo_test.go:10-55).  Regenerate with
    python tests/golden/make_golden.py
Loaded with numpy.load(allow_pickle=False).
"""
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, ROOT)

from dss_amd import workload as W  # noqa: E402
from oracle import oracle as O  # noqa: E402

# (lat, lng) polygons from the reference tests / prober fixtures (data only).
REF_POLYGONS = [
    # pkg/models/geo_test.go:11-29 (KAT), pkg/geo/testdata/testdata.go:10
    [(37.427636, -122.170502), (37.408799, -122.064069), (37.421265, -122.086504)],
    # pkg/geo/s2_test.go:13 (odd number of points -> 3 points)
    [(37.4047, -122.1474), (37.4037, -122.1485), (37.4035, -122.1466)],
    # pkg/geo/s2_test.go:19 (clockwise -> reversal path)
    [(0.000, 0.000), (0.000, 0.005), (-0.005, 0.0025)],
    # pkg/geo/s2_test.go:25 (duplicate last vertex)
    [(37.4047, -122.1474), (37.4037, -122.1485), (37.4035, -122.1466), (37.4035, -122.1466)],
    # monitoring/prober/rid/common.py:7-27 VERTICES
    [(-23.6558, 130.6205), (-23.6898, 130.6301), (-23.6709, 130.6700), (-23.6407, 130.6466)],
    # monitoring/prober/rid/common.py:29-49 HUGE_VERTICES (-> area too large)
    [(-23, 130), (-24, 130), (-24, 132), (-23, 132)],
    # monitoring/prober/scd/resources/op_request_3.json (3 identical vertices)
    [(37.78943798147498, -122.45464324951172)] * 3,
    # monitoring/prober/scd/resources/op_request_1.json extent 0 (closed ring)
    [(32.59415886402617, -117.1035655786647), (32.59415886402617, -117.1038398819344),
     (32.64920727813973, -117.1038398819344), (32.64920727813973, -117.1035655786647),
     (32.59415886402617, -117.1035655786647)],
    # op_request_1.json extent 1
    [(32.629403155814224, -117.07235209637365), (32.62913940035541, -117.07227677467183),
     (32.61019036953776, -117.15071909262814), (32.61045408389095, -117.15079458449262),
     (32.629403155814224, -117.07235209637365)],
    # op_request_1.json extent 2
    [(32.63060966167485, -117.09038826289287), (32.630365389882776, -117.09026347832622),
     (32.60141106631151, -117.15717622635013), (32.601655284082824, -117.15730113575759),
     (32.63060966167485, -117.09038826289287)],
    # out of range / too few points (status fixtures)
    [(91.0, 0.0), (0.0, 0.0), (1.0, 1.0)],
    [(37.4, -122.1), (37.5, -122.2)],
]
# (lat, lng, radius_m) circles from the prober (monitoring/prober/scd/*)
REF_CIRCLES = [(-56, 178, 50), (-56, 178, 300), (89.999, 0, 200), (89.999, 180, 300), (90, 0, 300),
               (12, -34, 300), (12.00001, -34.00001, 50), (0, 0, 0), (37.0, -122.0, -5.0)]


def edge_case_footprints(rng, n):
    """Footprints at poles, the antimeridian, the equator and cube-face
    edges/corners, where the projection and clipping code is stressed."""
    centres = [(89.95, 10.0), (-89.95, -100.0), (0.0, 179.999), (0.0, -179.999), (0.0, 0.0),
               (35.2643896827546, 45.0), (-35.2643896827546, 135.0), (0.0, 45.0), (45.0, 0.0), (0.0, 135.0),
               (45.0, 90.0), (-45.0, -90.0), (35.26, -135.0), (10.0, 45.0000001), (60.0, 179.9999)]
    out = []
    for k in range(n):
        la, lg = centres[k % len(centres)]
        sub = W.metro_footprints(rng, 1, (la, la, lg, lg), rmax=2500.0)
        if k % 2 == 1 and sub.kind[0] == W.KIND_POLYGON:
            sub.kind[0] = 2  # DSSG_KIND_POINTS: geo.Covering without the range check (Q5)
        out.append(sub)
    return out


def concat(fps):
    kind = np.concatenate([f.kind for f in fps])
    rad = np.concatenate([f.radius_m for f in fps])
    lat = np.concatenate([f.lat for f in fps])
    lng = np.concatenate([f.lng for f in fps])
    counts = np.concatenate([np.diff(f.voff) for f in fps])
    voff = np.zeros(len(kind) + 1, dtype=np.int64)
    np.cumsum(counts, out=voff[1:])
    return W.Footprints(kind, voff, lat, lng, rad)


def ref_footprints():
    fps = []
    for poly in REF_POLYGONS:
        la = np.array([p[0] for p in poly], dtype=np.float64)
        lg = np.array([p[1] for p in poly], dtype=np.float64)
        fps.append(W.Footprints(np.array([0], np.int32), np.array([0, len(poly)], np.int64), la, lg,
                                np.zeros(1, np.float32)))
    for la, lg, r in REF_CIRCLES:
        fps.append(W.Footprints(np.array([1], np.int32), np.array([0, 1], np.int64), np.array([la], np.float64),
                                np.array([lg], np.float64), np.array([r], np.float32)))
    return fps


def main():
    rng = np.random.default_rng(20201015)
    fps = ref_footprints()
    fps.append(W.metro_footprints(rng, 1000))
    fps.extend(edge_case_footprints(rng, 300))
    # corridors (long thin polygons, config 4 shape) and small city blocks
    fps.append(W.metro_footprints(rng, 100, W.CONUS, circle_frac=0.0, rmin=2000.0, rmax=12000.0))
    cov = concat(fps)
    offs, cells, status, area = O.cover_batch(cov.kind, cov.voff, cov.lat, cov.lng, cov.radius_m)
    np.savez_compressed(os.path.join(HERE, "covering.npz"), kind=cov.kind, voff=cov.voff, lat=cov.lat, lng=cov.lng,
                        radius_m=cov.radius_m, offs=offs, cells=cells, status=status, area_km2=area)
    print("covering:", cov.n, "footprints,", len(cells), "cells, status counts", np.bincount(status))

    # search: 3000 intents + 500 queries in a 20x20 km box (dense overlap),
    # with NULL and boundary combinations (Q8-Q10).
    srng = np.random.default_rng(20201016)
    box = (37.40, 37.58, -122.20, -121.98)
    it = W.metro_footprints(srng, 3000, box)
    ia = W.intent_attrs(srng, 3000)
    q = W.metro_footprints(srng, 500, box)
    qa = W.query_attrs(srng, 500)
    # boundary cases: exact-equality times and altitudes against intent 0..49
    for k in range(50):
        j = k
        if k % 5 == 0:
            qa.t0[k], qa.t1[k] = ia.t1[j], ia.t1[j] + 1000      # q.start == e.end (closed, Q10)
        elif k % 5 == 1:
            qa.t0[k], qa.t1[k] = ia.t0[j] - 1000, ia.t0[j]      # q.end == e.start
        elif k % 5 == 2:
            qa.alt_lo[k], qa.alt_hi[k] = ia.alt_hi[j], ia.alt_hi[j] + 5
        elif k % 5 == 3:
            qa.alt_lo[k], qa.alt_hi[k] = -np.inf, np.inf         # NULL altitudes
        else:
            qa.t0[k], qa.t1[k] = np.iinfo(np.int64).min, np.iinfo(np.int64).max
    # some intents with NULL start / NULL end / NULL altitude (Q9)
    ia.t0[100:110] = np.iinfo(np.int64).min
    ia.t1[110:120] = np.iinfo(np.int64).min
    ia.alt_lo[120:130] = -np.inf
    ia.alt_hi[130:140] = np.inf
    io, ic, ist, _ = O.cover_batch(it.kind, it.voff, it.lat, it.lng, it.radius_m)
    qo, qc, qst, _ = O.cover_batch(q.kind, q.voff, q.lat, q.lng, q.radius_m)
    now = W.T0_US + 6 * W.HOUR_US
    tlo = np.maximum(qa.t0, now)
    owner = srng.integers(0, 7, 3000).astype(np.int32)
    rq, re = O.search(io, ic, ia.alt_lo, ia.alt_hi, ia.t0, ia.t1, owner, qo, qc, qa.alt_lo, qa.alt_hi, tlo, qa.t1)
    qown = srng.integers(-1, 7, 500).astype(np.int32)
    sq, se = O.search(io, ic, np.full(3000, -np.inf, np.float32), np.full(3000, np.inf, np.float32), ia.t0, ia.t1,
                      owner, qo, qc, np.full(500, -np.inf, np.float32), np.full(500, np.inf, np.float32),
                      np.full(500, now, np.int64), np.full(500, np.iinfo(np.int64).max, np.int64), qown)
    np.savez_compressed(os.path.join(HERE, "search.npz"), e_offs=io, e_cells=ic, e_alt_lo=ia.alt_lo,
                        e_alt_hi=ia.alt_hi, e_t0=ia.t0, e_t1=ia.t1, e_owner=owner, q_offs=qo, q_cells=qc,
                        q_alt_lo=qa.alt_lo, q_alt_hi=qa.alt_hi, q_start=qa.t0, q_end=qa.t1, now=np.int64(now),
                        pairs_q=rq, pairs_e=re, q_owner=qown, subs_q=sq, subs_e=se)
    print("search:", len(rq), "op pairs,", len(sq), "subscription pairs")


if __name__ == "__main__":
    main()
