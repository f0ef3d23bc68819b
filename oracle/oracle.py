"""ORACLE / TEST INFRASTRUCTURE ONLY.

ctypes front-end for oracle/build/liboracle.so, the CPU restatement of the
reference covering + search semantics.  Only tests/, __graft_entry__.smoke()
and bench.py's cpu_baseline leg may import this module; the product path
(dss_amd) never does.
"""
from __future__ import annotations

import ctypes as C
import os
import subprocess

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
_LIB_PATH = os.path.join(_HERE, "build", "liboracle.so")
_lib = None

OK = 0
ERR_BAD_COORD_SET = 1
ERR_NOT_ENOUGH_POINTS = 2
ERR_ODD_COORDS = 3
ERR_RADIUS = 4
ERR_AREA_TOO_LARGE = 5

KIND_POLYGON = 0
KIND_CIRCLE = 1


def build(force: bool = False) -> str:
    if force or not os.path.exists(_LIB_PATH):
        subprocess.check_call(["make", "-s", "-C", _HERE])
    return _LIB_PATH


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(_LIB_PATH):
            build()
        L = C.CDLL(_LIB_PATH)
        P = C.POINTER
        d, i32, i64, u64, sz = C.c_double, C.c_int32, C.c_int64, C.c_uint64, C.c_size_t
        L.orc_polygon_covering.argtypes = [P(d), P(d), C.c_int, P(u64), sz, P(sz), P(d)]
        L.orc_polygon_covering.restype = C.c_int
        L.orc_circle_covering.argtypes = [d, d, C.c_float, P(u64), sz, P(sz)]
        L.orc_circle_covering.restype = C.c_int
        L.orc_covering_xyz.argtypes = [P(d), C.c_int, P(u64), sz, P(sz), P(d)]
        L.orc_covering_xyz.restype = C.c_int
        L.orc_point_from_degrees.argtypes = [d, d, P(d)]
        L.orc_cellid_from_degrees.argtypes = [d, d, C.c_int]
        L.orc_cellid_from_degrees.restype = u64
        L.orc_loop_area.argtypes = [P(d), C.c_int]
        L.orc_loop_area.restype = d
        L.orc_regular_loop.argtypes = [d, d, C.c_float, C.c_int, P(d)]
        L.orc_cell_uv_bound.argtypes = [u64, P(d)]
        L.orc_cell_center.argtypes = [u64, P(d)]
        L.orc_cellid_from_face_ij_level.argtypes = [C.c_int, C.c_int, C.c_int, C.c_int, P(C.c_int)]
        L.orc_cellid_from_face_ij_level.restype = u64
        for name in ("sin", "cos", "tan", "atan", "asin"):
            f = getattr(L, f"orc_go_{name}")
            f.argtypes = [d]
            f.restype = d
        L.orc_go_atan2.argtypes = [d, d]
        L.orc_go_atan2.restype = d
        L.orc_cover_batch.argtypes = [i64, P(i32), P(i64), P(d), P(d), P(C.c_float), C.c_int,
                                      P(P(i64)), P(P(u64)), P(i32), P(d)]
        L.orc_cover_batch.restype = C.c_int
        L.orc_search.argtypes = [i64, P(i64), P(u64), P(C.c_float), P(C.c_float), P(i64), P(i64), P(i32),
                                 i64, P(i64), P(u64), P(C.c_float), P(C.c_float), P(i64), P(i64), P(i32),
                                 C.c_int, P(P(C.c_uint32)), P(P(C.c_uint32))]
        L.orc_search.restype = i64
        L.orc_index_new.argtypes = [i64, P(i64), P(u64), P(C.c_float), P(C.c_float), P(i64), P(i64), P(i32)]
        L.orc_index_new.restype = C.c_void_p
        L.orc_index_search.argtypes = [C.c_void_p, i64, P(i64), P(u64), P(C.c_float), P(C.c_float), P(i64),
                                       P(i64), P(i32), C.c_int, P(P(C.c_uint32)), P(P(C.c_uint32))]
        L.orc_index_search.restype = i64
        L.orc_index_free.argtypes = [C.c_void_p]
        L.orc_free.argtypes = [C.c_void_p]
        _lib = L
    return _lib


def _p(a, t):
    return a.ctypes.data_as(C.POINTER(t))


def polygon_covering(lats, lngs):
    """pkg/models/geo.go:252 GeoPolygon.CalculateCovering -> (status, cells, area_km2)."""
    L = lib()
    lat = np.ascontiguousarray(lats, dtype=np.float64)
    lng = np.ascontiguousarray(lngs, dtype=np.float64)
    need = C.c_size_t(0)
    area = C.c_double(0)
    cap = 4096
    while True:
        out = np.zeros(cap, dtype=np.uint64)
        rc = L.orc_polygon_covering(_p(lat, C.c_double), _p(lng, C.c_double), len(lat), _p(out, C.c_uint64),
                                    cap, C.byref(need), C.byref(area))
        if rc == OK and need.value > cap:
            cap = need.value
            continue
        return rc, (out[: need.value].copy() if rc == OK else None), area.value


def circle_covering(lat, lng, radius_m):
    """pkg/models/geo.go:224 GeoCircle.CalculateCovering -> (status, cells)."""
    L = lib()
    need = C.c_size_t(0)
    cap = 4096
    while True:
        out = np.zeros(cap, dtype=np.uint64)
        rc = L.orc_circle_covering(float(lat), float(lng), float(np.float32(radius_m)), _p(out, C.c_uint64), cap,
                                   C.byref(need))
        if rc == OK and need.value > cap:
            cap = need.value
            continue
        return rc, (out[: need.value].copy() if rc == OK else None)


def point_from_degrees(lat, lng):
    out = np.zeros(3)
    lib().orc_point_from_degrees(float(lat), float(lng), _p(out, C.c_double))
    return out


def cellid_from_degrees(lat, lng, level=13):
    return int(lib().orc_cellid_from_degrees(float(lat), float(lng), level))


def covering_xyz(xyz):
    """pkg/geo/s2.go:99 Covering on S2 points (reverses a copy in place like Go)."""
    L = lib()
    pts = np.ascontiguousarray(np.array(xyz, dtype=np.float64).reshape(-1, 3).copy())
    need = C.c_size_t(0)
    area = C.c_double(0)
    cap = 4096
    while True:
        out = np.zeros(cap, dtype=np.uint64)
        work = pts.copy()
        rc = L.orc_covering_xyz(_p(work, C.c_double), len(work), _p(out, C.c_uint64), cap, C.byref(need),
                                C.byref(area))
        if rc == OK and need.value > cap:
            cap = need.value
            continue
        return rc, (out[: need.value].copy() if rc == OK else None), area.value


def cover_batch(kind, voff, lat, lng, radius_m, nthreads=8):
    """Batch covering; returns (offs, cells, status, area_km2)."""
    L = lib()
    kind = np.ascontiguousarray(kind, dtype=np.int32)
    voff = np.ascontiguousarray(voff, dtype=np.int64)
    lat = np.ascontiguousarray(lat, dtype=np.float64)
    lng = np.ascontiguousarray(lng, dtype=np.float64)
    rad = np.ascontiguousarray(radius_m, dtype=np.float32)
    n = len(kind)
    status = np.zeros(n, dtype=np.int32)
    area = np.zeros(n, dtype=np.float64)
    po = C.POINTER(C.c_int64)()
    pc = C.POINTER(C.c_uint64)()
    L.orc_cover_batch(n, _p(kind, C.c_int32), _p(voff, C.c_int64), _p(lat, C.c_double), _p(lng, C.c_double),
                      _p(rad, C.c_float), nthreads, C.byref(po), C.byref(pc), _p(status, C.c_int32),
                      _p(area, C.c_double))
    offs = np.ctypeslib.as_array(po, shape=(n + 1,)).copy()
    cells = np.ctypeslib.as_array(pc, shape=(max(int(offs[-1]), 1),))[: int(offs[-1])].copy()
    L.orc_free(C.cast(po, C.c_void_p))
    L.orc_free(C.cast(pc, C.c_void_p))
    return offs, cells, status, area


def search(e_offs, e_cells, e_alt_lo, e_alt_hi, e_t0, e_t1, e_owner,
           q_offs, q_cells, q_alt_lo, q_alt_hi, q_tlo, q_thi, q_owner=None, nthreads=8):
    """Generic overlap search (see oracle.h); returns sorted (q, e) uint32 arrays."""
    L = lib()
    a = lambda x, t: np.ascontiguousarray(x, dtype=t)  # noqa: E731
    e_offs, e_cells = a(e_offs, np.int64), a(e_cells, np.uint64)
    e_alt_lo, e_alt_hi = a(e_alt_lo, np.float32), a(e_alt_hi, np.float32)
    e_t0, e_t1 = a(e_t0, np.int64), a(e_t1, np.int64)
    ne = len(e_offs) - 1
    e_owner = a(e_owner if e_owner is not None else np.zeros(ne), np.int32)
    q_offs, q_cells = a(q_offs, np.int64), a(q_cells, np.uint64)
    q_alt_lo, q_alt_hi = a(q_alt_lo, np.float32), a(q_alt_hi, np.float32)
    q_tlo, q_thi = a(q_tlo, np.int64), a(q_thi, np.int64)
    nq = len(q_offs) - 1
    qown = a(q_owner, np.int32) if q_owner is not None else None
    oq = C.POINTER(C.c_uint32)()
    oe = C.POINTER(C.c_uint32)()
    n = L.orc_search(ne, _p(e_offs, C.c_int64), _p(e_cells, C.c_uint64), _p(e_alt_lo, C.c_float),
                     _p(e_alt_hi, C.c_float), _p(e_t0, C.c_int64), _p(e_t1, C.c_int64), _p(e_owner, C.c_int32),
                     nq, _p(q_offs, C.c_int64), _p(q_cells, C.c_uint64), _p(q_alt_lo, C.c_float),
                     _p(q_alt_hi, C.c_float), _p(q_tlo, C.c_int64), _p(q_thi, C.c_int64),
                     _p(qown, C.c_int32) if qown is not None else C.POINTER(C.c_int32)(),
                     nthreads, C.byref(oq), C.byref(oe))
    rq = np.ctypeslib.as_array(oq, shape=(max(n, 1),))[:n].copy()
    re = np.ctypeslib.as_array(oe, shape=(max(n, 1),))[:n].copy()
    L.orc_free(C.cast(oq, C.c_void_p))
    L.orc_free(C.cast(oe, C.c_void_p))
    return rq, re


class Index:
    """Posting list built once; `search` is the timed CPU-baseline call."""

    def __init__(self, e_offs, e_cells, e_alt_lo, e_alt_hi, e_t0, e_t1, e_owner=None):
        L = lib()
        a = lambda x, t: np.ascontiguousarray(x, dtype=t)  # noqa: E731
        self._keep = [a(e_offs, np.int64), a(e_cells, np.uint64), a(e_alt_lo, np.float32), a(e_alt_hi, np.float32),
                      a(e_t0, np.int64), a(e_t1, np.int64)]
        o, c, lo, hi, t0, t1 = self._keep
        own = a(e_owner, np.int32) if e_owner is not None else None
        self.h = L.orc_index_new(len(o) - 1, _p(o, C.c_int64), _p(c, C.c_uint64), _p(lo, C.c_float),
                                 _p(hi, C.c_float), _p(t0, C.c_int64), _p(t1, C.c_int64),
                                 _p(own, C.c_int32) if own is not None else C.POINTER(C.c_int32)())

    def search(self, q_offs, q_cells, q_alt_lo, q_alt_hi, q_tlo, q_thi, q_owner=None, nthreads=8):
        L = lib()
        a = lambda x, t: np.ascontiguousarray(x, dtype=t)  # noqa: E731
        qo, qc = a(q_offs, np.int64), a(q_cells, np.uint64)
        lo, hi, tl, th = a(q_alt_lo, np.float32), a(q_alt_hi, np.float32), a(q_tlo, np.int64), a(q_thi, np.int64)
        own = a(q_owner, np.int32) if q_owner is not None else None
        oq = C.POINTER(C.c_uint32)()
        oe = C.POINTER(C.c_uint32)()
        n = L.orc_index_search(self.h, len(qo) - 1, _p(qo, C.c_int64), _p(qc, C.c_uint64), _p(lo, C.c_float),
                               _p(hi, C.c_float), _p(tl, C.c_int64), _p(th, C.c_int64),
                               _p(own, C.c_int32) if own is not None else C.POINTER(C.c_int32)(), nthreads,
                               C.byref(oq), C.byref(oe))
        rq = np.ctypeslib.as_array(oq, shape=(max(n, 1),))[:n].copy()
        re = np.ctypeslib.as_array(oe, shape=(max(n, 1),))[:n].copy()
        L.orc_free(C.cast(oq, C.c_void_p))
        L.orc_free(C.cast(oe, C.c_void_p))
        return rq, re

    def __del__(self):
        try:
            lib().orc_index_free(self.h)
        except Exception:
            pass


# ------------------------------------------------- subscription-store queries
# Pure-Python restatements of the SQL (small cases only).

def notify(e_offs, e_cells, e_t1, counters, q_offs, q_cells, now):
    """RID UpdateNotificationIdxsInCells (pkg/rid/cockroach/subscriptions.go:
    204-219) / SCD fetchSubscriptionsForNotification (pkg/scd/store/cockroach/
    subscriptions.go:128-173), one UPDATE per query in batch order:
    `notification_index += 1 WHERE cells && $q AND ends_at >= now RETURNING`.
    Returns (q, e, value) sorted by (e, q) and the final counters."""
    cnt = [int(x) for x in counters]
    cell_sets = [set(int(c) for c in e_cells[e_offs[e]:e_offs[e + 1]]) for e in range(len(e_offs) - 1)]
    out = []
    for q in range(len(q_offs) - 1):
        qs = set(int(c) for c in q_cells[q_offs[q]:q_offs[q + 1]])
        for e, cs in enumerate(cell_sets):
            if int(e_t1[e]) >= now and cs & qs:
                cnt[e] += 1
                out.append((e, q, cnt[e]))
    out.sort()
    return (np.array([q for _, q, _ in out], np.uint32), np.array([e for e, _, _ in out], np.uint32),
            np.array([v for _, _, v in out], np.int64), np.array(cnt, np.int64))


def owner_subscriptions(e_owner, e_t1, q_owner, now):
    """SCD SearchSubscriptions (pkg/scd/store/cockroach/subscriptions.go:
    497-545): LEFT JOIN keeps every row, so `owner = $2 AND ends_at >= $3`
    alone decides (quirk Q7).  Returns sorted (q, e)."""
    rq, re = [], []
    for q, o in enumerate(q_owner):
        for e in range(len(e_owner)):
            if int(e_owner[e]) == int(o) and int(e_t1[e]) >= now:
                rq.append(q)
                re.append(e)
    return np.array(rq, np.uint32), np.array(re, np.uint32)


def max_subscription_count(e_offs, e_cells, e_owner, e_t1, q_offs, q_cells, q_owner, now):
    """RID MaxSubscriptionCountInCellsByOwner (pkg/rid/cockroach/
    subscriptions.go:83-116): unnest(cells) of the owner's unexpired rows,
    filtered by `cell_id = ANY($3)`, COUNT(*) GROUP BY cell_id, IFNULL(MAX, 0).
    A stored array's repeats count each time."""
    out = np.zeros(len(q_offs) - 1, np.int64)
    for q in range(len(q_offs) - 1):
        qs = set(int(c) for c in q_cells[q_offs[q]:q_offs[q + 1]])
        per = {}
        for e in range(len(e_offs) - 1):
            if int(e_owner[e]) != int(q_owner[q]) or int(e_t1[e]) < now:
                continue
            for c in e_cells[e_offs[e]:e_offs[e + 1]]:
                if int(c) in qs:
                    per[int(c)] = per.get(int(c), 0) + 1
        out[q] = max(per.values()) if per else 0
    return out


def token(cell: int) -> str:
    """s2.CellID.ToToken: hex with trailing zeros stripped."""
    if cell == 0:
        return "X"
    return f"{cell:016x}".rstrip("0")


def from_token(tok: str) -> int:
    return int(tok.ljust(16, "0"), 16)
