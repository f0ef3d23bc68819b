"""GPU parity of the general covering pipeline (batches above the wave path's
16384 footprints) on the geometry its special paths handle -- GPU == CPU
oracle bit for bit (status, cells, area):

* small loops straddling cube-face edges and corners (multi-face: the
  descent, started at the bound's level-13 cells by k_start / k_start13);
* zero-area loops (Q3: open polylines; the descent's coarse test before the
  exact list), across face edges and inside faces;
* small loops with vertices on level-13 cell corners and edges 1e-15..1e-12
  off cell boundary lines (k_cand_fp's float prefilter next to the exact
  double tests);
* footprints that the triage hands to the exact setup (k_setup_exact,
  a wave per listed footprint): fan loops around a pole.

Semantics: pkg/geo/s2.go:99-122 (Covering), pkg/models/geo.go:224-268.
"""
import numpy as np
import pytest

from test_gpu_covering import _check_batch, _corner_uv, _face_uv_to_latlng

pytestmark = pytest.mark.gpu


def _base_footprints(rng):
    polys = []
    d = 4e-5
    for face in range(6):
        # straddling each face edge and corner: a few level-13 cells on each side
        for (u, v) in ((1.0, 0.3), (-1.0, -0.2), (0.4, 1.0), (-0.7, -1.0), (1.0, 1.0), (-1.0, 1.0), (1.0, -1.0)):
            for s in (1.0, 2.0, 5.0):
                e = s * d
                polys.append([_face_uv_to_latlng(face, *p) for p in
                              ((u - e, v - e), (u + e, v - e), (u + e, v + e), (u - e, v + e))])
                polys.append([_face_uv_to_latlng(face, *p) for p in
                              ((u + e, v + e), (u + e, v - e), (u - e, v - e), (u - e, v + e))])  # clockwise: Q4
                # zero area (A, B, A): an open polyline across the edge
                a, b = (u - e, v - 0.5 * e), (u + e, v + 0.5 * e)
                polys.append([_face_uv_to_latlng(face, *p) for p in (a, b, a)])
        # inside the face: cell corners, boundary-hugging edges, polylines
        for _ in range(4):
            u, v = _corner_uv(rng)
            a = rng.uniform(0, 2 * np.pi)
            polys.append([_face_uv_to_latlng(face, *p) for p in
                          ((u, v), (u + d * np.cos(a), v + d * np.sin(a)), (u + d * np.cos(a + 2), v + d * np.sin(a + 2)))])
            for off in (0.0, 1e-15, -1e-13, 1e-12):
                uu = u + off
                polys.append([_face_uv_to_latlng(face, *p) for p in
                              ((uu, v - 2 * d), (uu, v + 2 * d), (uu + (d if off >= 0 else -d), v))])
            p0, p1 = (u, v), (u + 3 * d, v + 1.5 * d)
            polys.append([_face_uv_to_latlng(face, *p) for p in (p0, p1, p0)])
    # around the poles (fan terms far from the fan origin: the exact setup)
    for lat0 in (89.9995, -89.9995):
        for k in (3, 5, 8):
            polys.append([(lat0, -180.0 + 360.0 * i / k) for i in range(k)])
    return polys


@pytest.mark.parametrize("seed", [7, 8])
def test_general_pipeline_special_paths(oracle, seed):
    from dss_amd import geo
    rng = np.random.default_rng(seed)
    base = _base_footprints(rng)
    # replicate with small seeded jitter past the wave path's batch limit
    reps = 20000 // len(base) + 1
    polys = []
    for r in range(reps):
        for p in base:
            if r == 0:
                polys.append(p)
                continue
            j = rng.normal(0, 2e-6, size=(len(p), 2))
            polys.append([(float(np.clip(la + dj[0], -90, 90)), float(((ln + dj[1] + 180) % 360) - 180))
                          for (la, ln), dj in zip(p, j)])
    assert len(polys) > 16384
    kind = np.zeros(len(polys), np.int32)
    voff = np.zeros(len(polys) + 1, np.int64)
    voff[1:] = np.cumsum([len(p) for p in polys])
    lat = np.array([q[0] for p in polys for q in p], dtype=np.float64)
    lng = np.array([q[1] for p in polys for q in p], dtype=np.float64)
    rad = np.zeros(len(polys), np.float32)
    offs, cells, status, area = oracle.cover_batch(kind, voff, lat, lng, rad)
    res = geo.cover_batch(kind, voff, lat, lng, rad)
    _check_batch(dict(status=status, offs=offs, cells=cells, area_km2=area), res)
    assert (status == 0).sum() > len(polys) // 2


def _origin_latlng():
    """OriginPoint (s2 point.go OriginPoint) in degrees."""
    o = np.array([-0.0099994664350250197, 0.0025924542609324121, 0.99994664350250195])
    o /= np.linalg.norm(o)
    return float(np.degrees(np.arcsin(o[2]))), float(np.degrees(np.arctan2(o[1], o[0])))


def _offset(lat, lng, dist_rad, bearing):
    """The point dist_rad from (lat, lng) along bearing (radians)."""
    la, ln = np.radians(lat), np.radians(lng)
    la2 = np.arcsin(np.sin(la) * np.cos(dist_rad) + np.cos(la) * np.sin(dist_rad) * np.cos(bearing))
    ln2 = ln + np.arctan2(np.sin(bearing) * np.sin(dist_rad) * np.cos(la), np.cos(dist_rad) - np.sin(la) * np.sin(la2))
    return float(np.degrees(la2)), float(((np.degrees(ln2) + 180) % 360) - 180)


def test_general_pipeline_around_origin_point(oracle):
    """The setup's origin shortcuts (circles whose cap excludes OriginPoint;
    polygons k_orient proves simple, counter-clockwise or clockwise, whose
    0.05 rad cap excludes it) next to the footprints that keep the crossing
    walk: circles and rings containing OriginPoint, passing just beside it,
    and with their caps' edge at 0.99 .. 1.01 of the distance.  GPU (general
    pipeline) == oracle, bit for bit."""
    from dss_amd import geo
    rng = np.random.default_rng(11)
    olat, olng = _origin_latlng()
    circles, polys = [], []
    for r_m in (80.0, 1500.0, 30000.0):
        r = r_m / 6371010.0
        for f in (0.0, 0.5, 0.97, 0.999, 1.001, 1.03, 2.0, 10.0):
            for b in (0.3, 2.1, 4.4):
                circles.append((*_offset(olat, olng, f * r, b), r_m))
    for ring in (2e-5, 4e-4, 8e-3):  # ring radius (rad)
        for f in (0.0, 0.6, 1.02, 3.0, 0.05 / ring + 2.0, 0.05 / ring + 40.0):
            for k in (3, 5, 9):
                clat, clng = _offset(olat, olng, f * ring, rng.uniform(0, 2 * np.pi))
                pts = [_offset(clat, clng, ring, 2 * np.pi * i / k) for i in range(k)]
                polys.append(pts)
                polys.append(pts[::-1])  # the other orientation (Q4 reversal of a clockwise ring)
    base = [("c", c) for c in circles] + [("p", p) for p in polys]
    reps = 17000 // len(base) + 1
    kinds, verts, rads = [], [], []
    for r in range(reps):
        for t, g in base:
            j = 0.0 if r == 0 else 1e-7
            if t == "c":
                kinds.append(1)
                verts.append([(g[0] + rng.normal(0, j), g[1] + rng.normal(0, j))])
                rads.append(g[2])
            else:
                kinds.append(0)
                verts.append([(la + rng.normal(0, j), ln + rng.normal(0, j)) for la, ln in g])
                rads.append(0.0)
    assert len(kinds) > 16384
    kind = np.array(kinds, np.int32)
    voff = np.zeros(len(verts) + 1, np.int64)
    voff[1:] = np.cumsum([len(v) for v in verts])
    lat = np.array([q[0] for v in verts for q in v], dtype=np.float64)
    lng = np.array([q[1] for v in verts for q in v], dtype=np.float64)
    rad = np.array(rads, np.float32)
    offs, cells, status, area = oracle.cover_batch(kind, voff, lat, lng, rad)
    res = geo.cover_batch(kind, voff, lat, lng, rad)
    _check_batch(dict(status=status, offs=offs, cells=cells, area_km2=area), res)
    assert (status == 0).sum() > len(kinds) // 2
