"""GPU parity: gfx950 covering (through the C ABI) == CPU oracle, bit for bit.

Covers the reference KAT (pkg/models/geo_test.go:10-55), the status-level
cases of pkg/geo/s2_test.go, the committed golden fixtures (reference fixture
geometries, poles, antimeridian, cube-face edges/corners, corridors), and
seeded random batches at config-0 shape.
"""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu

KAT = ("808fb0ac 808fb744 808fb754 808fb75c 808fb9fc 808fba04 808fba0c 808fba14 808fba1c 808fba5c "
       "808fba64 808fba6c 808fba74 808fba8c 808fbad4 808fbadc 808fbae4 808fbaec 808fbaf4 808fbb2c").split()


def tok(c):
    return f"{int(c):016x}".rstrip("0")


def test_polygon_covering_kat():
    from dss_amd.geo import GeoPolygon, LatLngPoint
    got = GeoPolygon([LatLngPoint(37.427636, -122.170502), LatLngPoint(37.408799, -122.064069),
                      LatLngPoint(37.421265, -122.086504)]).CalculateCovering()
    assert [tok(c) for c in got] == KAT


@pytest.mark.parametrize("area,exc", [
    ("37.4047,-122.1474,37.4037,-122.1485,37.4035,-122.1466", None),
    ("0.000,0.000, 0.000,0.005, -0.005,0.0025", None),
    ("37.4047,-122.1474,37.4037,-122.1485,37.4035,-122.1466,37.4035,-122.1466", None),
    ("37.427636,-122.170502,37.408799,-122.064069,37.421265,-122.086504", None),
    ("", "OddNumberOfCoordinatesError"),
    ("37.427636,-122.170502,37.408799,-122.064069", "NotEnoughPointsError"),
    ("37.427636,-122.170502,37.408799", "OddNumberOfCoordinatesError"),
    ("37.4,-122.1,abc,-122.2,37.5,-122.3", "BadCoordSetError"),
    ("-23,130,-24,130,-24,132,-23,132", "ErrAreaTooLarge"),
    # Go's splitAtComma gives no empty final token: 7 tokens -> 3 points + a dropped latitude
    ("37.4047,-122.1474,37.4037,-122.1485,37.4035,-122.1466,1,", None),
    ("37.4047,-122.1474,37.4037,-122.1485,37.4035,-122.1466,", "OddNumberOfCoordinatesError"),
    (",37.4047,-122.1474,37.4037,-122.1485,37.4035", "BadCoordSetError"),
    ("37.4047,-122.1474,,37.4037,-122.1485,37.4035,-122.1466,1", "BadCoordSetError"),
    ("37.4047,-122.147_4,37.4037,-122.1485,37.4035,-122.1466", "BadCoordSetError"),
    (" 37.4047 ,-122.1474,\t37.4037,-122.1485,37.4035,-122.1466 ", None),  # TrimSpace
    ("0x1.2ap5,-122.1474,37.4037,-122.1485,37.4035,-122.1466", None),    # Go hex float syntax
])
def test_area_to_cell_ids(oracle, area, exc):
    """pkg/geo/s2.go:129-166 through the C ABI: the status, and the cells
    equal to the restatement (tests/test_oracle_kat.py) over the oracle's
    Covering."""
    from dss_amd import geo
    from test_oracle_kat import area_to_cell_ids
    if exc is None:
        cells = geo.AreaToCellIDs(area)
        rc, want = area_to_cell_ids(oracle, area)
        assert rc == oracle.OK
        assert len(cells) > 0 and [int(c) for c in cells] == [int(c) for c in want]
    else:
        with pytest.raises(getattr(geo, exc)):
            geo.AreaToCellIDs(area)


def test_area_too_large_message_matches_oracle(oracle):
    from dss_amd import geo
    _, _, area = oracle.polygon_covering([-23, -24, -24, -23], [130, 130, 132, 132])
    with pytest.raises(geo.ErrAreaTooLarge) as ei:
        geo.AreaToCellIDs("-23,130,-24,130,-24,132,-23,132")
    assert str(ei.value) == "area is too large (%fkm² > %fkm²)" % (area, 2500.0)


def _check_batch(g, res):
    assert np.array_equal(res.status, g["status"]), np.nonzero(res.status != g["status"])
    bad = np.nonzero(np.diff(res.offs) != np.diff(g["offs"]))[0]
    assert len(bad) == 0, f"cell-count mismatch at footprints {bad[:10]}"
    if not np.array_equal(res.cells, g["cells"]):
        diff = np.nonzero(res.cells != g["cells"])[0]
        fps = np.unique(np.searchsorted(g["offs"], diff, side="right") - 1)
        f = int(fps[0])
        a, b = int(g["offs"][f]), int(g["offs"][f + 1])
        raise AssertionError(f"{len(fps)} footprints differ, first {f}: got {[tok(c) for c in res.cells[a:b]]} "
                             f"want {[tok(c) for c in g['cells'][a:b]]}")
    assert np.array_equal(res.area_km2.view(np.uint64), g["area_km2"].view(np.uint64))


def test_golden_covering(golden_covering):
    from dss_amd import geo
    g = golden_covering
    res = geo.cover_batch(g["kind"], g["voff"], g["lat"], g["lng"], g["radius_m"])
    _check_batch(g, res)


@pytest.mark.parametrize("seed", [0, 1])
def test_random_metro_batch(oracle, seed):
    from dss_amd import geo, workload as W
    rng = np.random.default_rng(1000 + seed)
    fp = W.metro_footprints(rng, 20000)
    offs, cells, status, area = oracle.cover_batch(fp.kind, fp.voff, fp.lat, fp.lng, fp.radius_m)
    res = geo.cover_batch(fp.kind, fp.voff, fp.lat, fp.lng, fp.radius_m)
    _check_batch(dict(status=status, offs=offs, cells=cells, area_km2=area), res)


def test_corridors_and_blocks(oracle):
    from dss_amd import geo, workload as W
    rng = np.random.default_rng(77)
    a = W.metro_footprints(rng, 2000, W.CONUS, circle_frac=0.0, rmin=3000.0, rmax=40000.0)
    offs, cells, status, area = oracle.cover_batch(a.kind, a.voff, a.lat, a.lng, a.radius_m)
    res = geo.cover_batch(a.kind, a.voff, a.lat, a.lng, a.radius_m)
    _check_batch(dict(status=status, offs=offs, cells=cells, area_km2=area), res)


def test_big_circle_and_many_vertices(oracle):
    from dss_amd import geo
    # a 400 km circle (no area cap for circles, Q2) and a 200-vertex polygon
    th = np.linspace(0, 2 * np.pi, 200, endpoint=False)
    la = 10 + 0.05 * np.sin(th)
    lg = 20 + 0.05 * np.cos(th)
    kind = np.array([1, 0], np.int32)
    voff = np.array([0, 1, 201], np.int64)
    lat = np.concatenate([[45.0], la])
    lng = np.concatenate([[7.0], lg])
    rad = np.array([400000.0, 0.0], np.float32)
    offs, cells, status, area = oracle.cover_batch(kind, voff, lat, lng, rad)
    res = geo.cover_batch(kind, voff, lat, lng, rad)
    _check_batch(dict(status=status, offs=offs, cells=cells, area_km2=area), res)
    assert offs[1] > 50000


def test_empty_batch():
    from dss_amd import geo
    res = geo.cover_batch(np.zeros(0, np.int32), np.zeros(1, np.int64), np.zeros(0), np.zeros(0), np.zeros(0))
    assert len(res.cells) == 0 and len(res.offs) == 1


def _ring(clat, clng, r_deg, k, cw, jitter=None):
    th = np.linspace(0, 2 * np.pi, k, endpoint=False)
    rr = r_deg * (np.ones(k) if jitter is None else jitter)
    la, lg = clat + rr * np.sin(th), clng + rr * np.cos(th) / np.cos(np.radians(clat))
    return (la[::-1], lg[::-1]) if cw else (la, lg)


def test_fan_orientation_edge_cases(oracle):
    """k_orient's three cases against the oracle: loops whose fan-sum sign is
    predicted (forward only / reversed only) and the undecided ones that
    evaluate both fans -- near the 2500 km2 cap, beyond the 0.05 rad window,
    bow-ties and spikes whose fan terms cancel, degenerate and repeated
    vertices, down to metre-sized loops."""
    from dss_amd import geo
    rng = np.random.default_rng(404)
    polys = []
    for cw in (False, True):
        for r_deg in (1e-5, 3e-4, 0.01, 0.2, 0.25, 0.27, 0.29, 2.0, 3.5):   # 1 m .. ~390 km
            for k in (3, 4, 7, 12):
                polys.append(_ring(37.5, -122.2, r_deg, k, cw))
        # spiky stars: alternating radii, fan terms of both signs
        for k in (8, 16, 30):
            jit = np.where(np.arange(k) % 2 == 0, 1.0, rng.uniform(0.02, 0.2))
            polys.append(_ring(37.5, -122.2, 0.02, k, cw, jit))
    # bow-tie (self-intersecting: the fan terms cancel), collinear, repeated vertices
    polys.append((np.array([37.0, 37.01, 37.0, 37.01]), np.array([-122.0, -121.99, -121.99, -122.0])))
    polys.append((np.array([37.0, 37.005, 37.01]), np.array([-122.0, -121.995, -121.99])))
    polys.append((np.array([37.0, 37.0, 37.01, 37.01, 37.0]), np.array([-122.0, -122.0, -121.99, -122.0, -122.0])))
    polys.append((np.array([37.0, 37.01, 37.0, 37.0]), np.array([-122.0, -121.99, -121.98, -122.0])))
    kind = np.zeros(len(polys), np.int32)
    voff = np.zeros(len(polys) + 1, np.int64)
    voff[1:] = np.cumsum([len(p[0]) for p in polys])
    lat = np.concatenate([p[0] for p in polys])
    lng = np.concatenate([p[1] for p in polys])
    rad = np.zeros(len(polys), np.float32)
    offs, cells, status, area = oracle.cover_batch(kind, voff, lat, lng, rad)
    res = geo.cover_batch(kind, voff, lat, lng, rad)
    _check_batch(dict(status=status, offs=offs, cells=cells, area_km2=area), res)
    # both outcomes of the cap occur
    assert (status == 0).any() and (status != 0).any()


# ---- adversarial geometry: cell boundaries, face edges, poles, antimeridian
def _face_uv_to_latlng(face, u, v):
    """S2 face (u, v) -> (lat, lng) degrees (s2 stuv.go faceUVToXYZ)."""
    x, y, z = [(1, u, v), (-u, 1, v), (-u, -v, 1), (-1, -v, -u), (v, -1, -u), (v, u, -1)][face]
    return np.degrees(np.arctan2(z, np.hypot(x, y))), np.degrees(np.arctan2(y, x))


def _st_to_uv(s):
    return (4 * s * s - 1) / 3 if s >= 0.5 else (1 - 4 * (1 - s) * (1 - s)) / 3


def _corner_uv(rng):
    """(u, v) of a random level-13 cell corner (i, j multiples of 2^17)."""
    k = 1 << 13
    return _st_to_uv(rng.integers(1, k) / k), _st_to_uv(rng.integers(1, k) / k)


def test_adversarial_cell_boundaries(oracle):
    """SURVEY s8(c) residual risk: cells within 1e-15..1e-12 (u, v) of a
    footprint edge.  Footprints with a vertex on a level-13 cell corner, with
    an edge running along a cell boundary line (a constant-u great circle)
    and shifted off it by 1e-15..1e-12, on cube-face edges and face corners;
    GPU == oracle bit for bit (status, cells, area)."""
    from dss_amd import geo
    rng = np.random.default_rng(2024)
    polys = []
    d = 4e-5  # ~ a level-13 cell in (u, v) is ~1.2e-4 near the face centre
    for face in range(6):
        for _ in range(6):
            u, v = _corner_uv(rng)
            # a vertex exactly on the corner, two more nearby
            a = rng.uniform(0, 2 * np.pi)
            pts = [(u, v), (u + d * np.cos(a), v + d * np.sin(a)), (u + d * np.cos(a + 2), v + d * np.sin(a + 2))]
            polys.append([_face_uv_to_latlng(face, *p) for p in pts])
            # an edge along the constant-u boundary line, then shifted off it
            for off in (0.0, 1e-15, -1e-15, 1e-14, -1e-13, 1e-12, -1e-12):
                uu = u + off
                pts = [(uu, v - 2 * d), (uu, v + 2 * d), (uu + (d if off >= 0 else -d), v)]
                polys.append([_face_uv_to_latlng(face, *p) for p in pts])
        # face edges and corners (u, v = +-1)
        for (u, v) in ((1.0, 0.3), (-1.0, -0.2), (0.4, 1.0), (1.0, 1.0), (-1.0, 1.0), (1.0 - 1e-13, -1.0)):
            for sgn in (1, -1):
                pts = [(u, v), (u - sgn * d, v), (u, v - sgn * d)]
                polys.append([_face_uv_to_latlng(face, *p) for p in pts])
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


def test_circles_at_poles_and_antimeridian(oracle):
    """20-gon circles (Q2) of 50 m .. 2 km centred on / next to the poles and
    on both sides of the antimeridian (the prober's near-pole pins,
    monitoring/prober/scd/test_operations_simple.py:32,47,100)."""
    from dss_amd import geo
    centres = [(90.0, 0.0), (-90.0, 0.0), (89.999, 0.0), (89.999, 180.0), (-89.9995, -45.0), (0.0, 180.0),
               (0.0, -180.0), (12.0, 179.9999), (-33.0, -179.99995), (51.5, 180.0), (45.0, 45.0), (35.26438968, 45.0)]
    radii = (50.0, 120.0, 300.0, 800.0, 2000.0)
    lat = np.array([c[0] for c in centres for _ in radii])
    lng = np.array([c[1] for c in centres for _ in radii])
    rad = np.array([r for _ in centres for r in radii], np.float32)
    n = len(lat)
    kind = np.ones(n, np.int32)
    voff = np.arange(n + 1, dtype=np.int64)
    offs, cells, status, area = oracle.cover_batch(kind, voff, lat, lng, rad)
    res = geo.cover_batch(kind, voff, lat, lng, rad)
    _check_batch(dict(status=status, offs=offs, cells=cells, area_km2=area), res)
    assert (status == 0).all()
