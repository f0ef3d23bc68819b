"""GPU parity of the general covering's exact setup (k_setup_exact: one wave
per footprint the triage leaves undecided -- vertices, origin walk, Area's fan
sum and the face mask spread over the lanes) against the CPU restatement of
golang/geo, bit for bit (status, loopAreaKm2 bits, level-13 cells).

In production the triage (k_setup) decides all but ~1 footprint per 1M, so a
test knob (dssg_set_tuning "cover_exact_setup") sends every general-path
footprint through the exact setup; "cover_wave" 0 keeps small batches on the
general path.  The batches are the covering suites' own: the configs'
seeded workloads, the golden fixtures, face edges and corners, zero-area
polylines, clockwise rings (Q4 reversal), loops around OriginPoint and the
poles, 200-vertex polygons (several lane passes), bad coordinates.

Semantics: pkg/geo/s2.go:99-122 (Covering), pkg/models/geo.go:224-268.
"""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu

COVER_WAVE_DEFAULT = 16384  # CoverEngine::wave_max_
SLOT_ORDER_DEFAULT = 1  # CoverEngine::slot_order_


@pytest.fixture
def exact_setup():
    from dss_amd import _lib
    ctx = _lib.context(0)
    ctx.set_tuning("cover_wave", 0)
    ctx.set_tuning("cover_exact_setup", 1)
    try:
        yield
    finally:
        ctx.set_tuning("cover_exact_setup", 0)
        ctx.set_tuning("cover_wave", COVER_WAVE_DEFAULT)


def _check(oracle, kind, voff, lat, lng, rad):
    from dss_amd import geo
    from test_gpu_covering import _check_batch
    offs, cells, status, area = oracle.cover_batch(kind, voff, lat, lng, rad)
    res = geo.cover_batch(kind, voff, lat, lng, rad)
    _check_batch(dict(status=status, offs=offs, cells=cells, area_km2=area), res)
    return status


@pytest.mark.parametrize("cfg,scale", [(0, 0.1), (1, 0.005), (2, 0.0005), (3, 0.001), (4, 0.0002)])
def test_exact_setup_on_config_batches(exact_setup, oracle, cfg, scale):
    from dss_amd import workload as W
    _, q, _, it, _, _ = W.config(cfg, scale=scale)
    for fp in (q, it):
        _check(oracle, fp.kind, fp.voff, fp.lat, fp.lng, fp.radius_m)


def test_exact_setup_on_golden_fixtures(exact_setup, golden_covering):
    from dss_amd import geo
    from test_gpu_covering import _check_batch
    g = golden_covering
    _check_batch(g, geo.cover_batch(g["kind"], g["voff"], g["lat"], g["lng"], g["radius_m"]))


def _flat(polys, circles=()):
    kinds, voff, lat, lng, rad = [], [0], [], [], []
    for pts in polys:
        kinds.append(0)
        lat += [a for a, _ in pts]
        lng += [b for _, b in pts]
        voff.append(len(lat))
        rad.append(0.0)
    for la, ln, r in circles:
        kinds.append(1)
        lat.append(la)
        lng.append(ln)
        voff.append(len(lat))
        rad.append(r)
    return (np.array(kinds, np.int32), np.array(voff, np.int64), np.array(lat, np.float64),
            np.array(lng, np.float64), np.array(rad, np.float32))


def test_exact_setup_special_geometry(exact_setup, oracle):
    from test_gpu_cover_general import _base_footprints, _offset, _origin_latlng
    rng = np.random.default_rng(21)
    polys = _base_footprints(rng)
    ring = [(37.40, -122.10), (37.41, -122.10), (37.41, -122.08), (37.40, -122.08)]
    polys += [ring, ring[::-1], [(-23, 130), (-24, 130), (-24, 132), (-23, 132)],
              [(-23, 130), (-23, 132), (-24, 132), (-24, 130)], [(91, 0), (0, 0), (1, 1)], [(37.4, -122.1)] * 2,
              [(37.789437, -122.454643)] * 3, ring + [ring[0]]]
    # many vertices: several passes of the lanes over the edges and fan terms,
    # both orientations
    for k in (63, 64, 65, 129, 200):
        th = np.linspace(0, 2 * np.pi, k, endpoint=False)
        pts = [(float(10 + 0.05 * np.sin(t)), float(20 + 0.05 * np.cos(t))) for t in th]
        polys += [pts, pts[::-1]]
    olat, olng = _origin_latlng()
    circles = []
    for r_m in (80.0, 1500.0, 30000.0):
        for f in (0.0, 0.5, 0.999, 1.001, 2.0):
            circles.append((*_offset(olat, olng, f * r_m / 6371010.0, 1.3), r_m))
            ring_pts = [_offset(olat, olng, r_m / 6371010.0, 2 * np.pi * i / 7) for i in range(7)]
            polys += [ring_pts, ring_pts[::-1]]
    circles += [(89.9999, 0.0, 2000.0), (-89.9999, 10.0, 2000.0), (0.0, 179.9999, 5000.0), (45.0, 7.0, 400000.0),
                (91.0, 0.0, 100.0), (10.0, 10.0, 0.0)]
    st = _check(oracle, *_flat(polys, circles))
    assert (st == 0).sum() > len(st) // 2
    assert len(set(st.tolist())) >= 3  # ok, bad coordinates, too few points / area


def test_exact_setup_metro_seeds(exact_setup, oracle):
    from dss_amd import workload as W
    for seed in (0, 1):
        fp = W.metro_footprints(np.random.default_rng(1000 + seed), 20000)
        _check(oracle, fp.kind, fp.voff, fp.lat, fp.lng, fp.radius_m)


@pytest.mark.parametrize("slot_order", [1, 0])
def test_cover_slot_order(oracle, slot_order):
    """The general pipeline gives the oracle's coverings with its vertex
    slots polygons-first (k_setup's footprint order) or in footprint order
    ("cover_slot_order")."""
    from dss_amd import _lib
    from dss_amd import workload as W
    from test_gpu_cover_general import _base_footprints
    ctx = _lib.context(0)
    ctx.set_tuning("cover_wave", 0)
    ctx.set_tuning("cover_slot_order", slot_order)
    try:
        _, q, _, _, _, _ = W.config(2, scale=0.002)
        _check(oracle, q.kind, q.voff, q.lat, q.lng, q.radius_m)
        _check(oracle, *_flat(_base_footprints(np.random.default_rng(3))))
    finally:
        ctx.set_tuning("cover_slot_order", SLOT_ORDER_DEFAULT)
        ctx.set_tuning("cover_wave", COVER_WAVE_DEFAULT)
