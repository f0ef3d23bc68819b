"""GPU parity of the covering's wave path (k_cover_wave: one wavefront per
footprint, loop staged in LDS) against the general pipeline and the oracle.

The wave path must give, footprint for footprint, exactly what the general
per-thread pipeline gives (status, loopAreaKm2 bits, level-13 cell list), and
both must equal the CPU restatement of golang/geo (oracle/).  Footprints the
wave path cannot decide are covered by the general pipeline inside the same
call; the batches here mix both kinds."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def _both_paths(fp):
    from dss_amd import _lib, geo
    ctx = _lib.context(0)
    ctx.set_tuning("cover_wave", 1 << 40)  # every batch through the wave path
    try:
        wave = geo.cover_batch(fp.kind, fp.voff, fp.lat, fp.lng, fp.radius_m)
        ctx.set_tuning("cover_wave", 0)
        gen = geo.cover_batch(fp.kind, fp.voff, fp.lat, fp.lng, fp.radius_m)
    finally:
        ctx.set_tuning("cover_wave", COVER_WAVE_DEFAULT)
    return wave, gen


COVER_WAVE_DEFAULT = 16384  # CoverEngine::wave_max_


def _same(a, b):
    assert np.array_equal(a.status, b.status)
    assert np.array_equal(a.area_km2.view(np.uint64), b.area_km2.view(np.uint64))
    assert np.array_equal(a.offs, b.offs)
    assert np.array_equal(a.cells, b.cells)


@pytest.mark.parametrize("cfg,scale", [(0, 0.05), (1, 0.002), (2, 0.0002), (3, 0.0004), (4, 0.0002)])
def test_wave_path_equals_general_and_oracle(cfg, scale, oracle):
    from dss_amd import workload as W
    _, q, _, it, _, _ = W.config(cfg, scale=scale)
    for fp in (q, it):
        wave, gen = _both_paths(fp)
        _same(wave, gen)
    # the oracle on the query batch
    o_offs, o_cells, o_st, o_area = oracle.cover_batch(q.kind, q.voff, q.lat, q.lng, q.radius_m)
    wave, _ = _both_paths(q)
    assert np.array_equal(wave.offs, o_offs) and np.array_equal(wave.cells, o_cells)
    assert np.array_equal(wave.status, o_st)
    assert np.array_equal(wave.area_km2.view(np.uint64), np.asarray(o_area, np.float64).view(np.uint64))


def test_wave_path_on_golden_fixtures(golden_covering):
    from types import SimpleNamespace
    g = golden_covering
    fp = SimpleNamespace(kind=g["kind"], voff=g["voff"], lat=g["lat"], lng=g["lng"], radius_m=g["radius_m"])
    wave, gen = _both_paths(fp)
    _same(wave, gen)
    assert np.array_equal(wave.offs, g["offs"]) and np.array_equal(wave.cells, g["cells"])
    assert np.array_equal(wave.status, g["status"])


def test_wave_path_reversal_and_errors(oracle):
    """Clockwise rings (Q4 reversal through the reversed fan terms), rings
    over the area cap, bad coordinates, too few points, repeated vertices
    (polyline: general path), big circles (general path), in one batch."""
    from types import SimpleNamespace
    ring = [(37.40, -122.10), (37.41, -122.10), (37.41, -122.08), (37.40, -122.08)]
    polys = [ring, ring[::-1], [(-23, 130), (-24, 130), (-24, 132), (-23, 132)],
             [(-23, 130), (-23, 132), (-24, 132), (-24, 130)], [(91, 0), (0, 0), (1, 1)], [(37.4, -122.1)] * 2,
             [(37.789437, -122.454643)] * 3, ring + [ring[0]]]
    kinds, voff, lat, lng, rad = [], [0], [], [], []
    for pts in polys:
        kinds.append(0)
        lat += [a for a, _ in pts]
        lng += [b for _, b in pts]
        voff.append(len(lat))
        rad.append(0.0)
    # (0, 0, 3.3e6 m): 0.52 rad, not a small loop (general path); ~30M cells, past the oracle's
    # 2^24-cell limit, so it is compared wave path vs general path only
    for la, ln, r in ((37.4, -122.1, 300.0), (89.999, 180.0, 300.0), (-56, 178, 50.0), (0, 0, 3.3e6),
                      (37.4, -122.1, 0.0), (12.0, -34.0, 300.0), (0, 0, 1.0e6)):
        kinds.append(1)
        lat.append(la)
        lng.append(ln)
        voff.append(len(lat))
        rad.append(r)
    fp = SimpleNamespace(kind=np.array(kinds, np.int32), voff=np.array(voff, np.int64), lat=np.array(lat),
                         lng=np.array(lng), radius_m=np.array(rad, np.float32))
    wave, gen = _both_paths(fp)
    _same(wave, gen)
    big = len(polys) + 3
    keep = np.array([i for i in range(len(kinds)) if i != big])
    sub = SimpleNamespace(kind=fp.kind[keep], voff=np.concatenate([[0], np.cumsum(np.diff(fp.voff)[keep])]),
                          lat=np.concatenate([fp.lat[fp.voff[i]:fp.voff[i + 1]] for i in keep]),
                          lng=np.concatenate([fp.lng[fp.voff[i]:fp.voff[i + 1]] for i in keep]),
                          radius_m=fp.radius_m[keep])
    wave, _ = _both_paths(sub)
    o_offs, o_cells, o_st, o_area = oracle.cover_batch(sub.kind, sub.voff, sub.lat, sub.lng, sub.radius_m)
    assert np.array_equal(wave.status, o_st)
    assert np.array_equal(wave.offs, o_offs) and np.array_equal(wave.cells, o_cells)
    assert np.array_equal(wave.area_km2.view(np.uint64), np.asarray(o_area, np.float64).view(np.uint64))
