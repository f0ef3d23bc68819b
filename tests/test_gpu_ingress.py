"""GPU batched ingress: models.UnionVolumes4D (pkg/models/geo.go:126-190) for
a batch of multi-extent requests (dssg_union_volumes_device) against the
oracle: every extent covered by the CPU restatement, the union / min / max /
first-error logic restated from the Go source below."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def _expected(oracle, req):
    """UnionVolumes4D restated over oracle coverings: (error status, cells,
    lo, hi, start, end) -- NULLs as None."""
    from dss_amd import _lib, geo
    cells, lo, hi, s, e = set(), None, None, None, None
    for v in req:
        if v.EndTime is not None:
            e = v.EndTime if e is None else max(e, v.EndTime)
        if v.StartTime is not None:
            s = v.StartTime if s is None else min(s, v.StartTime)
        sv = v.SpatialVolume
        if sv is None:
            continue
        if sv.AltitudeLo is not None:
            lo = np.float32(sv.AltitudeLo) if lo is None else min(lo, np.float32(sv.AltitudeLo))
        if sv.AltitudeHi is not None:
            hi = np.float32(sv.AltitudeHi) if hi is None else max(hi, np.float32(sv.AltitudeHi))
        fp = sv.Footprint
        if fp is None:
            continue
        if isinstance(fp, geo.GeoCircle):
            o, c, st, ar = oracle.cover_batch([_lib.KIND_CIRCLE], [0, 1], [fp.Center.Lat], [fp.Center.Lng],
                                              [np.float32(fp.RadiusMeter)])
        else:
            n = len(fp.Vertices)
            o, c, st, ar = oracle.cover_batch([_lib.KIND_POLYGON], [0, n], [p.Lat for p in fp.Vertices],
                                              [p.Lng for p in fp.Vertices], [0.0])
        if st[0] != 0:
            return int(st[0]), None, None, None, None, None
        cells |= set(int(x) for x in c)
    return 0, cells, lo, hi, s, e


def _random_requests(rng, n):
    from dss_amd import geo
    T = 1_700_000_000_000_000
    reqs = []
    for i in range(n):
        req = []
        for _ in range(rng.integers(1, 5)):
            clat, clng = rng.uniform(37.3, 37.8), rng.uniform(-122.5, -121.9)
            r = rng.random()
            if r < 0.45:
                k = rng.integers(3, 9)
                ang = np.sort(rng.uniform(0, 2 * np.pi, k))
                rad = rng.uniform(0.002, 0.03)
                fp = geo.GeoPolygon([geo.LatLngPoint(clat + rad * np.sin(a), clng + rad * np.cos(a)) for a in ang])
            elif r < 0.8:
                fp = geo.GeoCircle(geo.LatLngPoint(clat, clng), float(rng.uniform(50, 2000)))
            elif r < 0.9:
                fp = None
            elif r < 0.94:   # huge box: ErrAreaTooLarge
                fp = geo.GeoPolygon([geo.LatLngPoint(clat, clng), geo.LatLngPoint(clat + 1, clng),
                                     geo.LatLngPoint(clat + 1, clng + 2), geo.LatLngPoint(clat, clng + 2)])
            elif r < 0.97:   # errBadCoordSet
                fp = geo.GeoPolygon([geo.LatLngPoint(91, clng), geo.LatLngPoint(clat, clng),
                                     geo.LatLngPoint(clat, clng + 0.01)])
            else:            # errNotEnoughPointsInPolygon
                fp = geo.GeoPolygon([geo.LatLngPoint(clat, clng), geo.LatLngPoint(clat, clng + 0.01)])
            sv = None if rng.random() < 0.05 else geo.Volume3D(
                AltitudeLo=None if rng.random() < 0.2 else float(rng.uniform(0, 300)),
                AltitudeHi=None if rng.random() < 0.2 else float(rng.uniform(300, 600)), Footprint=fp)
            st = None if rng.random() < 0.15 else int(T + rng.integers(0, 10**9))
            en = None if rng.random() < 0.15 else int(T + rng.integers(10**9, 2 * 10**9))
            req.append(geo.Volume4D(SpatialVolume=sv, StartTime=st, EndTime=en))
        reqs.append(req)
    return reqs


def test_union_volumes_batch_against_oracle(oracle):
    from dss_amd import geo
    rng = np.random.default_rng(21)
    reqs = _random_requests(rng, 400)
    got = geo.UnionVolumes4DBatch(reqs)
    n_err = 0
    for req, g in zip(reqs, got):
        st, cells, lo, hi, s, e = _expected(oracle, req)
        if st != 0:
            n_err += 1
            assert isinstance(g, geo.GeoError) and type(g) is type(geo.error_for_status(st, 1.0)), (st, g)
            continue
        assert not isinstance(g, geo.GeoError), g
        assert g.StartTime == s and g.EndTime == e
        if g.SpatialVolume is None:
            assert all(v.SpatialVolume is None for v in req)
            continue
        assert g.SpatialVolume.AltitudeLo == (None if lo is None else float(lo))
        assert g.SpatialVolume.AltitudeHi == (None if hi is None else float(hi))
        fp = g.SpatialVolume.Footprint
        assert (fp is None) == (not any(v.SpatialVolume is not None and v.SpatialVolume.Footprint is not None
                                        for v in req))
        if fp is not None:
            assert set(fp.keys()) == cells
    assert n_err > 0


def test_union_matches_host_mirror():
    """The device batch and the host mirror geo.UnionVolumes4D agree."""
    from dss_amd import geo
    rng = np.random.default_rng(5)
    for req, g in zip(reqs := _random_requests(rng, 60), geo.UnionVolumes4DBatch(reqs)):
        try:
            h = geo.UnionVolumes4D(*req)
        except geo.GeoError as err:
            assert isinstance(g, geo.GeoError) and type(g) is type(err)
            continue
        assert g.StartTime == h.StartTime and g.EndTime == h.EndTime
        if h.SpatialVolume is not None and h.SpatialVolume.Footprint is not None:
            assert set(g.SpatialVolume.Footprint.keys()) == set(h.SpatialVolume.Footprint.keys())


def test_union_null_altitude_feeds_search(oracle):
    """A union volume whose extents carry no altitude comes back with the
    search's NULL sentinels (-INF / +INF), so passing dssg_volumes straight to
    a search matches like the reference's COALESCE(..., true)
    (pkg/scd/store/cockroach/operations.go:394-397)."""
    import ctypes as C
    import torch
    from dss_amd import _lib, device as D
    from dss_amd.store import EntityIndex
    ctx = _lib.context()
    dev = "cuda:0"
    # one volume: a circle with no altitude bounds and no times
    t = lambda a, dt: torch.as_tensor(np.asarray(a, dtype=dt), device=dev)  # noqa: E731
    bufs = [t([0, 1], np.int64), t([_lib.KIND_CIRCLE], np.int32), t([0, 1], np.int64), t([37.5], np.float64),
            t([-122.2], np.float64), t([300.0], np.float32), t([1], np.uint8), t([np.nan], np.float32),
            t([np.nan], np.float32), t([_lib.TIME_NULL_START], np.int64), t([_lib.TIME_NULL_END_Q], np.int64)]
    out = _lib.Volumes()
    ctx.check(ctx.L.dssg_union_volumes_device(ctx.h, 1, *[D._ptr(b) for b in bufs], D._stream_ptr(), C.byref(out)))
    offs = D.copy_back(ctx, out.offs, 2, np.int64)
    cells = D.copy_back(ctx, out.cells, int(offs[-1]), np.uint64)
    lo = D.copy_back(ctx, out.alt_lo, 1, np.float32)
    hi = D.copy_back(ctx, out.alt_hi, 1, np.float32)
    assert lo[0] == -np.inf and hi[0] == np.inf
    # an operation in the same place, 1000-1100 m, now .. now + 1 h
    now = 1_600_000_000_000_000
    rc, e_cells = oracle.circle_covering(37.5, -122.2, 100.0)
    idx = EntityIndex(np.array([0, len(e_cells)], np.int64), np.asarray(e_cells, np.uint64),
                      np.array([1000.0], np.float32), np.array([1100.0], np.float32), np.array([now], np.int64),
                      np.array([now + 3_600_000_000], np.int64))
    rq, re = idx.search_operations_batch(offs, cells, lo, hi, [_lib.TIME_NULL_START], [_lib.TIME_NULL_END_Q], now)
    assert list(rq) == [0] and list(re) == [0]
