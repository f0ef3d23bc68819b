"""GPU: the explicit geometries and outcomes of the reference's own tests,
taken through the GPU covering and the GPU search together (not only the
covering): every assertion below restates one the reference makes.

  * pkg/geo/s2_test.go:12-52 -- AreaToCellIDs successes and failures; the
    successful areas, stored as ISAs, are found by a search with their own
    cells and by one with testdata.Loop where they overlap it;
  * pkg/rid/server/server_test.go:35-41, 589-593 -- mustPolygonToCellIDs(
    testdata.LoopPolygon) (GeoPolygonFromRIDProto(...).CalculateCovering) and
    TestDefaultRegionCovererProducesResults (AreaToCellIDs(testdata.Loop)):
    the same 20 cells, and SearchIdentificationServiceAreas with Area =
    testdata.Loop finds the ISA stored over that polygon;
  * pkg/rid/application/isa_test.go:77-134 (TestISAUpdateIdxCells) -- an ISA
    over three sibling cells is updated to the fourth: the fan-out covers
    CellUnionFromUnion(old, new) re-levelled (four level-13 cells, not their
    parent), both subscriptions are notified once (index 1) and the search by
    the new cells finds the ISA.
"""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu

LOOP = "37.427636,-122.170502,37.408799,-122.064069,37.421265,-122.086504"  # pkg/geo/testdata
LOOP_LAT = [37.427636, 37.408799, 37.421265]
LOOP_LNG = [-122.170502, -122.064069, -122.086504]
T0 = 1_600_000_000_000_000
HOUR = 3_600_000_000

S2_OK = ["37.4047,-122.1474,37.4037,-122.1485,37.4035,-122.1466",                  # s2_test.go:12-16
         "0.000,0.000, 0.000,0.005, -0.005,0.0025",                                 # :18-22 opposite winding
         "37.4047,-122.1474,37.4037,-122.1485,37.4035,-122.1466,37.4035,-122.1466",  # :24-28 even count
         LOOP]                                                                       # :30-34
S2_FAIL = ["", "37.427636,-122.170502,37.408799,-122.064069", "37.427636,-122.170502,37.408799"]  # :36-52


def test_s2_test_areas_through_cover_and_search(oracle):
    from dss_amd import geo
    from dss_amd.store import EntityIndex, SearchISAs
    for area in S2_FAIL:
        with pytest.raises(geo.GeoError):
            geo.AreaToCellIDs(area)
    covers = [geo.AreaToCellIDs(a) for a in S2_OK]
    assert all(len(c) > 0 for c in covers)
    # each area stored as an ISA (RID: no altitude), searched with its own
    # cells and with testdata.Loop's
    idx = EntityIndex.from_lists(covers, t0=[T0] * len(covers), t1=[T0 + HOUR] * len(covers))
    loop_cells = geo.AreaToCellIDs(LOOP)
    io = np.concatenate([[0], np.cumsum([len(c) for c in covers])]).astype(np.int64)
    ic = np.concatenate([np.asarray(c, np.uint64) for c in covers])
    for k, c in enumerate(covers):
        got = SearchISAs(idx, c, T0, None)
        assert k in got
        want = [e for e in range(len(covers)) if np.intersect1d(covers[e], c).size]
        assert sorted(got) == want
    got = SearchISAs(idx, loop_cells, T0, None)
    oq, oe = oracle.search(io, ic, np.full(len(covers), -np.inf, np.float32), np.full(len(covers), np.inf, np.float32),
                           np.full(len(covers), T0), np.full(len(covers), T0 + HOUR), None,
                           np.array([0, len(loop_cells)]), np.asarray(loop_cells, np.uint64), np.array([-np.inf], np.float32),
                           np.array([np.inf], np.float32), np.array([T0]), np.array([np.iinfo(np.int64).max]))
    assert sorted(got) == sorted(int(e) for e in oe) and 3 in got


def test_rid_server_loop_polygon_and_search():
    from dss_amd import geo
    from dss_amd.store import AppSearchISAs, EntityIndex
    poly = geo.GeoPolygon([geo.LatLngPoint(a, b) for a, b in zip(LOOP_LAT, LOOP_LNG)]).CalculateCovering()
    area = geo.AreaToCellIDs(LOOP)
    assert poly == area and len(poly) == 20
    # the stored ISA over mustPolygonToCellIDs(LoopPolygon), and one far away
    far = geo.GeoPolygon([geo.LatLngPoint(40.70, -74.00), geo.LatLngPoint(40.71, -74.00),
                          geo.LatLngPoint(40.71, -74.01)]).CalculateCovering()
    idx = EntityIndex.from_lists([poly, far], t0=[T0, T0], t1=[T0 + HOUR, T0 + HOUR])
    # SearchIdentificationServiceAreas(Area: testdata.Loop), earliest/latest nil
    assert AppSearchISAs(idx, area, None, None, now_us=T0 + 1) == [0]
    assert AppSearchISAs(idx, area, None, None, now_us=T0 + 2 * HOUR) == []  # expired


def test_isa_update_idx_cells():
    from dss_amd import geo
    from dss_amd.store import SearchISAs, Store, UpdateNotificationIdxsInCells, EntityIndex
    a, b, c, d = 17106221850767130624, 17106221885126868992, 17106221919486607360, 17106221953846345728
    # the four are siblings: CellUnionFromUnion normalises their union to the
    # parent, Levelify expands it back to the four level-13 cells
    parent_lsb = 1 << 36
    parent = (a & ~((parent_lsb << 1) - 1)) | parent_lsb
    assert geo.Levelify([parent]) == [a, b, c, d]
    now = T0
    subs = [[a, c], [d]]  # isa_test.go:104-122
    sidx = EntityIndex.from_lists(subs, t0=[now, now], t1=[now + HOUR, now + HOUR])
    sidx.set_notification_index([0, 0])
    # InsertISA(update): UpdateNotificationIdxsInCells(Levelify(union(old, new)))
    cells = geo.Levelify([parent])
    rows = UpdateNotificationIdxsInCells(sidx, cells, now)
    assert sorted(rows) == [(0, 1), (1, 1)]  # require.Len(subs, 2); NotificationIndex == 1
    # the ISA table after the update: the ISA holds {d}
    st = Store()
    st.upsert([7], [[a, b, c]], [-np.inf], [np.inf], [now], [now + HOUR])
    st.upsert([7], [[d]], [-np.inf], [np.inf], [now], [now + HOUR])
    q, e = st.search_batch([0, 1], [d], [-np.inf], [np.inf], [now], [np.iinfo(np.int64).max])
    assert e.tolist() == [7]  # isas, err := app.SearchISAs(ctx, isa.Cells, &startTime, nil); Len 1
    q, e = st.search_batch([0, 1], [a], [-np.inf], [np.inf], [now], [np.iinfo(np.int64).max])
    assert e.tolist() == []  # the old cells no longer hold it
    st.free()
    assert SearchISAs(EntityIndex.from_lists([[d]], t0=[now], t1=[now + HOUR]), [d], now, None) == [0]
