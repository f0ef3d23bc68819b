"""The reference's prober scenarios end to end on the GPU path: request JSON
-> proto -> model (dss_amd/proto.py) -> UnionVolumes4D / covering on the GPU
-> the GPU write path (MutableOperationStore.UpsertOperation, whose conflict
search is the GPU join) -> SearchOperations on the GPU.  Expected outcomes
are the ones the prober asserts against a live DSS:

  * monitoring/prober/scd/test_operation_simple.py:18,112-165 -- op circle
    (-56, 178) r = 50 m, 60 min; found by the r = 300 m query with no time
    bounds, earliest now+59 min / latest now+1 min; not found with earliest
    now+61 min or latest now-1 min;
  * monitoring/prober/scd/test_operations_simple.py:32,47,264-300 -- near-pole
    circles (90, 0) and (89.999, 0), r = 200 m, both found by the circle
    (89.999, 180) r = 300 m;
  * monitoring/prober/scd/test_operation_special_cases.py with
    resources/op_request_{1,2,3}.json -- the 5-extent request is accepted
    (200), the 10-degree polygon is rejected by the covering (400), the
    degenerate 3-vertex polygon query succeeds (200) as a one-cell polyline.
The JSON fixtures are read from tests/golden/prober_requests.json (copied
request data; /root/reference is not on the GPU box)."""
import json
import os
import re

import pytest

pytestmark = pytest.mark.gpu

HERE = os.path.dirname(os.path.abspath(__file__))
MIN_US = 60 * 1_000_000
NOW = 1_800_000_000_000_000  # a fixed "utcnow" (us)


def rfc3339_us(s: str) -> int:
    """RFC3339 'YYYY-MM-DDTHH:MM:SS[.frac]Z' -> unix microseconds."""
    import calendar
    m = re.fullmatch(r"(\d{4})-(\d\d)-(\d\d)T(\d\d):(\d\d):(\d\d)(?:\.(\d+))?Z", s)
    assert m, s
    y, mo, d, h, mi, se = (int(x) for x in m.groups()[:6])
    frac = (m.group(7) or "0")[:6].ljust(6, "0")
    return calendar.timegm((y, mo, d, h, mi, se)) * 1_000_000 + int(frac)


def vol4_json(vol4: dict) -> dict:
    """A prober JSON Volume4D with its RFC3339 times as the proto's us values."""
    out = dict(vol4)
    for k in ("time_start", "time_end"):
        if k in vol4:
            out[k] = {"value": rfc3339_us(vol4[k]["value"])}
    return out


def circle(lat, lng, r):
    return {"center": {"lat": lat, "lng": lng}, "radius": {"value": r, "units": "M"}}


def vol4(t0, t1, a0, a1, c):
    v = {"volume": {"outline_circle": c, "altitude_lower": {"value": a0}, "altitude_upper": {"value": a1}}}
    if t0 is not None:
        v["time_start"] = {"value": t0}
    if t1 is not None:
        v["time_end"] = {"value": t1}
    return v


def put_op(store, op_id, extents, owner="uss1", key=()):
    """operations_handler.go PutOperationReference's model steps: every
    extent -> Volume4D, UnionVolumes4D, the union's covering, then
    UpsertOperation (conflict search + write on the GPU)."""
    from dss_amd import geo, proto, store as S
    vols = [proto.Volume4DFromSCDProto(e) for e in extents]
    (u,) = geo.UnionVolumes4DBatch([vols])
    if isinstance(u, geo.GeoError):
        raise u
    cells = u.CalculateSpatialCovering()
    sv = u.SpatialVolume
    op = S.Operation(op_id, owner, cells, sv.AltitudeLo, sv.AltitudeHi, u.StartTime, u.EndTime)
    return store.UpsertOperation(op, list(key), NOW, "2027-01-15T08:00:00Z")


def query(store, area):
    """operations_handler.go SearchOperationReferences: the area's covering,
    then SearchOperations (now = NOW)."""
    from dss_amd import proto
    v = proto.Volume4DFromSCDProto(area)
    cells = v.CalculateSpatialCovering()
    sv = v.SpatialVolume
    return {o.ID for o in store.SearchOperations(cells, sv.AltitudeLo, sv.AltitudeHi, v.StartTime, v.EndTime, NOW)}


def test_operation_simple_time_window_pins():
    from dss_amd import store as S
    st = S.MutableOperationStore()
    put_op(st, "op1", [vol4(NOW, NOW + 60 * MIN_US, 0, 120, circle(-56, 178, 50))])
    q = lambda t0, t1: query(st, vol4(t0, t1, 0, 5000, circle(-56, 178, 300)))  # noqa: E731
    assert q(None, None) == {"op1"}                       # test_get_op_by_search
    assert q(NOW + 59 * MIN_US, None) == {"op1"}          # earliest_time_included
    assert q(NOW + 61 * MIN_US, None) == set()            # earliest_time_excluded
    assert q(None, NOW + 1 * MIN_US) == {"op1"}           # latest_time_included
    assert q(None, NOW - 1 * MIN_US) == set()             # latest_time_excluded
    assert q(NOW, NOW) == {"op1"}                         # test_op_does_not_exist_query's volume, op present


def test_operations_simple_near_pole_pins():
    from dss_amd import store as S
    st = S.MutableOperationStore()
    put_op(st, "op1", [vol4(NOW, NOW + 60 * MIN_US, 0, 120, circle(90, 0, 200))], owner="uss1")
    # op2 overlaps op1: without op1's OVN the write is a conflict (409)
    with pytest.raises(S.MissingOVNs) as e:
        put_op(st, "op2", [vol4(NOW, NOW + 60 * MIN_US, 0, 120, circle(89.999, 0, 200))], owner="uss2")
    assert e.value.missing == ["op1"]
    put_op(st, "op2", [vol4(NOW, NOW + 60 * MIN_US, 0, 120, circle(89.999, 0, 200))], owner="uss2",
           key=[st.ops["op1"].OVN])
    assert query(st, vol4(NOW, NOW, 0, 5000, circle(89.999, 180, 300))) == {"op1", "op2"}


def _requests():
    with open(os.path.join(HERE, "golden", "prober_requests.json")) as f:
        return json.load(f)


def test_op_request_1_five_extents_accepted(oracle):
    from dss_amd import geo, proto, store as S
    req = _requests()["op_request_1"]
    extents = [vol4_json(e) for e in req["extents"]]
    assert len(extents) == 5
    st = S.MutableOperationStore()
    op = put_op(st, "2df6b920-b6ee-4082-b6e7-75eb4fde25d1", extents)
    # the union's cells == the union of the oracle's per-extent coverings
    want = set()
    for e in extents:
        vs = e["volume"]["outline_polygon"]["vertices"]
        rc, cells, _ = oracle.polygon_covering([v["lat"] for v in vs], [v["lng"] for v in vs])
        assert rc == 0
        want |= {int(c) for c in cells}
    assert sorted(want) == sorted(op.Cells)
    assert op.StartTime == min(rfc3339_us(e["time_start"]["value"]) for e in req["extents"])
    assert op.EndTime == max(rfc3339_us(e["time_end"]["value"]) for e in req["extents"])
    # visible to a search over its own union volume, then deleted (200, 200)
    u = geo.UnionVolumes4DBatch([[proto.Volume4DFromSCDProto(e) for e in extents]])[0]
    sv = u.SpatialVolume
    found = st.SearchOperations(op.Cells, sv.AltitudeLo, sv.AltitudeHi, None, None, 0)
    assert [o.ID for o in found] == [op.ID]
    st.DeleteOperation(op.ID, "uss1")
    assert st.SearchOperations(op.Cells, sv.AltitudeLo, sv.AltitudeHi, None, None, 0) == []


def test_op_request_2_rejected_by_the_covering(oracle):
    from dss_amd import geo, proto, store as S
    req = _requests()["op_request_2"]
    extents = [vol4_json(e) for e in req["extents"]]
    with pytest.raises(geo.GeoError) as e:
        put_op(S.MutableOperationStore(), "op", extents)
    vs = extents[0]["volume"]["outline_polygon"]["vertices"]
    rc, _, _ = oracle.polygon_covering([v["lat"] for v in vs], [v["lng"] for v in vs])
    assert rc != 0 and type(e.value) is type(geo.error_for_status(_status_of(oracle, rc), 1.0))
    # the same through the single-volume model path
    with pytest.raises(geo.GeoError):
        proto.Volume4DFromSCDProto(extents[0]).CalculateSpatialCovering()


def _status_of(oracle, rc):
    return {oracle.ERR_BAD_COORD_SET: 1, oracle.ERR_NOT_ENOUGH_POINTS: 2, oracle.ERR_RADIUS: 4,
            oracle.ERR_AREA_TOO_LARGE: 5}[rc]


def test_op_request_3_degenerate_polygon_query(oracle):
    from dss_amd import store as S
    req = _requests()["op_request_3"]
    area = vol4_json(req["area_of_interest"])
    vs = area["volume"]["outline_polygon"]["vertices"]
    lat, lng = vs[0]["lat"], vs[0]["lng"]
    from dss_amd import proto
    cells = proto.Volume4DFromSCDProto(area).CalculateSpatialCovering()
    assert cells == [oracle.cellid_from_degrees(lat, lng, 13)]
    # 200: the query runs; an op over that cell inside the window is found
    st = S.MutableOperationStore()
    t0 = rfc3339_us(req["area_of_interest"]["time_start"]["value"])
    put_op(st, "op", [vol4(t0, t0 + 10 * MIN_US, 0, 500, circle(lat, lng, 30))])
    v = proto.Volume4DFromSCDProto(area)
    found = st.SearchOperations(cells, v.SpatialVolume.AltitudeLo, v.SpatialVolume.AltitudeHi, v.StartTime, v.EndTime,
                                t0)
    assert [o.ID for o in found] == ["op"]
