"""CPU: the oracle against the reference's own known-answer tests.

Pins the covering restatement on pkg/models/geo_test.go:10-55 (exact 20-cell
KAT) and the status-level cases of pkg/geo/s2_test.go:12-52 and the prober.
"""
import math
import re

import numpy as np
import pytest

KAT_TOKENS = ("808fb0ac 808fb744 808fb754 808fb75c 808fb9fc 808fba04 808fba0c 808fba14 808fba1c 808fba5c "
              "808fba64 808fba6c 808fba74 808fba8c 808fbad4 808fbadc 808fbae4 808fbaec 808fbaf4 808fbb2c").split()


_GO_FLOAT = re.compile(r"[+-]?(?:(?:\d+\.?\d*|\.\d+)(?:[eE][+-]?\d+)?"
                       r"|0[xX](?:[0-9a-fA-F]+\.?[0-9a-fA-F]*|\.[0-9a-fA-F]+)[pP][+-]?\d+"
                       r"|[iI][nN][fF](?:[iI][nN][iI][tT][yY])?|[nN][aA][nN])")


def go_split_at_comma(area: str):
    """bufio.Scanner with pkg/geo/s2.go:68-82 splitAtComma: tokens between
    commas; at EOF the rest is one more token unless it is empty (so a
    trailing comma yields no empty final token)."""
    toks, pos = [], 0
    while True:
        if pos == len(area):  # atEOF && len(data) == 0
            return toks
        i = area.find(",", pos)
        if i < 0:
            toks.append(area[pos:])
            return toks
        toks.append(area[pos:i])
        pos = i + 1


def go_parse_float(tok: str):
    """strconv.ParseFloat(tok, 64) acceptance (Go syntax: decimal, hex with a
    p exponent, inf/infinity/nan; no underscores without a base prefix);
    None = error."""
    if not _GO_FLOAT.fullmatch(tok):
        return None
    if "x" in tok or "X" in tok:
        return float.fromhex(tok)
    return float(tok)


def area_to_cell_ids(O, area: str):
    """pkg/geo/s2.go:129-166 restated on top of the oracle's Covering: the
    comma count decides odd / not-enough first, then every token parses
    (TrimSpace, ParseFloat) and each (lat, lng) pair becomes a point; a
    trailing lone latitude is dropped."""
    num = area.count(",") + 1
    if num % 2 == 1:
        return O.ERR_ODD_COORDS, None
    if num // 2 < 3:
        return O.ERR_NOT_ENOUGH_POINTS, None
    vals = []
    for tok in go_split_at_comma(area):
        v = go_parse_float(tok.strip())
        if v is None:
            return O.ERR_BAD_COORD_SET, None
        vals.append(v)
    pts = [O.point_from_degrees(vals[i], vals[i + 1]) for i in range(0, len(vals) - 1, 2)]
    rc, cells, _ = O.covering_xyz(np.array(pts))
    return rc, cells


def test_go_split_at_comma():
    assert go_split_at_comma("1,2,3") == ["1", "2", "3"]
    assert go_split_at_comma("1,2,3,") == ["1", "2", "3"]
    assert go_split_at_comma(",1") == ["", "1"]
    assert go_split_at_comma("1,,2") == ["1", "", "2"]
    assert go_parse_float("1_000") is None and go_parse_float("0x1p-2") == 0.25 and go_parse_float("") is None


def test_polygon_covering_kat(oracle):
    # pkg/models/geo_test.go:10-55
    rc, cells, _ = oracle.polygon_covering([37.427636, 37.408799, 37.421265], [-122.170502, -122.064069, -122.086504])
    assert rc == oracle.OK
    assert [oracle.token(int(c)) for c in cells] == KAT_TOKENS


@pytest.mark.parametrize("area,ok", [
    ("37.4047,-122.1474,37.4037,-122.1485,37.4035,-122.1466", True),            # s2_test.go:12-16
    ("0.000,0.000, 0.000,0.005, -0.005,0.0025", True),                           # :18-22 (CW -> reversal)
    ("37.4047,-122.1474,37.4037,-122.1485,37.4035,-122.1466,37.4035,-122.1466", True),  # :24-28
    ("37.427636,-122.170502,37.408799,-122.064069,37.421265,-122.086504", True),  # :30-34 testdata.Loop
    ("", False),                                                                 # :36-40
    ("37.427636,-122.170502,37.408799,-122.064069", False),                     # :42-46 two points
    ("37.427636,-122.170502,37.408799", False),                                  # :48-52 odd coords
    # trailing comma: no empty final token (splitAtComma at EOF), so 7 tokens -> 3 points + a dropped lat
    ("37.4047,-122.1474,37.4037,-122.1485,37.4035,-122.1466,1,", True),
    ("37.4047,-122.1474,37.4037,-122.1485,37.4035,-122.1466,", False),           # 7 coords: odd
    (",37.4047,-122.1474,37.4037,-122.1485,37.4035", False),                    # empty first token
    ("37.4047,-122.1474,,37.4037,-122.1485,37.4035,-122.1466,1", False),       # empty middle token
    ("37.4047,-122.147_4,37.4037,-122.1485,37.4035,-122.1466", False),          # Go rejects underscores
])
def test_area_to_cell_ids_status(oracle, area, ok):
    rc, cells = area_to_cell_ids(oracle, area)
    assert (rc == oracle.OK) == ok
    if ok:
        assert cells is not None and len(cells) > 0


def test_area_too_large_prober_huge(oracle):
    # monitoring/prober/rid/common.py:29-49 HUGE polygon -> 413 (AreaTooLarge)
    rc, cells, area = oracle.polygon_covering([-23, -24, -24, -23], [130, 130, 132, 132])
    assert rc == oracle.ERR_AREA_TOO_LARGE
    # Q1 + Q4: the box (~2.27e4 km^2, pi^2-inflated to ~2.24e5) is over the cap
    # in its given order, so it is reversed, and the error reports the area of
    # the reversed loop -- its complement on the sphere.
    assert area > 5.0e9
    _, _, area2 = oracle.polygon_covering([-23, -23, -24, -24], [130, 132, 132, 130])
    assert 2.0e5 < area2 < 2.5e5


def test_degenerate_polygon_is_polyline(oracle):
    # op_request_3.json: three identical vertices -> zero area -> Polyline covering
    lat, lng = 37.78943798147498, -122.45464324951172
    rc, cells, area = oracle.polygon_covering([lat] * 3, [lng] * 3)
    assert rc == oracle.OK and area == 0.0
    assert [int(c) for c in cells] == [oracle.cellid_from_degrees(lat, lng, 13)]


def test_polygon_checks_coordinates_before_count(oracle):
    # Q17: pkg/models/geo.go:257-266
    rc, _, _ = oracle.polygon_covering([91.0, 0.0], [0.0, 0.0])
    assert rc == oracle.ERR_BAD_COORD_SET
    rc, _, _ = oracle.polygon_covering([90.0, 0.0], [180.0, 0.0])
    assert rc == oracle.ERR_NOT_ENOUGH_POINTS


def test_circle_status(oracle):
    assert oracle.circle_covering(0, 0, 0)[0] == oracle.ERR_RADIUS
    assert oracle.circle_covering(0, 0, float("nan"))[0] == oracle.ERR_RADIUS
    assert oracle.circle_covering(91, 0, 10)[0] == oracle.ERR_BAD_COORD_SET
    rc, cells = oracle.circle_covering(-56, 178, 50)   # scd/test_operation_simple.py:18
    assert rc == oracle.OK and len(cells) >= 1


def test_circle_overlap_pins(oracle):
    # scd/test_operation_simple.py: op circle r=50 m found by query r=300 m
    _, a = oracle.circle_covering(-56, 178, 50)
    _, b = oracle.circle_covering(-56, 178, 300)
    assert set(a.tolist()) <= set(b.tolist())
    # scd/test_subscription_simple.py:22,96
    _, c = oracle.circle_covering(12, -34, 300)
    _, d = oracle.circle_covering(12.00001, -34.00001, 50)
    assert set(c.tolist()) & set(d.tolist())


def test_go_math_close_to_libm(oracle):
    rng = np.random.default_rng(1)
    for x in rng.uniform(-7, 7, 200):
        for go, ref in ((oracle.lib().orc_go_sin, math.sin), (oracle.lib().orc_go_cos, math.cos),
                        (oracle.lib().orc_go_atan, math.atan)):
            assert abs(go(x) - ref(x)) <= 2 * math.ulp(ref(x)) + 1e-300
        y = rng.uniform(-3, 3)
        assert abs(oracle.lib().orc_go_atan2(y, x) - math.atan2(y, x)) <= 4e-16 * max(1, abs(math.atan2(y, x)))


def test_regular_loop_is_ccw_20gon(oracle):
    import ctypes as C
    xyz = np.zeros(60)
    oracle.lib().orc_regular_loop(37.0, -122.0, 1000.0, 20, xyz.ctypes.data_as(C.POINTER(C.c_double)))
    pts = xyz.reshape(20, 3)
    assert np.allclose(np.linalg.norm(pts, axis=1), 1.0, atol=1e-15)
    c = oracle.point_from_degrees(37.0, -122.0)
    d = np.arccos(np.clip(pts @ c, -1, 1)) * 6371010.0
    assert np.allclose(d, 1000.0, rtol=1e-6)  # arccos near 1 is ill-conditioned
    # counter-clockwise about the centre (the interior is the small cap)
    for k in range(20):
        a, b = pts[k] - c, pts[(k + 1) % 20] - c
        assert np.dot(np.cross(a, b), c) > 0


# ---- subscription-store KATs (pkg/rid/cockroach/subscriptions_test.go,
# pkg/rid/application/isa_test.go) pinned on the oracle restatements
POOL_CELL = 12494535935418957824
OVERFLOW_CELL = 17106221850767130624
# subscriptionsPool (subscriptions_test.go:19-64): owners myself, myself, me
POOL_CELLS = [[OVERFLOW_CELL, POOL_CELL], [POOL_CELL], [POOL_CELL]]
POOL_OWNER = [0, 0, 1]   # "myself" -> 0, "me" -> 1


def _pool_csr():
    import numpy as np
    offs = np.cumsum([0] + [len(c) for c in POOL_CELLS]).astype(np.int64)
    cells = np.array([c for cs in POOL_CELLS for c in cs], np.uint64)
    return offs, cells


def test_oracle_max_subscription_count_kat(oracle):
    # subscriptions_test.go:275-287: MaxSubscriptionCountInCellsByOwner({pool cell}, "myself") == 2
    import numpy as np
    offs, cells = _pool_csr()
    t1 = np.full(3, 10**15, np.int64)
    got = oracle.max_subscription_count(offs, cells, POOL_OWNER, t1, np.array([0, 1]), np.array([POOL_CELL], np.uint64),
                                        [0], 0)
    assert got.tolist() == [2]
    # repeats inside a stored array count each time (RID unnest(cells))
    got = oracle.max_subscription_count(np.array([0, 2]), np.array([POOL_CELL, POOL_CELL], np.uint64), [0], [10**15],
                                        np.array([0, 1]), np.array([POOL_CELL], np.uint64), [0], 0)
    assert got.tolist() == [2]


def test_oracle_notification_fanout_kat(oracle):
    # isa_test.go:266-324: subscriptions start at 42; inserting an ISA over the
    # pool cell notifies all three (43), deleting it notifies them again (44)
    import numpy as np
    offs, cells = _pool_csr()
    t1 = np.full(3, 10**15, np.int64)
    q_offs, q_cells = np.array([0, 1]), np.array([POOL_CELL], np.uint64)
    _, e, v, cnt = oracle.notify(offs, cells, t1, [42, 42, 42], q_offs, q_cells, 0)
    assert sorted(e.tolist()) == [0, 1, 2] and v.tolist() == [43, 43, 43]
    _, e, v, cnt = oracle.notify(offs, cells, t1, cnt, q_offs, q_cells, 0)
    assert v.tolist() == [44, 44, 44] and cnt.tolist() == [44, 44, 44]


def test_oracle_scd_subscription_search_ignores_cells(oracle):
    # quirk Q7 (pkg/scd/store/cockroach/subscriptions.go:497-545)
    q, e = oracle.owner_subscriptions([0, 1, 0, 0], [10, 10, 5, 10], [0], 8)
    assert e.tolist() == [0, 3]
