"""Proto -> model -> GPU covering, end to end (dss_amd/proto.py): Q16 radius
units, SCD / RID volumes and RID SetExtents, cells compared with the oracle."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu

KAT = [(37.427636, -122.170502), (37.408799, -122.064069), (37.421265, -122.086504)]


def test_q16_non_meter_radius_fails_the_covering():
    from dss_amd import geo, proto
    for units in ("FT", "KM", ""):
        v = proto.Volume4DFromSCDProto({"volume": {"outline_circle": {"center": {"lat": 37.4, "lng": -122.1},
                                                                      "radius": {"value": 300, "units": units}}}})
        with pytest.raises(geo.RadiusMustBeLargerThan0Error):
            v.CalculateSpatialCovering()


def test_scd_circle_and_polygon_cover_like_the_oracle(oracle):
    from dss_amd import proto
    v = proto.Volume4DFromSCDProto({"volume": {"outline_circle": {"center": {"lat": 37.4, "lng": -122.1},
                                                                  "radius": {"value": 300, "units": "M"}}}})
    rc, want = oracle.circle_covering(37.4, -122.1, 300.0)
    assert rc == 0 and v.CalculateSpatialCovering() == [int(c) for c in want]
    v = proto.Volume4DFromSCDProto({"volume": {"outline_polygon": {"vertices": [{"lat": a, "lng": b} for a, b in KAT]}}})
    rc, want, _ = oracle.polygon_covering([a for a, _ in KAT], [b for _, b in KAT])
    assert rc == 0 and v.CalculateSpatialCovering() == [int(c) for c in want] and len(want) == 20


def test_rid_set_extents_covers_the_footprint(oracle):
    from dss_amd import proto
    isa = proto.IdentificationServiceArea()
    isa.SetExtents({"time_start": 100, "time_end": 200,
                    "spatial_volume": {"altitude_lo": 10.0, "altitude_hi": 20.0,
                                       "footprint": {"vertices": [{"lat": a, "lng": b} for a, b in KAT]}}})
    rc, want, _ = oracle.polygon_covering([a for a, _ in KAT], [b for _, b in KAT])
    assert isa.Cells == [int(c) for c in want]
    assert (isa.StartTime, isa.EndTime, isa.AltitudeLo, isa.AltitudeHi) == (100, 200, 10.0, 20.0)
