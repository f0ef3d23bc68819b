"""Proto -> model conversion of the request volumes, as the reference does it
before any covering or search (the quirks the GPU path must see exactly):

  * SCD (pkg/models/geo.go:436-510): Volume4DFromSCDProto,
    Volume3DFromSCDProto, GeoCircleFromSCDProto, GeoPolygonFromSCDProto.
    Q8: a missing altitude_lower / altitude_upper is 0.0 (GetValue() of a nil
    message), not NULL.  Q16: the circle radius is
    unitToMeterMultiplicativeFactors[units] * value in float32, and the map
    holds only "M" -- any other unit gives radius 0, so the covering fails
    with errRadiusMustBeLargerThan0.
  * RID (pkg/models/geo.go:276-329): Volume4DFromRIDProto,
    Volume3DFromRIDProto (footprint required; altitudes proto.Float32 of the
    plain floats, i.e. 0.0 when absent).
  * RID IdentificationServiceArea.SetExtents
    (pkg/rid/models/identification_service_area.go:71-105): nil extents are a
    no-op; times copied; a missing spatial_volume or footprint is an error;
    the cells are the GPU covering of the footprint polygon.

Protos are plain dicts shaped like their JSON form (no protobuf runtime in
the image); timestamps are microseconds since the epoch.  The coverings run
on the GPU (geo.GeoPolygon / GeoCircle).
"""
from __future__ import annotations

from dataclasses import dataclass
from typing import List, Optional

import numpy as np

from . import geo

# pkg/models/geo.go:40-42 -- the only unit the reference knows
UNIT_TO_METER = {"M": np.float32(1.0)}


class ProtoError(ValueError):
    pass


def _f32(x) -> float:
    return float(np.float32(x))


def _value(msg: Optional[dict], default=0.0):
    """GetX().GetValue() on a wrapper message: its value, or the zero value
    when the message is absent."""
    if msg is None:
        return default
    return msg.get("value", default)


def LatLngPointFromSCDProto(p: dict) -> geo.LatLngPoint:
    return geo.LatLngPoint(float(p.get("lat", 0.0)), float(p.get("lng", 0.0)))


def GeoCircleFromSCDProto(c: dict) -> geo.GeoCircle:
    """pkg/models/geo.go:496-502 (Q16: unknown units -> factor 0)."""
    r = c.get("radius") or {}
    factor = UNIT_TO_METER.get(r.get("units", ""), np.float32(0.0))
    radius = np.float32(factor) * np.float32(r.get("value", 0.0))
    return geo.GeoCircle(LatLngPointFromSCDProto(c.get("center") or {}), float(radius))


def GeoPolygonFromSCDProto(p: dict) -> geo.GeoPolygon:
    return geo.GeoPolygon([LatLngPointFromSCDProto(v) for v in p.get("vertices", [])])


def Volume3DFromSCDProto(vol3: Optional[dict]) -> geo.Volume3D:
    """pkg/models/geo.go:468-490 (Q8: missing altitudes are 0.0)."""
    vol3 = vol3 or {}
    lo = _f32(_value(vol3.get("altitude_lower")))
    hi = _f32(_value(vol3.get("altitude_upper")))
    circle, polygon = vol3.get("outline_circle"), vol3.get("outline_polygon")
    if circle is not None and polygon is not None:
        raise ProtoError("both circle and polygon specified in outline geometry")
    if polygon is not None:
        return geo.Volume3D(AltitudeHi=hi, AltitudeLo=lo, Footprint=GeoPolygonFromSCDProto(polygon))
    if circle is not None:
        return geo.Volume3D(AltitudeHi=hi, AltitudeLo=lo, Footprint=GeoCircleFromSCDProto(circle))
    return geo.Volume3D(AltitudeHi=hi, AltitudeLo=lo)


def Volume4DFromSCDProto(vol4: dict) -> geo.Volume4D:
    """pkg/models/geo.go:436-466 (time_start / time_end are Time messages
    wrapping a timestamp)."""
    out = geo.Volume4D(SpatialVolume=Volume3DFromSCDProto(vol4.get("volume")))
    ts, te = vol4.get("time_start"), vol4.get("time_end")
    if ts is not None:
        out.StartTime = int(ts["value"])
    if te is not None:
        out.EndTime = int(te["value"])
    return out


def Volume3DFromRIDProto(vol3: dict) -> geo.Volume3D:
    """pkg/models/geo.go:305-320."""
    fp = vol3.get("footprint")
    if fp is None:
        raise ProtoError("spatial_volume missing required footprint")
    return geo.Volume3D(AltitudeHi=_f32(vol3.get("altitude_hi", 0.0)), AltitudeLo=_f32(vol3.get("altitude_lo", 0.0)),
                        Footprint=geo.GeoPolygon([LatLngPointFromSCDProto(v) for v in fp.get("vertices", [])]))


def Volume4DFromRIDProto(vol4: dict) -> geo.Volume4D:
    """pkg/models/geo.go:276-303 (time_start / time_end are bare timestamps)."""
    out = geo.Volume4D(SpatialVolume=Volume3DFromRIDProto(vol4.get("spatial_volume") or {}))
    if vol4.get("time_start") is not None:
        out.StartTime = int(vol4["time_start"])
    if vol4.get("time_end") is not None:
        out.EndTime = int(vol4["time_end"])
    return out


@dataclass
class IdentificationServiceArea:
    """The fields SetExtents writes (pkg/rid/models/identification_service_area.go:16-26)."""
    Cells: Optional[List[int]] = None
    StartTime: Optional[int] = None
    EndTime: Optional[int] = None
    AltitudeHi: Optional[float] = None
    AltitudeLo: Optional[float] = None

    def SetExtents(self, extents: Optional[dict]) -> None:
        """identification_service_area.go:71-105."""
        if extents is None:
            return
        if extents.get("time_start") is not None:
            self.StartTime = int(extents["time_start"])
        if extents.get("time_end") is not None:
            self.EndTime = int(extents["time_end"])
        space = extents.get("spatial_volume")
        if space is None:
            raise ProtoError("missing required spatial_volume")
        self.AltitudeHi = _f32(space.get("altitude_hi", 0.0))
        self.AltitudeLo = _f32(space.get("altitude_lo", 0.0))
        fp = space.get("footprint")
        if fp is None:
            raise ProtoError("spatial_volume missing required footprint")
        self.Cells = geo.GeoPolygon([LatLngPointFromSCDProto(v) for v in fp.get("vertices", [])]).CalculateCovering()
