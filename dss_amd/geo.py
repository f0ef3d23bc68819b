"""Covering API mirroring the reference's pkg/geo and pkg/models geometry.

Same names, argument meaning and error behaviour as
  pkg/geo/s2.go            Covering, AreaToCellIDs, DistanceMetersToAngle,
                           ErrAreaTooLarge, Levelify, ValidateCell
  pkg/models/geo.go        GeoPolygon / GeoCircle .CalculateCovering,
                           Volume4D / Volume3D, UnionVolumes4D
all computed by the gfx950 kernels behind include/dssgpu.h.  Cell unions are
Python lists / numpy arrays of uint64 S2 CellIDs (sorted, level 13).
"""
from __future__ import annotations

import ctypes as C
from dataclasses import dataclass, field
from typing import List, Optional, Sequence

import numpy as np

from . import _lib
from ._lib import (KIND_CIRCLE, KIND_POINTS, KIND_POLYGON, ST_AREA_TOO_LARGE, ST_BAD_COORD_SET, ST_NOT_ENOUGH_POINTS,
                   ST_ODD_COORDS, ST_OK, ST_RADIUS)

DEFAULT_MINIMUM_CELL_LEVEL = 13  # pkg/geo/s2.go:19
DEFAULT_MAXIMUM_CELL_LEVEL = 13  # pkg/geo/s2.go:22
MAX_ALLOWED_AREA_KM2 = 2500.0    # pkg/geo/s2.go:23
RADIUS_EARTH_METER = 6371010.0   # pkg/geo/s2.go:24


class GeoError(ValueError):
    """Base of the Go sentinel errors on the covering path."""


class BadCoordSetError(GeoError):
    def __init__(self):
        super().__init__("coordinates did not create a well formed area")  # pkg/geo/s2.go:39


class NotEnoughPointsError(GeoError):
    def __init__(self):
        super().__init__("not enough points in polygon")  # pkg/geo/s2.go:38


class OddNumberOfCoordinatesError(GeoError):
    def __init__(self):
        super().__init__("odd number of coordinates in area string")  # pkg/geo/s2.go:37


class RadiusMustBeLargerThan0Error(GeoError):
    def __init__(self):
        super().__init__("radius must be larger than 0")  # pkg/models/geo.go:38


class ErrAreaTooLarge(GeoError):
    """pkg/geo/s2.go:59-66; message formatted as fmt.Sprintf at :112-114."""

    def __init__(self, area_km2: float):
        super().__init__("area is too large (%fkm² > %fkm²)" % (area_km2, MAX_ALLOWED_AREA_KM2))
        self.area_km2 = area_km2


class MissingSpatialVolumeError(GeoError):
    def __init__(self):
        super().__init__("missing spatial volume")  # pkg/models/geo.go:31


class MissingFootprintError(GeoError):
    def __init__(self):
        super().__init__("missing footprint")  # pkg/models/geo.go:34


def error_for_status(status: int, area_km2: float = 0.0) -> Optional[GeoError]:
    if status == ST_OK:
        return None
    if status == ST_BAD_COORD_SET:
        return BadCoordSetError()
    if status == ST_NOT_ENOUGH_POINTS:
        return NotEnoughPointsError()
    if status == ST_ODD_COORDS:
        return OddNumberOfCoordinatesError()
    if status == ST_RADIUS:
        return RadiusMustBeLargerThan0Error()
    if status == ST_AREA_TOO_LARGE:
        return ErrAreaTooLarge(area_km2)
    return GeoError(f"unknown covering status {status}")


def DistanceMetersToAngle(distance: float) -> float:
    """pkg/geo/s2.go:85-87."""
    return distance / RADIUS_EARTH_METER


def ValidateCell(cell: int) -> None:
    """pkg/geo/s2.go:50-55: level from the lowest set bit only (Q12)."""
    cell = int(cell) & (2**64 - 1)
    lsb = cell & -cell
    level = 30 - ((lsb.bit_length() - 1) >> 1) if cell else -1
    if level != DEFAULT_MINIMUM_CELL_LEVEL:
        raise GeoError("cells must be at level 13 at current implementation")


# ------------------------------------------------------------------ batch
@dataclass
class CoverResult:
    offs: np.ndarray      # int64 [n+1]
    cells: np.ndarray     # uint64 [offs[n]]
    status: np.ndarray    # int32 [n]
    area_km2: np.ndarray  # float64 [n]

    def cells_of(self, i: int) -> np.ndarray:
        return self.cells[self.offs[i]:self.offs[i + 1]]


def _ptr(a, t):
    return a.ctypes.data_as(C.POINTER(t))


def cover_batch(kind, voff, lat, lng, radius_m=None, device: int = 0) -> CoverResult:
    """Batch covering through dssg_cover_batch (host buffers)."""
    ctx = _lib.context(device)
    kind = np.ascontiguousarray(kind, dtype=np.int32)
    voff = np.ascontiguousarray(voff, dtype=np.int64)
    lat = np.ascontiguousarray(lat, dtype=np.float64)
    lng = np.ascontiguousarray(lng, dtype=np.float64)
    n = len(kind)
    rad = np.ascontiguousarray(radius_m if radius_m is not None else np.zeros(n), dtype=np.float32)
    offs = np.zeros(n + 1, dtype=np.int64)
    status = np.zeros(max(n, 1), dtype=np.int32)
    area = np.zeros(max(n, 1), dtype=np.float64)
    need = C.c_int64(0)
    cap = max(16, 64 * n)
    while True:
        cells = np.zeros(cap, dtype=np.uint64)
        rc = ctx.L.dssg_cover_batch(ctx.h, n, _ptr(kind, C.c_int32), _ptr(voff, C.c_int64), _ptr(lat, C.c_double),
                                    _ptr(lng, C.c_double), _ptr(rad, C.c_float), _ptr(offs, C.c_int64),
                                    _ptr(cells, C.c_uint64), cap, C.byref(need), _ptr(status, C.c_int32),
                                    _ptr(area, C.c_double))
        if rc == _lib.DSSG_ERR_CAPACITY:
            cap = int(need.value)
            continue
        ctx.check(rc)
        return CoverResult(offs, cells[: need.value].copy(), status[:n], area[:n])


def _single(kind, lats, lngs, radius=0.0) -> np.ndarray:
    lats = np.asarray(lats, dtype=np.float64)
    lngs = np.asarray(lngs, dtype=np.float64)
    r = cover_batch([kind], [0, len(lats)], lats, lngs, [radius])
    err = error_for_status(int(r.status[0]), float(r.area_km2[0]))
    if err is not None:
        raise err
    return r.cells_of(0)


def Covering(lats: Sequence[float], lngs: Sequence[float]) -> List[int]:
    """pkg/geo/s2.go:99 Covering on points given as degrees (no range check)."""
    return [int(c) for c in _single(KIND_POINTS, lats, lngs)]


def AreaToCellIDs(area: str) -> List[int]:
    """pkg/geo/s2.go:129-166."""
    ctx = _lib.context()
    need = C.c_int64(0)
    st = C.c_int32(0)
    ar = C.c_double(0)
    cap = 4096
    while True:
        out = np.zeros(cap, dtype=np.uint64)
        rc = ctx.L.dssg_area_to_cell_ids(ctx.h, area.encode(), _ptr(out, C.c_uint64), cap, C.byref(need),
                                         C.byref(st), C.byref(ar))
        if rc == _lib.DSSG_ERR_CAPACITY:
            cap = int(need.value)
            continue
        ctx.check(rc)
        err = error_for_status(st.value, ar.value)
        if err is not None:
            raise err
        return [int(c) for c in out[: need.value]]


@dataclass
class LatLngPoint:
    Lat: float
    Lng: float


@dataclass
class GeoPolygon:
    """pkg/models/geo.go:247-268."""
    Vertices: List[LatLngPoint] = field(default_factory=list)

    def CalculateCovering(self) -> List[int]:
        if self is None:
            raise BadCoordSetError()
        lats = [v.Lat for v in self.Vertices]
        lngs = [v.Lng for v in self.Vertices]
        return [int(c) for c in _single(KIND_POLYGON, lats, lngs)]


@dataclass
class GeoCircle:
    """pkg/models/geo.go:217-239 (RadiusMeter is float32)."""
    Center: LatLngPoint
    RadiusMeter: float

    def CalculateCovering(self) -> List[int]:
        r = float(np.float32(self.RadiusMeter))
        return [int(c) for c in _single(KIND_CIRCLE, [self.Center.Lat], [self.Center.Lng], r)]


class GeometryFunc:
    """pkg/models/geo.go:99,213-215."""

    def __init__(self, fn):
        self.fn = fn

    def CalculateCovering(self):
        return self.fn()


class _PrecomputedCellGeometry(dict):
    """pkg/models/geo.go:101-122: a set; CalculateCovering returns it unsorted (Q14)."""

    def CalculateCovering(self):
        return list(self.keys())


@dataclass
class Volume3D:
    AltitudeHi: Optional[float] = None
    AltitudeLo: Optional[float] = None
    Footprint: object = None

    def CalculateCovering(self):
        if self.Footprint is None:
            raise MissingFootprintError()
        return self.Footprint.CalculateCovering()


@dataclass
class Volume4D:
    SpatialVolume: Optional[Volume3D] = None
    EndTime: Optional[int] = None    # microseconds since epoch
    StartTime: Optional[int] = None

    def CalculateSpatialCovering(self):
        if self.SpatialVolume is None:
            raise MissingSpatialVolumeError()
        return self.SpatialVolume.CalculateCovering()


def UnionVolumes4D(*volumes: Volume4D) -> Volume4D:
    """pkg/models/geo.go:126-190 (covers every extent; union in a map, Q14)."""
    result = Volume4D()
    for v in volumes:
        if v.EndTime is not None:
            result.EndTime = v.EndTime if result.EndTime is None else max(result.EndTime, v.EndTime)
        if v.StartTime is not None:
            result.StartTime = v.StartTime if result.StartTime is None else min(result.StartTime, v.StartTime)
        if v.SpatialVolume is not None:
            if result.SpatialVolume is None:
                result.SpatialVolume = Volume3D()
            sv, rv = v.SpatialVolume, result.SpatialVolume
            if sv.AltitudeLo is not None:
                rv.AltitudeLo = sv.AltitudeLo if rv.AltitudeLo is None else min(rv.AltitudeLo, sv.AltitudeLo)
            if sv.AltitudeHi is not None:
                rv.AltitudeHi = sv.AltitudeHi if rv.AltitudeHi is None else max(rv.AltitudeHi, sv.AltitudeHi)
            if sv.Footprint is not None:
                cells = sv.Footprint.CalculateCovering()
                if rv.Footprint is None:
                    rv.Footprint = _PrecomputedCellGeometry()
                for c in cells:
                    rv.Footprint[c] = None
    return result


def Levelify(cells: Sequence[int]) -> List[int]:
    """pkg/geo/s2.go:44-48: CellUnion.Denormalize(13, 1) -- coarser cells are
    replaced by their level-13 descendants, finer cells kept, order kept."""
    out = []
    lsb13 = 1 << 34
    for c in cells:
        c = int(c)
        lsb = c & -c
        level = 30 - ((lsb.bit_length() - 1) >> 1)
        if level >= 13:
            out.append(c)
        else:
            first = c - lsb + lsb13
            out.extend(first + k * (lsb13 << 1) for k in range(4 ** (13 - level)))
    return out


def UnionVolumes4DBatch(requests: Sequence[Sequence[Volume4D]], device: int = 0) -> list:
    """models.UnionVolumes4D (pkg/models/geo.go:126-190) for a batch of
    requests on the GPU (dssg_union_volumes_device): one cover launch for
    every extent of every request, then a per-request union of the cells.
    Returns, per request, the GeoError UnionVolumes4D would return or the
    union Volume4D (its Footprint the union cell set, sorted).  Footprints
    must be GeoPolygon / GeoCircle (GeometryFunc cells are already covered)."""
    import torch  # plumbing: device buffers
    from . import device as D
    vol_offs, kinds, voff, lat, lng, rad, has_fp, alo, ahi, t0, t1, spatial = [0], [], [0], [], [], [], [], [], [], [], [], []
    for req in requests:
        sp = False
        for v in req:
            sv = v.SpatialVolume
            sp = sp or sv is not None
            fp = sv.Footprint if sv is not None else None
            if isinstance(fp, GeoPolygon):
                kinds.append(KIND_POLYGON)
                lat += [p.Lat for p in fp.Vertices]
                lng += [p.Lng for p in fp.Vertices]
                rad.append(0.0)
            elif isinstance(fp, GeoCircle):
                kinds.append(KIND_CIRCLE)
                lat.append(fp.Center.Lat)
                lng.append(fp.Center.Lng)
                rad.append(float(np.float32(fp.RadiusMeter)))
            elif fp is None:
                kinds.append(KIND_POINTS)  # no vertices; ignored (has_fp = 0)
                rad.append(0.0)
            else:
                raise TypeError("UnionVolumes4DBatch: footprints must be GeoPolygon or GeoCircle")
            voff.append(len(lat))
            has_fp.append(1 if fp is not None else 0)
            alo.append(np.nan if sv is None or sv.AltitudeLo is None else np.float32(sv.AltitudeLo))
            ahi.append(np.nan if sv is None or sv.AltitudeHi is None else np.float32(sv.AltitudeHi))
            t0.append(_lib.TIME_NULL_START if v.StartTime is None else v.StartTime)
            t1.append(_lib.TIME_NULL_END_Q if v.EndTime is None else v.EndTime)
        vol_offs.append(len(kinds))
        spatial.append(sp)
    ctx = _lib.context(device)
    dev = f"cuda:{device}"
    t = lambda a, dt: torch.as_tensor(np.asarray(a, dtype=dt) if len(a) else np.zeros(1, dt), device=dev)  # noqa: E731
    bufs = [t(vol_offs, np.int64), t(kinds, np.int32), t(voff, np.int64), t(lat, np.float64), t(lng, np.float64),
            t(rad, np.float32), t(has_fp, np.uint8), t(alo, np.float32), t(ahi, np.float32), t(t0, np.int64),
            t(t1, np.int64)]
    out = _lib.Volumes()
    ctx.check(ctx.L.dssg_union_volumes_device(ctx.h, len(requests), *[D._ptr(b) for b in bufs], D._stream_ptr(),
                                              C.byref(out)))
    n = len(requests)
    offs = D.copy_back(ctx, out.offs, n + 1, np.int64)
    cells = D.copy_back(ctx, out.cells, int(offs[-1]), np.uint64)
    st = D.copy_back(ctx, out.status, n, np.int32)
    area = D.copy_back(ctx, out.area_km2, n, np.float64)
    lo = D.copy_back(ctx, out.alt_lo, n, np.float32)
    hi = D.copy_back(ctx, out.alt_hi, n, np.float32)
    s0 = D.copy_back(ctx, out.t0, n, np.int64)
    s1 = D.copy_back(ctx, out.t1, n, np.int64)
    fp = D.copy_back(ctx, out.has_footprint, n, np.uint8)
    res = []
    for i in range(n):
        err = error_for_status(int(st[i]), float(area[i]))
        if err is not None:
            res.append(err)
            continue
        v = Volume4D(StartTime=None if s0[i] == _lib.TIME_NULL_START else int(s0[i]),
                     EndTime=None if s1[i] == _lib.TIME_NULL_END_Q else int(s1[i]))
        if spatial[i]:
            v.SpatialVolume = Volume3D(AltitudeLo=None if lo[i] == -np.inf else float(lo[i]),
                                       AltitudeHi=None if hi[i] == np.inf else float(hi[i]))
            if fp[i]:
                g = _PrecomputedCellGeometry()
                for c in cells[offs[i]:offs[i + 1]]:
                    g[int(c)] = None
                v.SpatialVolume.Footprint = g
        res.append(v)
    return res
