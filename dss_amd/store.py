"""Store-side search API mirroring the reference's store interfaces.

  scdstore.OperationStore.SearchOperations   pkg/scd/store/store.go:29
      impl pkg/scd/store/cockroach/operations.go:374-445
  repos.ISA.SearchISAs                       pkg/rid/repos/isa.go:27
      impl pkg/rid/cockroach/identification_service_area.go:166-197
      app clamp pkg/rid/application/isa.go:38-45
  repos.Subscription.SearchSubscriptions[ByOwner] pkg/rid/repos/subscription.go:26-29
      impl pkg/rid/cockroach/subscriptions.go:222-273
  scdstore.SubscriptionStore.SearchSubscriptions pkg/scd/store/store.go:35
      impl pkg/scd/store/cockroach/subscriptions.go:498-545 (Q7: cells ignored)
  repos.Subscription.UpdateNotificationIdxsInCells / MaxSubscriptionCountInCellsByOwner
      impl pkg/rid/cockroach/subscriptions.go:83-116, 204-219
  SCD fetchSubscriptionsForNotification / fetchMaxSubscriptionCountByCellAndOwner
      pkg/scd/store/cockroach/subscriptions.go:128-173, 255-283

Stored entities live in a GPU-resident `EntityIndex` (dssg_index).  Entity
ids are dense 0..n-1 indices that the caller maps to its rows (UUIDs).
Times are int64 microseconds; None means SQL NULL.
"""
from __future__ import annotations

import ctypes as C
from typing import List, Optional, Sequence, Tuple

import numpy as np

from . import _lib
from .geo import GeoError, Volume4D

NULL_START = _lib.TIME_NULL_START
NULL_END = _lib.TIME_NULL_END
NULL_END_Q = _lib.TIME_NULL_END_Q


class BadRequest(ValueError):
    """dsserr.BadRequest (pkg/errors/errors.go:88-90) -> codes.InvalidArgument."""


class Internal(RuntimeError):
    """dsserr.Internal -> codes.Internal."""


def _p(a, t):
    return a.ctypes.data_as(C.POINTER(t))


def _csr(cell_lists: Sequence[Sequence[int]]) -> Tuple[np.ndarray, np.ndarray]:
    offs = np.zeros(len(cell_lists) + 1, dtype=np.int64)
    for i, c in enumerate(cell_lists):
        offs[i + 1] = offs[i] + len(c)
    cells = np.zeros(int(offs[-1]), dtype=np.uint64)
    for i, c in enumerate(cell_lists):
        cells[offs[i]:offs[i + 1]] = np.asarray([int(x) & (2**64 - 1) for x in c], dtype=np.uint64)
    return offs, cells


def _f32_or(v: Optional[float], null: float) -> float:
    return null if v is None else float(np.float32(v))


class EntityIndex:
    """GPU-resident index of stored entities (operational intents, ISAs,
    subscriptions): replaces scd_cells_operations / RID cells INT64[] +
    INVERTED INDEX.  NULL conventions as include/dssgpu.h."""

    def __init__(self, cell_offs, cells, alt_lo=None, alt_hi=None, t0=None, t1=None, owner=None, device: int = 0,
                 cell_range=None):
        """cell_range=(lo, hi): a cell-range shard (dssg_index_build_range):
        postings only for cells in [lo, hi] (uint64 order), entity cell lists
        whole."""
        self.ctx = _lib.context(device)
        offs = np.ascontiguousarray(cell_offs, dtype=np.int64)
        n = len(offs) - 1
        cells = np.ascontiguousarray(cells, dtype=np.uint64)
        alo = np.ascontiguousarray(alt_lo if alt_lo is not None else np.full(n, -np.inf), dtype=np.float32)
        ahi = np.ascontiguousarray(alt_hi if alt_hi is not None else np.full(n, np.inf), dtype=np.float32)
        a0 = np.ascontiguousarray(t0 if t0 is not None else np.full(n, NULL_START), dtype=np.int64)
        a1 = np.ascontiguousarray(t1 if t1 is not None else np.full(n, 2**63 - 1), dtype=np.int64)
        own = np.ascontiguousarray(owner, dtype=np.int32) if owner is not None else None
        h = C.c_void_p()
        lo, hi = cell_range if cell_range is not None else (0, 2**64 - 1)
        rc = self.ctx.L.dssg_index_build_range(self.ctx.h, n, _p(offs, C.c_int64), _p(cells, C.c_uint64),
                                               _p(alo, C.c_float), _p(ahi, C.c_float), _p(a0, C.c_int64),
                                               _p(a1, C.c_int64),
                                               _p(own, C.c_int32) if own is not None else C.POINTER(C.c_int32)(),
                                               int(lo), int(hi), C.byref(h))
        self.ctx.check(rc)
        self.h = h
        self.n = n

    @classmethod
    def from_lists(cls, cell_lists, alt_lo=None, alt_hi=None, t0=None, t1=None, owner=None, device=0,
                   cell_range=None):
        offs, cells = _csr(cell_lists)
        return cls(offs, cells, alt_lo, alt_hi, t0, t1, owner, device, cell_range)

    @property
    def num_postings(self) -> int:
        return int(self.ctx.L.dssg_index_num_postings(self.h))

    def info(self) -> dict:
        """dssg_index_info: postings, distinct cells, long-duration and
        long-footprint postings, the largest cell's postings, dcap (us)."""
        import ctypes as C
        v = [C.c_int64() for _ in range(6)]
        self.ctx.check(self.ctx.L.dssg_index_info(self.h, *[C.byref(x) for x in v]))
        return dict(zip(["postings", "cells", "long_duration_postings", "long_footprint_postings", "max_cell_postings",
                         "dcap_us"], [x.value for x in v]))

    def free(self):
        if getattr(self, "h", None):
            self.ctx.L.dssg_index_free(self.h)
            self.h = None

    def __del__(self):
        try:
            self.free()
        except Exception:
            pass

    # -------------------------------------------------------------- batches
    def _call(self, fn, nq, *args) -> Tuple[np.ndarray, np.ndarray]:
        need = C.c_int64(0)
        cap = max(1024, nq * 8)
        while True:
            oq = np.zeros(cap, dtype=np.uint32)
            oe = np.zeros(cap, dtype=np.uint32)
            rc = fn(self.ctx.h, self.h, nq, *args, _p(oq, C.c_uint32), _p(oe, C.c_uint32), cap, C.byref(need))
            if rc == _lib.DSSG_ERR_CAPACITY:
                cap = int(need.value) + 1
                continue
            self.ctx.check(rc)
            return oq[: need.value].copy(), oe[: need.value].copy()

    def search_batch(self, q_offs, q_cells, alt_lo, alt_hi, tlo, thi, owner=None):
        """Generic join (dssg_search); pairs sorted by (query, entity)."""
        q_offs = np.ascontiguousarray(q_offs, dtype=np.int64)
        q_cells = np.ascontiguousarray(q_cells, dtype=np.uint64)
        nq = len(q_offs) - 1
        lo = np.ascontiguousarray(alt_lo, dtype=np.float32)
        hi = np.ascontiguousarray(alt_hi, dtype=np.float32)
        tl = np.ascontiguousarray(tlo, dtype=np.int64)
        th = np.ascontiguousarray(thi, dtype=np.int64)
        ow = np.ascontiguousarray(owner, dtype=np.int32) if owner is not None else None
        return self._call(self.ctx.L.dssg_search, nq, _p(q_offs, C.c_int64), _p(q_cells, C.c_uint64),
                          _p(lo, C.c_float), _p(hi, C.c_float), _p(tl, C.c_int64), _p(th, C.c_int64),
                          _p(ow, C.c_int32) if ow is not None else C.POINTER(C.c_int32)())

    def search_operations_batch(self, q_offs, q_cells, alt_lo, alt_hi, start, end, now_us):
        q_offs = np.ascontiguousarray(q_offs, dtype=np.int64)
        q_cells = np.ascontiguousarray(q_cells, dtype=np.uint64)
        nq = len(q_offs) - 1
        lo = np.ascontiguousarray(alt_lo, dtype=np.float32)
        hi = np.ascontiguousarray(alt_hi, dtype=np.float32)
        s = np.ascontiguousarray(start, dtype=np.int64)
        e = np.ascontiguousarray(end, dtype=np.int64)
        return self._call(self.ctx.L.dssg_search_operations, nq, _p(q_offs, C.c_int64), _p(q_cells, C.c_uint64),
                          _p(lo, C.c_float), _p(hi, C.c_float), _p(s, C.c_int64), _p(e, C.c_int64), int(now_us))

    def search_isas_batch(self, q_offs, q_cells, earliest, latest):
        q_offs = np.ascontiguousarray(q_offs, dtype=np.int64)
        q_cells = np.ascontiguousarray(q_cells, dtype=np.uint64)
        nq = len(q_offs) - 1
        ea = np.ascontiguousarray(earliest, dtype=np.int64)
        la = np.ascontiguousarray(latest, dtype=np.int64)
        return self._call(self.ctx.L.dssg_search_isas, nq, _p(q_offs, C.c_int64), _p(q_cells, C.c_uint64),
                          _p(ea, C.c_int64), _p(la, C.c_int64))

    def search_subscriptions_batch(self, q_offs, q_cells, now_us, owner=None):
        q_offs = np.ascontiguousarray(q_offs, dtype=np.int64)
        q_cells = np.ascontiguousarray(q_cells, dtype=np.uint64)
        nq = len(q_offs) - 1
        ow = np.ascontiguousarray(owner, dtype=np.int32) if owner is not None else None
        return self._call(self.ctx.L.dssg_search_subscriptions, nq, _p(q_offs, C.c_int64), _p(q_cells, C.c_uint64),
                          _p(ow, C.c_int32) if ow is not None else C.POINTER(C.c_int32)(), int(now_us))


    # ------------------------------------------- subscription-store queries
    def set_notification_index(self, values):
        v = np.ascontiguousarray(values, dtype=np.int64)
        if len(v) != self.n:
            raise ValueError("one notification index per entity")
        self.ctx.check(self.ctx.L.dssg_index_set_notification_index(self.ctx.h, self.h, _p(v, C.c_int64)))

    def notification_index(self) -> np.ndarray:
        v = np.zeros(max(self.n, 1), dtype=np.int64)
        self.ctx.check(self.ctx.L.dssg_index_get_notification_index(self.ctx.h, self.h, _p(v, C.c_int64)))
        return v[: self.n]

    def notify_batch(self, q_offs, q_cells, now_us):
        """dssg_notify_subscriptions: (q, e, notification index after the
        increment), sorted by (e, q); the counters advance."""
        q_offs = np.ascontiguousarray(q_offs, dtype=np.int64)
        q_cells = np.ascontiguousarray(q_cells, dtype=np.uint64)
        nq = len(q_offs) - 1
        need = C.c_int64(0)
        cap = max(1024, nq * 8)
        while True:
            oq = np.zeros(cap, dtype=np.uint32)
            oe = np.zeros(cap, dtype=np.uint32)
            ov = np.zeros(cap, dtype=np.int64)
            rc = self.ctx.L.dssg_notify_subscriptions(self.ctx.h, self.h, nq, _p(q_offs, C.c_int64),
                                                      _p(q_cells, C.c_uint64), int(now_us), _p(oq, C.c_uint32),
                                                      _p(oe, C.c_uint32), _p(ov, C.c_int64), cap, C.byref(need))
            if rc == _lib.DSSG_ERR_CAPACITY:
                cap = int(need.value) + 1
                continue
            self.ctx.check(rc)
            n = need.value
            return oq[:n].copy(), oe[:n].copy(), ov[:n].copy()

    def owner_subscriptions_batch(self, owner, now_us):
        ow = np.ascontiguousarray(owner, dtype=np.int32)
        return self._call(self.ctx.L.dssg_owner_subscriptions, len(ow), _p(ow, C.c_int32), int(now_us))

    def max_subscription_count_batch(self, q_offs, q_cells, owner, now_us) -> np.ndarray:
        q_offs = np.ascontiguousarray(q_offs, dtype=np.int64)
        q_cells = np.ascontiguousarray(q_cells, dtype=np.uint64)
        ow = np.ascontiguousarray(owner, dtype=np.int32)
        nq = len(q_offs) - 1
        out = np.zeros(max(nq, 1), dtype=np.int64)
        self.ctx.check(self.ctx.L.dssg_max_subscription_count(self.ctx.h, self.h, nq, _p(q_offs, C.c_int64),
                                                              _p(q_cells, C.c_uint64), _p(ow, C.c_int32),
                                                              int(now_us), _p(out, C.c_int64)))
        return out[:nq]


# ------------------------------------------------------------ reference API
def SearchOperations(index: EntityIndex, v4d: Volume4D, owner=None, now_us: int = 0) -> List[int]:
    """operations.go:374-445 searchOperations; `owner` is ignored (Q6)."""
    if v4d.SpatialVolume is None or v4d.SpatialVolume.Footprint is None:
        raise BadRequest("missing geospatial footprint for query")
    try:
        cells = v4d.SpatialVolume.Footprint.CalculateCovering()
    except GeoError as err:
        raise BadRequest(str(err)) from err
    if len(cells) == 0:
        raise BadRequest("missing cell IDs for query")
    offs, cc = _csr([cells])
    sv = v4d.SpatialVolume
    _, e = index.search_operations_batch(
        offs, cc, [_f32_or(sv.AltitudeLo, -np.inf)], [_f32_or(sv.AltitudeHi, np.inf)],
        [NULL_START if v4d.StartTime is None else v4d.StartTime],
        [NULL_END_Q if v4d.EndTime is None else v4d.EndTime], now_us)
    return [int(x) for x in e]


def SearchISAs(index: EntityIndex, cells: Sequence[int], earliest: Optional[int], latest: Optional[int]) -> List[int]:
    """identification_service_area.go:166-197 (store layer, no clamp)."""
    if len(cells) == 0:
        raise BadRequest("missing cell IDs for query")
    if earliest is None:
        raise Internal("must call with an earliest start time.")
    offs, cc = _csr([cells])
    _, e = index.search_isas_batch(offs, cc, [earliest], [NULL_END_Q if latest is None else latest])
    return [int(x) for x in e]


def AppSearchISAs(index: EntityIndex, cells, earliest: Optional[int], latest: Optional[int], now_us: int):
    """pkg/rid/application/isa.go:38-45: earliest = max(now, earliest) (Q15)."""
    if earliest is None or earliest < now_us:
        earliest = now_us
    return SearchISAs(index, cells, earliest, latest)


def SearchSubscriptions(index: EntityIndex, cells: Sequence[int], now_us: int) -> List[int]:
    """RID subscriptions.go:222-245."""
    if len(cells) == 0:
        raise BadRequest("no location provided")
    offs, cc = _csr([cells])
    _, e = index.search_subscriptions_batch(offs, cc, now_us)
    return [int(x) for x in e]


def SearchSubscriptionsByOwner(index: EntityIndex, cells: Sequence[int], owner: int, now_us: int) -> List[int]:
    """RID subscriptions.go:247-273."""
    if len(cells) == 0:
        raise BadRequest("no location provided")
    offs, cc = _csr([cells])
    _, e = index.search_subscriptions_batch(offs, cc, now_us, [owner])
    return [int(x) for x in e]


def UpdateNotificationIdxsInCells(index: EntityIndex, cells: Sequence[int], now_us: int) -> List[Tuple[int, int]]:
    """RID subscriptions.go:204-219: every unexpired subscription sharing a
    cell gets notification_index + 1; returns (entity, new index) rows."""
    offs, cc = _csr([cells])
    _, e, v = index.notify_batch(offs, cc, now_us)
    return [(int(a), int(b)) for a, b in zip(e, v)]


def FetchSubscriptionsForNotification(index: EntityIndex, cells: Sequence[int], now_us: int) -> List[Tuple[int, int]]:
    """SCD subscriptions.go:128-173 (DISTINCT subscription_id WHERE cell_id =
    ANY(cells), then the UPDATE ... WHERE ends_at >= now RETURNING): the same
    fan-out over the SCD cells table."""
    return UpdateNotificationIdxsInCells(index, cells, now_us)


def SCDSearchSubscriptions(index: EntityIndex, cells: Sequence[int], owner: int, now_us: int) -> List[int]:
    """scdstore.SubscriptionStore.SearchSubscriptions (pkg/scd/store/cockroach/
    subscriptions.go:497-545): every unexpired subscription of the owner; the
    cells do not filter (Q7) but an empty covering is still a BadRequest."""
    if len(cells) == 0:
        raise BadRequest("no location provided")
    _, e = index.owner_subscriptions_batch([owner], now_us)
    return [int(x) for x in e]


def MaxSubscriptionCountInCellsByOwner(index: EntityIndex, cells: Sequence[int], owner: int, now_us: int) -> int:
    """RID subscriptions.go:83-116 / SCD subscriptions.go:255-283."""
    offs, cc = _csr([cells])
    return int(index.max_subscription_count_batch(offs, cc, [owner], now_us)[0])


# ------------------------------------------------------------- write path
class Store:
    """dssg_store: a mutable entity index keyed by caller ids (uint32).
    Upserts/deletes are visible to every later search (base + delta index +
    tombstones on the GPU, include/dssgpu.h)."""

    def __init__(self, with_owner: bool = False, device: int = 0):
        self.ctx = _lib.context(device)
        h = C.c_void_p()
        self.ctx.check(self.ctx.L.dssg_store_create(self.ctx.h, 1 if with_owner else 0, C.byref(h)))
        self.h = h
        self.with_owner = with_owner

    def free(self):
        if getattr(self, "h", None):
            self.ctx.L.dssg_store_free(self.h)
            self.h = None

    def __del__(self):
        try:
            self.free()
        except Exception:
            pass

    def upsert(self, ids, cell_lists, alt_lo, alt_hi, t0, t1, owner=None):
        ids = np.ascontiguousarray(ids, dtype=np.uint32)
        offs, cells = _csr(cell_lists)
        lo = np.ascontiguousarray(alt_lo, dtype=np.float32)
        hi = np.ascontiguousarray(alt_hi, dtype=np.float32)
        a0 = np.ascontiguousarray(t0, dtype=np.int64)
        a1 = np.ascontiguousarray(t1, dtype=np.int64)
        ow = np.ascontiguousarray(owner, dtype=np.int32) if owner is not None else None
        self.ctx.check(self.ctx.L.dssg_store_upsert(
            self.ctx.h, self.h, len(ids), _p(ids, C.c_uint32), _p(offs, C.c_int64), _p(cells, C.c_uint64),
            _p(lo, C.c_float), _p(hi, C.c_float), _p(a0, C.c_int64), _p(a1, C.c_int64),
            _p(ow, C.c_int32) if ow is not None else C.POINTER(C.c_int32)()))

    def delete(self, ids) -> np.ndarray:
        ids = np.ascontiguousarray(ids, dtype=np.uint32)
        found = np.zeros(max(len(ids), 1), dtype=np.int32)
        self.ctx.check(self.ctx.L.dssg_store_delete(self.ctx.h, self.h, len(ids), _p(ids, C.c_uint32),
                                                    _p(found, C.c_int32)))
        return found[: len(ids)].astype(bool)

    def compact(self):
        self.ctx.check(self.ctx.L.dssg_store_compact(self.ctx.h, self.h))

    def stats(self) -> dict:
        v = [C.c_int64() for _ in range(4)]
        self.ctx.check(self.ctx.L.dssg_store_stats(self.h, *[C.byref(x) for x in v]))
        return dict(zip(["live", "base", "delta", "compactions"], [x.value for x in v]))

    def max_subscription_count_batch(self, q_offs, q_cells, owner, now_us) -> np.ndarray:
        """RID MaxSubscriptionCountInCellsByOwner (subscriptions.go:83-116)
        over the store's live rows (dssg_store_max_subscription_count)."""
        q_offs = np.ascontiguousarray(q_offs, dtype=np.int64)
        q_cells = np.ascontiguousarray(q_cells, dtype=np.uint64)
        ow = np.ascontiguousarray(owner, dtype=np.int32)
        nq = len(q_offs) - 1
        out = np.zeros(max(nq, 1), dtype=np.int64)
        self.ctx.check(self.ctx.L.dssg_store_max_subscription_count(
            self.ctx.h, self.h, nq, _p(q_offs, C.c_int64), _p(q_cells, C.c_uint64), _p(ow, C.c_int32), int(now_us),
            _p(out, C.c_int64)))
        return out[:nq]

    def search_batch(self, q_offs, q_cells, alt_lo, alt_hi, tlo, thi, owner=None):
        """(query, id) pairs, sorted; the generic predicate of dssg_search."""
        q_offs = np.ascontiguousarray(q_offs, dtype=np.int64)
        q_cells = np.ascontiguousarray(q_cells, dtype=np.uint64)
        nq = len(q_offs) - 1
        lo = np.ascontiguousarray(alt_lo, dtype=np.float32)
        hi = np.ascontiguousarray(alt_hi, dtype=np.float32)
        tl = np.ascontiguousarray(tlo, dtype=np.int64)
        th = np.ascontiguousarray(thi, dtype=np.int64)
        ow = np.ascontiguousarray(owner, dtype=np.int32) if owner is not None else None
        need = C.c_int64(0)
        cap = max(1024, nq * 8)
        while True:
            oq = np.zeros(cap, dtype=np.uint32)
            oe = np.zeros(cap, dtype=np.uint32)
            rc = self.ctx.L.dssg_store_search(
                self.ctx.h, self.h, nq, _p(q_offs, C.c_int64), _p(q_cells, C.c_uint64), _p(lo, C.c_float),
                _p(hi, C.c_float), _p(tl, C.c_int64), _p(th, C.c_int64),
                _p(ow, C.c_int32) if ow is not None else C.POINTER(C.c_int32)(), _p(oq, C.c_uint32),
                _p(oe, C.c_uint32), cap, C.byref(need))
            if rc == _lib.DSSG_ERR_CAPACITY:
                cap = int(need.value) + 1
                continue
            self.ctx.check(rc)
            return oq[: need.value].copy(), oe[: need.value].copy()


class NotFound(LookupError):
    """dsserr.NotFound -> codes.NotFound."""


class AlreadyExists(ValueError):
    """dsserr.AlreadyExists -> codes.AlreadyExists."""


class VersionMismatch(ValueError):
    """dsserr.VersionMismatch -> codes.Aborted."""


class PermissionDenied(PermissionError):
    """dsserr.PermissionDenied -> codes.PermissionDenied."""


class MissingOVNs(RuntimeError):
    """scderr.MissingOVNsInternalError: the key lacks the OVN of a conflicting
    operation; `missing` lists those operations' ids."""

    def __init__(self, missing):
        super().__init__("missing OVNs")
        self.missing = missing


def ovn_from_time(updated_at_rfc3339: str, salt: str) -> str:
    """NewOVNFromTime (pkg/scd/models/models.go:35-40):
    base64(sha256(salt + t.Format(RFC3339)))."""
    import base64
    import hashlib
    return base64.b64encode(hashlib.sha256((salt + updated_at_rfc3339).encode()).digest()).decode()


class Operation:
    """The scdmodels.Operation fields the write path reads (pkg/scd/models/
    operations.go:27-45); times are int64 us, None = NULL."""

    def __init__(self, id, owner, cells, altitude_lower=None, altitude_upper=None, start=None, end=None,
                 state="Accepted", version=0):
        self.ID, self.Owner, self.Cells = id, owner, list(cells)
        self.AltitudeLower, self.AltitudeUpper = altitude_lower, altitude_upper
        self.StartTime, self.EndTime = start, end
        self.State, self.Version = state, version
        self.OVN = ""
        self.UpdatedAt = None


class MutableOperationStore:
    """scdstore.OperationStore's write path over a GPU `Store`:
    UpsertOperation (pkg/scd/store/cockroach/operations.go:304-372),
    DeleteOperation (:239-301), SearchOperations (:374-445).  Rows and OVNs
    live here (host); cells + the 4D attributes live in the GPU store.
    Owners are strings here and small ints on the GPU (interned)."""

    def __init__(self, device: int = 0):
        self.gpu = Store(with_owner=False, device=device)
        self.ops = {}      # id -> Operation
        self.slot = {}     # id -> uint32 GPU id
        self.by_slot = {}  # GPU id -> op id
        self._next = 0

    def _slot_of(self, op_id):
        if op_id not in self.slot:
            self.slot[op_id] = self._next
            self.by_slot[self._next] = op_id
            self._next += 1
        return self.slot[op_id]

    def SearchOperations(self, cells, alt_lo, alt_hi, start, end, now_us) -> List["Operation"]:
        """searchOperations over already-covered cells (the store-internal
        GeometryFunc path, operations.go:337-348)."""
        if len(cells) == 0:
            raise BadRequest("missing cell IDs for query")
        offs, cc = _csr([cells])
        tlo = max(NULL_START if start is None else start, now_us)
        thi = NULL_END_Q if end is None else end
        _, ids = self.gpu.search_batch(offs, cc, [_f32_or(alt_lo, -np.inf)], [_f32_or(alt_hi, np.inf)], [tlo], [thi])
        return [self.ops[self.by_slot[int(i)]] for i in ids]

    def UpsertOperation(self, op: "Operation", key: Sequence[str], now_us: int, now_rfc3339: str):
        old = self.ops.get(op.ID)
        # Version.Empty() is v <= 0 (pkg/scd/models/models.go:56-58)
        if old is None and op.Version > 0:
            raise NotFound(op.ID)
        if old is not None and op.Version <= 0:
            raise AlreadyExists(op.ID)
        if old is not None and op.Version != old.Version:
            raise VersionMismatch("old version")
        if old is not None and old.Owner != op.Owner:
            raise PermissionDenied(f"Operation is owned by {old.Owner}")
        # ValidateTimeRange (pkg/scd/models/operations.go:78-94)
        if op.StartTime is None:
            raise BadRequest("Operation must have an time_start")
        if op.EndTime is None:
            raise BadRequest("Operation must have an time_end")
        if op.EndTime < op.StartTime:
            raise BadRequest("Operation time_end must be after time_start")
        if op.State in ("Accepted", "Activated"):
            keyset = set(key)
            found = self.SearchOperations(op.Cells, op.AltitudeLower, op.AltitudeUpper, op.StartTime, op.EndTime,
                                          now_us)
            missing = [o.ID for o in found if o.OVN not in keyset]
            if missing:
                raise MissingOVNs(missing)
        # pushOperation: version + 1, updated_at = transaction time, cells replaced
        op.Version = (old.Version if old is not None else 0) + 1
        op.UpdatedAt = now_rfc3339
        op.OVN = ovn_from_time(now_rfc3339, op.ID)
        s = self._slot_of(op.ID)
        self.gpu.upsert([s], [op.Cells], [_f32_or(op.AltitudeLower, -np.inf)], [_f32_or(op.AltitudeUpper, np.inf)],
                        [op.StartTime], [op.EndTime])
        self.ops[op.ID] = op
        return op

    def DeleteOperation(self, op_id, owner):
        old = self.ops.get(op_id)
        if old is None:
            raise NotFound(op_id)
        if old.Owner != owner:
            raise PermissionDenied(f"Operation is owned by {old.Owner}")
        self.gpu.delete([self.slot[op_id]])
        del self.ops[op_id]
        return old


class Batcher:
    """dssg_batcher: concurrent single SCD searchOperations requests (an
    uncovered footprint each) coalesced into one cover launch + one join per
    batch by the library's worker thread.  `search_operations` blocks the
    calling thread only (ctypes releases the GIL), so many Python threads --
    or Go goroutines through the same C call -- share batches."""

    def __init__(self, index: "EntityIndex", max_batch: int = 1024, max_wait_us: int = 200, device: int = 0):
        self.index = index  # the index must outlive the batcher
        self.L = _lib.load()
        h = C.c_void_p()
        rc = self.L.dssg_batcher_create(device, index.h, int(max_batch), int(max_wait_us), C.byref(h))
        if rc != _lib.DSSG_OK:
            raise _lib.DssgError(rc, self.L.dssg_strerror(rc).decode())
        self.h = h

    def search_operations(self, kind: int, lat, lng, radius_m: float, alt_lo: float, alt_hi: float, start: int,
                          end: int, now_us: int):
        """-> (status, entity ids); status DSSG_ST_* of the covering."""
        lat = np.ascontiguousarray(lat, dtype=np.float64)
        lng = np.ascontiguousarray(lng, dtype=np.float64)
        cap = 4096
        while True:
            out = np.empty(cap, dtype=np.uint32)
            needed, st, area = C.c_int64(), C.c_int32(), C.c_double()
            rc = self.L.dssg_batcher_search_operations(self.h, int(kind), len(lat), _p(lat, C.c_double),
                                                       _p(lng, C.c_double), float(radius_m), float(alt_lo),
                                                       float(alt_hi), int(start), int(end), int(now_us),
                                                       _p(out, C.c_uint32), cap, C.byref(needed), C.byref(st),
                                                       C.byref(area))
            if rc == _lib.DSSG_ERR_CAPACITY:
                cap = int(needed.value) + 1
                continue
            if rc != _lib.DSSG_OK:
                raise _lib.DssgError(rc, self.L.dssg_strerror(rc).decode())
            return int(st.value), out[: needed.value].copy()

    def stats(self):
        r, b = C.c_int64(), C.c_int64()
        self.L.dssg_batcher_stats(self.h, C.byref(r), C.byref(b))
        return int(r.value), int(b.value)

    def close(self):
        if getattr(self, "h", None):
            self.L.dssg_batcher_free(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass
