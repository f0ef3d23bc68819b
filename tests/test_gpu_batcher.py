"""The per-request path (dssg_batcher): concurrent single searchOperations
requests, each an uncovered footprint, coalesced into shared batches; every
caller's answer and covering status equal the oracle's (CPU covering + join
of the same request) and a direct batch search of its own request; covering
errors come back as statuses."""
import threading

import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def test_batcher_matches_oracle_and_direct_search(oracle):
    from dss_amd import geo, workload as W
    from dss_amd.store import Batcher, EntityIndex
    _, q, qa, it, ia, now = W.config(0, scale=0.02)
    ci = geo.cover_batch(it.kind, it.voff, it.lat, it.lng, it.radius_m)
    idx = EntityIndex(ci.offs, ci.cells, ia.alt_lo, ia.alt_hi, ia.t0, ia.t1)
    cq = geo.cover_batch(q.kind, q.voff, q.lat, q.lng, q.radius_m)
    wq, we = idx.search_operations_batch(cq.offs, cq.cells, qa.alt_lo, qa.alt_hi, qa.t0, qa.t1, now)
    want = [we[wq == i] for i in range(q.n)]
    # the oracle's answer per request (pkg/scd/store/cockroach/operations.go:376-402)
    io, ic, _, _ = oracle.cover_batch(it.kind, it.voff, it.lat, it.lng, it.radius_m)
    qo, qc, qst, _ = oracle.cover_batch(q.kind, q.voff, q.lat, q.lng, q.radius_m)
    oq, oe = oracle.search(io, ic, ia.alt_lo, ia.alt_hi, ia.t0, ia.t1, None, qo, qc, qa.alt_lo, qa.alt_hi,
                           np.maximum(qa.t0, now), qa.t1)
    want_o = [oe[oq == i] for i in range(q.n)]
    assert sum(len(w) for w in want_o) > 0
    b = Batcher(idx, max_batch=64, max_wait_us=500)
    got = [None] * q.n
    errors = []

    def worker(lo, hi):
        try:
            for i in range(lo, hi):
                v0, v1 = q.voff[i], q.voff[i + 1]
                st, ids = b.search_operations(q.kind[i], q.lat[v0:v1], q.lng[v0:v1], q.radius_m[i], qa.alt_lo[i],
                                              qa.alt_hi[i], qa.t0[i], qa.t1[i], now)
                got[i] = (st, ids)
        except Exception as e:  # surfaced below
            errors.append(e)

    T = 16
    ths = [threading.Thread(target=worker, args=(k * q.n // T, (k + 1) * q.n // T)) for k in range(T)]
    for t in ths:
        t.start()
    for t in ths:
        t.join()
    assert not errors, errors[0]
    for i in range(q.n):
        st, ids = got[i]
        assert st == int(cq.status[i]) == int(qst[i])
        assert np.array_equal(np.sort(ids), np.sort(want_o[i])), i
        assert np.array_equal(np.sort(ids), np.sort(want[i])), i
    nreq, nbatch = b.stats()
    assert nreq == q.n and nbatch < q.n  # requests really were coalesced
    # a covering error is a status, not an exception (the caller's BadRequest)
    st, ids = b.search_operations(1, [37.4], [-122.1], 0.0, 0, 100, 0, 10**12, now)
    assert st == 4 and len(ids) == 0  # DSSG_ST_RADIUS
    b.close()
    idx.free()


def test_batcher_capacity_retry_is_served_from_the_kept_answer():
    """ABI capacity protocol: DSSG_ERR_CAPACITY with *needed, then the same
    call with a bigger buffer returns the kept answer (no second batch)."""
    import ctypes as C
    from dss_amd import _lib, geo, workload as W
    from dss_amd.store import Batcher, EntityIndex, _p
    _, q, qa, it, ia, now = W.config(0, scale=0.02)
    ci = geo.cover_batch(it.kind, it.voff, it.lat, it.lng, it.radius_m)
    idx = EntityIndex(ci.offs, ci.cells, ia.alt_lo, ia.alt_hi, ia.t0, ia.t1)
    b = Batcher(idx, max_batch=64, max_wait_us=0)
    L = b.L
    for i in range(q.n):  # a request with >= 2 answers
        v0, v1 = q.voff[i], q.voff[i + 1]
        st, ids = b.search_operations(q.kind[i], q.lat[v0:v1], q.lng[v0:v1], q.radius_m[i], qa.alt_lo[i],
                                      qa.alt_hi[i], qa.t0[i], qa.t1[i], now)
        if len(ids) >= 2:
            break
    assert len(ids) >= 2
    la = np.ascontiguousarray(q.lat[v0:v1])
    ln = np.ascontiguousarray(q.lng[v0:v1])
    out = np.empty(1, np.uint32)
    need, stt, area = C.c_int64(), C.c_int32(), C.c_double()
    args = lambda o, cap: (b.h, int(q.kind[i]), len(la), _p(la, C.c_double), _p(ln, C.c_double),  # noqa: E731
                           float(q.radius_m[i]), float(qa.alt_lo[i]), float(qa.alt_hi[i]), int(qa.t0[i]),
                           int(qa.t1[i]), int(now), _p(o, C.c_uint32), cap, C.byref(need), C.byref(stt),
                           C.byref(area))
    assert L.dssg_batcher_search_operations(*args(out, 1)) == _lib.DSSG_ERR_CAPACITY
    assert need.value == len(ids)
    area1 = area.value
    nreq0, _ = b.stats()
    out = np.empty(need.value, np.uint32)
    assert L.dssg_batcher_search_operations(*args(out, need.value)) == _lib.DSSG_OK
    assert np.array_equal(out, np.sort(ids)) and stt.value == 0 and area.value == area1
    assert b.stats()[0] == nreq0  # served from the kept answer
    b.close()
    idx.free()


def test_batcher_rejects_another_devices_index():
    import ctypes as C
    from dss_amd import _lib
    from dss_amd.store import EntityIndex
    idx = EntityIndex(np.array([0, 1]), np.array([0x808fb0ac00000000 | (1 << 34)], np.uint64))
    L = _lib.load()
    h = C.c_void_p()
    assert L.dssg_batcher_create(1, idx.h, 64, 0, C.byref(h)) == _lib.DSSG_ERR_INVALID
    idx.free()
