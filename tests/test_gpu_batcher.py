"""The per-request path (dssg_batcher): concurrent single searchOperations
requests, each an uncovered footprint, coalesced into shared batches; every
caller's answer equals a direct batch search of its own request, covering
errors come back as statuses."""
import threading

import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def test_batcher_matches_direct_search():
    from dss_amd import geo, workload as W
    from dss_amd.store import Batcher, EntityIndex
    _, q, qa, it, ia, now = W.config(0, scale=0.02)
    ci = geo.cover_batch(it.kind, it.voff, it.lat, it.lng, it.radius_m)
    idx = EntityIndex(ci.offs, ci.cells, ia.alt_lo, ia.alt_hi, ia.t0, ia.t1)
    cq = geo.cover_batch(q.kind, q.voff, q.lat, q.lng, q.radius_m)
    wq, we = idx.search_operations_batch(cq.offs, cq.cells, qa.alt_lo, qa.alt_hi, qa.t0, qa.t1, now)
    want = [we[wq == i] for i in range(q.n)]
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
        assert st == int(cq.status[i])
        assert np.array_equal(np.sort(ids), np.sort(want[i])), i
    nreq, nbatch = b.stats()
    assert nreq == q.n and nbatch < q.n  # requests really were coalesced
    # a covering error is a status, not an exception (the caller's BadRequest)
    st, ids = b.search_operations(1, [37.4], [-122.1], 0.0, 0, 100, 0, 10**12, now)
    assert st == 4 and len(ids) == 0  # DSSG_ST_RADIUS
    b.close()
    idx.free()
