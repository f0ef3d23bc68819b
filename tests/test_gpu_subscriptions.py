"""GPU parity for the subscription-store queries:
notification fan-out, SCD owner-only subscription search (quirk Q7) and the
max-subscriptions-per-cell count -- the reference's own KATs restated, then
seeded random batches against the oracle restatements."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu

POOL_CELL = 12494535935418957824
OVERFLOW_CELL = 17106221850767130624
POOL_CELLS = [[OVERFLOW_CELL, POOL_CELL], [POOL_CELL], [POOL_CELL]]  # subscriptions_test.go:19-64
POOL_OWNER = [0, 0, 1]  # "myself", "myself", "me"
NOW = 1_600_000_000_000_000
DAY = 24 * 3600 * 10**6


def _pool_index():
    from dss_amd.store import EntityIndex
    return EntityIndex.from_lists(POOL_CELLS, t0=[NOW] * 3, t1=[NOW + DAY] * 3, owner=POOL_OWNER)


def test_max_subscription_count_kat():
    # subscriptions_test.go:275-287
    from dss_amd.store import MaxSubscriptionCountInCellsByOwner
    idx = _pool_index()
    assert MaxSubscriptionCountInCellsByOwner(idx, [POOL_CELL], 0, NOW) == 2
    assert MaxSubscriptionCountInCellsByOwner(idx, [POOL_CELL], 1, NOW) == 1
    assert MaxSubscriptionCountInCellsByOwner(idx, [OVERFLOW_CELL], 0, NOW) == 1
    assert MaxSubscriptionCountInCellsByOwner(idx, [OVERFLOW_CELL], 1, NOW) == 0   # IFNULL(MAX, 0)
    assert MaxSubscriptionCountInCellsByOwner(idx, [POOL_CELL], 0, NOW + 2 * DAY) == 0  # expired


def test_max_count_counts_repeats_in_stored_arrays():
    from dss_amd.store import EntityIndex, MaxSubscriptionCountInCellsByOwner
    idx = EntityIndex.from_lists([[POOL_CELL, POOL_CELL, OVERFLOW_CELL]], t1=[NOW + DAY], owner=[3])
    assert MaxSubscriptionCountInCellsByOwner(idx, [OVERFLOW_CELL, POOL_CELL, POOL_CELL], 3, NOW) == 2


def test_max_count_multiplicity_above_255():
    """A cell repeated more than 255 times in one stored array (ADVICE r5:
    the quad grain holds 8 bits per child): the build keeps the full count
    (it takes the cell grain), whether the grain is picked or forced to quads."""
    from dss_amd import _lib
    from dss_amd.store import EntityIndex, MaxSubscriptionCountInCellsByOwner
    sib = [(POOL_CELL & ~(3 << 35)) | (k << 35) for k in range(4)]  # the 4 level-13 cells of POOL_CELL's quad
    cells = [sib[0]] * 300 + sib[1:] + [sib[2]] * 2
    ctx = _lib.context()
    try:
        for grain in (0, 2):
            ctx.set_tuning("index_grain", grain)
            idx = EntityIndex.from_lists([cells, [sib[0]], sib], t1=[NOW + DAY] * 3, owner=[3, 3, 4])
            assert ctx.L.dssg_index_grain(idx.h) == 13, grain
            assert MaxSubscriptionCountInCellsByOwner(idx, [sib[0]], 3, NOW) == 301
            assert MaxSubscriptionCountInCellsByOwner(idx, [sib[2], sib[3]], 3, NOW) == 3
            assert MaxSubscriptionCountInCellsByOwner(idx, [sib[1]], 4, NOW) == 1
            idx.free()
    finally:
        ctx.set_tuning("index_grain", 0)


def test_notification_fanout_kat():
    # isa_test.go:266-324: 42 -> 43 on ISA insert -> 44 on ISA delete
    from dss_amd.store import UpdateNotificationIdxsInCells
    idx = _pool_index()
    idx.set_notification_index([42, 42, 42])
    rows = UpdateNotificationIdxsInCells(idx, [POOL_CELL], NOW)
    assert sorted(rows) == [(0, 43), (1, 43), (2, 43)]
    rows = UpdateNotificationIdxsInCells(idx, [POOL_CELL], NOW)
    assert sorted(rows) == [(0, 44), (1, 44), (2, 44)]
    assert idx.notification_index().tolist() == [44, 44, 44]
    # expired subscriptions are neither returned nor incremented
    assert UpdateNotificationIdxsInCells(idx, [POOL_CELL], NOW + 2 * DAY) == []
    assert idx.notification_index().tolist() == [44, 44, 44]


def test_scd_search_subscriptions_q7():
    from dss_amd.store import BadRequest, EntityIndex, SCDSearchSubscriptions
    idx = EntityIndex.from_lists([[POOL_CELL], [OVERFLOW_CELL], [POOL_CELL], [POOL_CELL]],
                                 t1=[NOW + DAY, NOW + DAY, NOW - 1, NOW + DAY], owner=[5, 5, 5, 6])
    # cells far from every subscription: still every unexpired one of the owner
    assert SCDSearchSubscriptions(idx, [0x1000000000000000 | (1 << 34)], 5, NOW) == [0, 1]
    assert SCDSearchSubscriptions(idx, [POOL_CELL], 6, NOW) == [3]
    assert SCDSearchSubscriptions(idx, [POOL_CELL], 7, NOW) == []
    with pytest.raises(BadRequest):
        SCDSearchSubscriptions(idx, [], 5, NOW)


def test_random_against_oracle(oracle):
    from dss_amd import geo, workload as W
    from dss_amd.store import EntityIndex
    _, q, qa, it, ia, now = W.config(0, scale=0.01)   # 100 queries, 1000 subscriptions
    rng = np.random.default_rng(11)
    ci = geo.cover_batch(it.kind, it.voff, it.lat, it.lng, it.radius_m)
    cq = geo.cover_batch(q.kind, q.voff, q.lat, q.lng, q.radius_m)
    owner = rng.integers(0, 7, it.n).astype(np.int32)
    t1 = ia.t1.copy()
    t1[rng.random(it.n) < 0.1] = np.iinfo(np.int64).min  # stored NULL ends_at: never matches (Q9)
    init = rng.integers(0, 100, it.n).astype(np.int64)
    idx = EntityIndex(ci.offs, ci.cells, ia.alt_lo, ia.alt_hi, ia.t0, t1, owner=owner)
    idx.set_notification_index(init)
    now_q = int(np.median(ia.t0))
    gq, ge, gv = idx.notify_batch(cq.offs, cq.cells, now_q)
    oq, oe, ov, cnt = oracle.notify(ci.offs, ci.cells, t1, init, cq.offs, cq.cells, now_q)
    assert len(oq) > 0
    assert np.array_equal(gq, oq) and np.array_equal(ge, oe) and np.array_equal(gv, ov)
    assert np.array_equal(idx.notification_index(), cnt)
    qown = rng.integers(0, 8, q.n).astype(np.int32)
    got = idx.max_subscription_count_batch(cq.offs, cq.cells, qown, now_q)
    want = oracle.max_subscription_count(ci.offs, ci.cells, owner, t1, cq.offs, cq.cells, qown, now_q)
    assert got.max() > 0 and np.array_equal(got, want)
    sq, se = idx.owner_subscriptions_batch(qown[:20], now_q)
    wq, we = oracle.owner_subscriptions(owner, t1, qown[:20], now_q)
    assert np.array_equal(sq, wq) and np.array_equal(se, we)


def test_store_max_count_kat_and_writes(oracle):
    """The GPU mirror's form (dssg_store_max_subscription_count, what the Go
    binding serves MaxSubscriptionCountInCellsByOwner from): the reference
    KAT (subscriptions_test.go:275-287) on a store, then random upserts,
    rewrites and deletes (rows split over the base, the delta and base
    tombstones) against the oracle over the live rows."""
    from dss_amd import geo, workload as W
    from dss_amd.store import Store
    st = Store(with_owner=True)
    st.upsert([0, 1, 2], POOL_CELLS, [-np.inf] * 3, [np.inf] * 3, [NOW] * 3, [NOW + DAY] * 3, owner=POOL_OWNER)
    cnt = lambda cells, ow, now: int(st.max_subscription_count_batch([0, len(cells)], cells, [ow], now)[0])  # noqa
    assert cnt([POOL_CELL], 0, NOW) == 2
    assert cnt([POOL_CELL], 1, NOW) == 1
    assert cnt([OVERFLOW_CELL], 1, NOW) == 0
    assert cnt([POOL_CELL], 0, NOW + 2 * DAY) == 0
    st.delete([1])
    assert cnt([POOL_CELL], 0, NOW) == 1
    st.upsert([1], [[POOL_CELL, POOL_CELL]], [0.0], [1.0], [NOW], [NOW + DAY], owner=[0])  # repeats count
    assert cnt([POOL_CELL], 0, NOW) == 3
    st.free()

    _, q, qa, it, ia, now = W.config(0, scale=0.02)   # 200 queries, 2000 subscriptions
    rng = np.random.default_rng(5)
    ci = geo.cover_batch(it.kind, it.voff, it.lat, it.lng, it.radius_m)
    cq = geo.cover_batch(q.kind, q.voff, q.lat, q.lng, q.radius_m)
    lists = [ci.cells[ci.offs[k]:ci.offs[k + 1]] for k in range(it.n)]
    owner = rng.integers(0, 5, it.n).astype(np.int32)
    t1 = ia.t1.copy()
    st = Store(with_owner=True)
    n0 = it.n // 2
    st.upsert(np.arange(n0), lists[:n0], ia.alt_lo[:n0], ia.alt_hi[:n0], ia.t0[:n0], t1[:n0], owner=owner[:n0])
    st.compact()  # the first half becomes the base
    rest = np.arange(n0, it.n)
    st.upsert(rest, [lists[k] for k in rest], ia.alt_lo[rest], ia.alt_hi[rest], ia.t0[rest], t1[rest],
              owner=owner[rest])
    rew = rng.choice(n0, 50, replace=False)  # base rows rewritten (tombstoned in the base, live in the delta)
    owner[rew] = rng.integers(0, 5, len(rew))
    st.upsert(rew, [lists[k] for k in rew], ia.alt_lo[rew], ia.alt_hi[rew], ia.t0[rew], t1[rew], owner=owner[rew])
    dead = rng.choice(it.n, 200, replace=False)
    st.delete(dead)
    live = np.ones(it.n, bool)
    live[dead] = False
    assert st.stats()["delta"] > 0
    qown = rng.integers(0, 6, q.n).astype(np.int32)
    now_q = int(np.median(ia.t0))
    got = st.max_subscription_count_batch(cq.offs, cq.cells, qown, now_q)
    keep = np.nonzero(live)[0]
    offs = np.concatenate([[0], np.cumsum([len(lists[k]) for k in keep])]).astype(np.int64)
    cells = np.concatenate([lists[k] for k in keep]).astype(np.uint64)
    want = oracle.max_subscription_count(offs, cells, owner[keep], t1[keep], cq.offs, cq.cells, qown, now_q)
    assert got.max() > 0 and np.array_equal(got, want)
    st.free()
