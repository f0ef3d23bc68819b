"""GPU parity: the gfx950 index + overlap join == the reference semantics.

Restates the reference's DB-gated search KATs as fixtures
(pkg/rid/cockroach/identification_service_area_test.go:33-136, :160-194;
pkg/rid/cockroach/subscriptions_test.go:173-258) and checks every pair set
against the CPU oracle bit for bit (set equality of (query, entity) pairs).
"""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu

OVERFLOW = 17106221850767130624            # identification_service_area_test.go:19 (face-7 id, Q12)
CELLS = [17106221850767130624, 17106221885126868992, 17106221919486607360, OVERFLOW]
MIN = 60_000_000


def isa_index(start, end):
    from dss_amd.store import EntityIndex
    return EntityIndex.from_lists([CELLS], t0=[start], t1=[end])


@pytest.mark.parametrize("name,cells,mut,expected", [
    ("search for empty cell", [17106221953846345728], lambda s, e: (s, None), 0),
    ("search for only one cell", [17106221850767130624], lambda s, e: (s, None), 1),
    ("search for only one cell with high bit set", [OVERFLOW], lambda s, e: (s, None), 1),
    ("search with nil ends_at", CELLS, lambda s, e: (s, None), 1),
    ("search with exact timestamps", CELLS, lambda s, e: (s, e), 1),
    ("search with non-matching time span", CELLS, lambda s, e: (e + 100 * 1_000_000, e + 200 * 1_000_000), 0),
    ("search with expanded time span", CELLS, lambda s, e: (s - 100 * 1_000_000, e + 100 * 1_000_000), 1),
])
def test_store_search_isas(name, cells, mut, expected, join_path):
    # identification_service_area_test.go:33-136 (start = now-1min, end = now+1h)
    from dss_amd.store import SearchISAs
    now = 1_600_000_000_000_000
    start, end = now - MIN, now + 60 * MIN
    idx = isa_index(start, end)
    earliest, latest = mut(start, end)
    assert len(SearchISAs(idx, cells, earliest, latest)) == expected, name


def test_store_expired_isa():
    # identification_service_area_test.go:160-194
    from dss_amd.store import SearchISAs
    now = 1_600_000_000_000_000
    idx = isa_index(now - MIN, now + 60 * MIN)
    t = now + 59 * MIN
    assert len(SearchISAs(idx, CELLS, t, None)) == 1
    t = now + 61 * MIN
    assert len(SearchISAs(idx, CELLS, t, None)) == 0


def test_search_errors():
    from dss_amd.store import BadRequest, Internal, SearchISAs, SearchSubscriptions
    idx = isa_index(0, 10)
    with pytest.raises(BadRequest):
        SearchISAs(idx, [], 0, None)
    with pytest.raises(Internal):
        SearchISAs(idx, CELLS, None, None)
    with pytest.raises(BadRequest):
        SearchSubscriptions(idx, [], 0)


def test_subscriptions_by_owner(join_path):
    # subscriptions_test.go:172-216: 3 owners, subscription i covers cells[:i+1]
    # (the list holds a duplicate and a face-7 "overflow" id, Q12)
    from dss_amd.store import EntityIndex, SearchSubscriptions, SearchSubscriptionsByOwner
    now = 1_600_000_000_000_000
    cells = [12494535935418957824, 12494535866699481088, 12494535901059219456, 12494535866699481088, OVERFLOW]
    idx = EntityIndex.from_lists([cells[:i + 1] for i in range(3)], t0=[now] * 3, t1=[now + 24 * 3600 * 10**6] * 3,
                                 owner=[0, 1, 2])
    assert len(SearchSubscriptions(idx, cells, now)) == 3
    for o in range(3):
        assert SearchSubscriptionsByOwner(idx, cells, o, now) == [o]


def test_expired_subscription(join_path):
    # subscriptions_test.go:218-255: end = now + 24h; found at +23h, gone at +25h
    from dss_amd.store import EntityIndex, SearchSubscriptionsByOwner
    now = 1_600_000_000_000_000
    hour = 3600 * 10**6
    idx = EntityIndex.from_lists([[12494535866699481088]], t1=[now + 24 * hour], owner=[7])
    assert SearchSubscriptionsByOwner(idx, [12494535866699481088], 7, now + 23 * hour) == [0]
    assert SearchSubscriptionsByOwner(idx, [12494535866699481088], 7, now + 25 * hour) == []


def test_golden_operations(golden_search, join_path):
    from dss_amd.store import EntityIndex
    g = golden_search
    idx = EntityIndex(g["e_offs"], g["e_cells"], g["e_alt_lo"], g["e_alt_hi"], g["e_t0"], g["e_t1"], g["e_owner"])
    rq, re = idx.search_operations_batch(g["q_offs"], g["q_cells"], g["q_alt_lo"], g["q_alt_hi"], g["q_start"],
                                         g["q_end"], int(g["now"]))
    assert np.array_equal(rq, g["pairs_q"]) and np.array_equal(re, g["pairs_e"])
    sq, se = idx.search_subscriptions_batch(g["q_offs"], g["q_cells"], int(g["now"]), g["q_owner"])
    assert np.array_equal(sq, g["subs_q"]) and np.array_equal(se, g["subs_e"])


def test_random_end_to_end(oracle, join_path):
    """Cover intents and queries on the GPU, build the index, join; compare
    with the oracle's covering + join on the same seeded inputs."""
    from dss_amd import geo, workload as W
    from dss_amd.store import EntityIndex
    _, q, qa, it, ia, now = W.config(0, scale=0.05)
    ci = geo.cover_batch(it.kind, it.voff, it.lat, it.lng, it.radius_m)
    cq = geo.cover_batch(q.kind, q.voff, q.lat, q.lng, q.radius_m)
    io, ic, _, _ = oracle.cover_batch(it.kind, it.voff, it.lat, it.lng, it.radius_m)
    qo, qc, _, _ = oracle.cover_batch(q.kind, q.voff, q.lat, q.lng, q.radius_m)
    assert np.array_equal(ci.cells, ic) and np.array_equal(cq.cells, qc)
    idx = EntityIndex(ci.offs, ci.cells, ia.alt_lo, ia.alt_hi, ia.t0, ia.t1)
    rq, re = idx.search_operations_batch(cq.offs, cq.cells, qa.alt_lo, qa.alt_hi, qa.t0, qa.t1, now)
    tlo = np.maximum(qa.t0, now)
    oq, oe = oracle.search(io, ic, ia.alt_lo, ia.alt_hi, ia.t0, ia.t1, None, qo, qc, qa.alt_lo, qa.alt_hi, tlo, qa.t1)
    assert len(oq) > 0
    assert np.array_equal(rq, oq) and np.array_equal(re, oe)


def test_unsorted_duplicate_query_cells(oracle, golden_search, join_path):
    """UnionVolumes4D hands the store unsorted cells (Q14); duplicates too."""
    from dss_amd.store import EntityIndex
    g = golden_search
    idx = EntityIndex(g["e_offs"], g["e_cells"], g["e_alt_lo"], g["e_alt_hi"], g["e_t0"], g["e_t1"])
    offs, cells = g["q_offs"], g["q_cells"]
    rng = np.random.default_rng(5)
    lists = []
    for i in range(len(offs) - 1):
        c = list(cells[offs[i]:offs[i + 1]])
        c = c + c[: len(c) // 2]
        rng.shuffle(c)
        lists.append(c)
    no = np.zeros(len(lists) + 1, np.int64)
    np.cumsum([len(c) for c in lists], out=no[1:])
    nc = np.array([x for c in lists for x in c], dtype=np.uint64)
    rq, re = idx.search_operations_batch(no, nc, g["q_alt_lo"], g["q_alt_hi"], g["q_start"], g["q_end"],
                                         int(g["now"]))
    assert np.array_equal(rq, g["pairs_q"]) and np.array_equal(re, g["pairs_e"])


def test_device_api_matches_host_api(golden_covering):
    """dssg_*_device over torch-allocated HBM buffers == host API."""
    import torch
    from dss_amd import _lib, device as D, geo, workload as W
    ctx = _lib.context()
    rng = np.random.default_rng(9)
    fp = W.metro_footprints(rng, 5000)
    dfp = D.DeviceFootprints.upload(fp)
    cells = D.cover(ctx, dfp)
    offs = D.copy_back(ctx, cells.offs, fp.n + 1, np.int64)
    got = D.copy_back(ctx, cells.cells, int(offs[-1]), np.uint64)
    ref = geo.cover_batch(fp.kind, fp.voff, fp.lat, fp.lng, fp.radius_m)
    assert np.array_equal(offs, ref.offs) and np.array_equal(got, ref.cells)
    ia = W.intent_attrs(rng, fp.n)
    t = lambda a: torch.as_tensor(a, device="cuda")  # noqa: E731
    idx = D.build_index(ctx, cells, t(ia.alt_lo), t(ia.alt_hi), t(ia.t0), t(ia.t1))
    qa = W.query_attrs(rng, fp.n)
    tlo = np.maximum(qa.t0, W.T0_US)
    pairs = D.search(ctx, idx, cells, t(qa.alt_lo), t(qa.alt_hi), t(tlo), t(qa.t1))
    torch.cuda.synchronize()
    q = D.copy_back(ctx, pairs.q, pairs.n, np.uint32)
    e = D.copy_back(ctx, pairs.e, pairs.n, np.uint32)
    ctx.L.dssg_index_free(idx)
    from dss_amd.store import EntityIndex
    hidx = EntityIndex(ref.offs, ref.cells, ia.alt_lo, ia.alt_hi, ia.t0, ia.t1)
    hq, he = hidx.search_batch(ref.offs, ref.cells, qa.alt_lo, qa.alt_hi, tlo, qa.t1)
    key = np.sort((q.astype(np.uint64) << np.uint64(32)) | e.astype(np.uint64))
    hkey = (hq.astype(np.uint64) << np.uint64(32)) | he.astype(np.uint64)
    assert np.array_equal(key, hkey)


@pytest.mark.parametrize("nq,ne,span_h,dur", [
    (3000, 6000, 24, "mixed"),     # long runs: > 64 records and > 64 postings per cell
    (64, 4096, 24, "mixed"),       # exactly one 64-record batch
    (130, 130, 2, "mixed"),        # run lengths around the 64 boundaries
    (2000, 3000, 1, "short"),      # RID-like 30 s windows, dense in time
    (500, 3000, 24, "long"),       # many long-duration entities (the long part of a cell)
])
def test_hot_cell_band_join(oracle, nq, ne, span_h, dur, join_path):
    """Hot cells: every footprint within a few level-13 cells, so one cell's
    records and postings span many 64-wide tiles and batches; the band join's
    record ranges (cooperative 64-ary search over start-sorted records), tile
    bounds and long-duration postings against the oracle."""
    from dss_amd.store import EntityIndex
    rng = np.random.default_rng(nq * 7 + ne)
    T, H, M = 1_600_000_000_000_000, 3_600_000_000, 60_000_000
    cells = np.array([oracle.cellid_from_degrees(37.5 + 0.01 * i, -122.2) for i in range(3)], dtype=np.uint64)

    def lists(n):
        k = rng.integers(1, 4, n)
        offs = np.zeros(n + 1, np.int64)
        np.cumsum(k, out=offs[1:])
        c = np.concatenate([np.sort(rng.choice(cells, int(x), replace=False)) for x in k])
        return offs, c.astype(np.uint64)

    eo, ec = lists(ne)
    qo, qc = lists(nq)
    e_t0 = T + rng.integers(0, span_h * H, ne)
    if dur == "short":
        e_t1 = e_t0 + 30_000_000
    elif dur == "long":
        e_t1 = e_t0 + np.where(rng.random(ne) < 0.3, rng.integers(10 * H, 30 * H, ne), rng.integers(5 * M, 2 * H, ne))
    else:
        e_t1 = e_t0 + rng.integers(5 * M, 2 * H, ne)
    e_lo = rng.uniform(0, 400, ne).astype(np.float32)
    e_hi = (e_lo + rng.uniform(10, 200, ne)).astype(np.float32)
    q_t0 = T + rng.integers(0, span_h * H, nq)
    q_t1 = q_t0 + (30_000_000 if dur == "short" else rng.integers(1 * M, 30 * M, nq))
    wide = rng.random(nq) < 0.05  # NULL end -> a wide window
    q_t1 = np.where(wide, np.iinfo(np.int64).max, q_t1)
    q_lo = rng.uniform(0, 400, nq).astype(np.float32)
    q_hi = (q_lo + rng.uniform(10, 200, nq)).astype(np.float32)
    idx = EntityIndex(eo, ec, e_lo, e_hi, e_t0, e_t1)
    rq, re = idx.search_operations_batch(qo, qc, q_lo, q_hi, q_t0, q_t1, T)
    tlo = np.maximum(q_t0, T)
    oq, oe = oracle.search(eo, ec, e_lo, e_hi, e_t0, e_t1, None, qo, qc, q_lo, q_hi, tlo, q_t1)
    assert len(oq) > 0
    assert np.array_equal(rq, oq) and np.array_equal(re, oe)
