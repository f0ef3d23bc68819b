"""GPU parity on the other BASELINE.json configs, at sizes
the oracle finishes in seconds: California hotspots (configs[2]), RID
city-block ISAs with 30 s windows (configs[3], SearchISAs semantics: no
altitude, identification_service_area.go:170-180) and continent-scale thin
corridors (configs[4]).  Coverings must be bit-identical and the pair sets
equal to the oracle's."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def _keys(q, e):
    return np.sort((np.asarray(q, np.uint64) << np.uint64(32)) | np.asarray(e, np.uint64))


# (2, 0.1): 1M California intents and 100k queries -- hotspot cells with
# hundreds of postings and records, and a few long footprints, so both join
# queues (short and long variants) run in one search
@pytest.mark.parametrize("cfg,scale", [(1, 0.02), (2, 0.002), (3, 0.004), (4, 0.0004), (2, 0.1), (3, 0.1),
                                       (4, 0.01)])
def test_config_parity(oracle, cfg, scale, join_path):
    from dss_amd import geo, workload as W
    from dss_amd.store import EntityIndex
    _, q, qa, it, ia, now = W.config(cfg, scale=scale)
    ci = geo.cover_batch(it.kind, it.voff, it.lat, it.lng, it.radius_m)
    cq = geo.cover_batch(q.kind, q.voff, q.lat, q.lng, q.radius_m)
    io, ic, ist, _ = oracle.cover_batch(it.kind, it.voff, it.lat, it.lng, it.radius_m)
    qo, qc, qst, _ = oracle.cover_batch(q.kind, q.voff, q.lat, q.lng, q.radius_m)
    assert np.array_equal(ci.offs, io) and np.array_equal(ci.cells, ic)
    assert np.array_equal(cq.offs, qo) and np.array_equal(cq.cells, qc)
    assert np.array_equal(ci.status, ist) and np.array_equal(cq.status, qst)
    tlo, thi = W.query_bounds(qa, now)
    idx = EntityIndex(ci.offs, ci.cells, ia.alt_lo, ia.alt_hi, ia.t0, ia.t1)
    if cfg == 3:
        gq, ge = idx.search_isas_batch(cq.offs, cq.cells, tlo, thi)
    else:
        gq, ge = idx.search_operations_batch(cq.offs, cq.cells, qa.alt_lo, qa.alt_hi, qa.t0, qa.t1, now)
    oq, oe = oracle.search(io, ic, ia.alt_lo, ia.alt_hi, ia.t0, ia.t1, None, qo, qc, qa.alt_lo, qa.alt_hi, tlo, thi)
    assert len(oq) > 0
    assert np.array_equal(_keys(gq, ge), _keys(oq, oe))
    if (cfg, scale) == (2, 0.1):
        assert idx.info()["long_footprint_postings"] > 0  # the long queue is exercised


# The posting grain forced both ways (the build picks one per index: quads
# for metro / California / corridor footprints, cells for city blocks):
# identical pair sets, on every join path's default shape.
@pytest.mark.parametrize("grain", [1, 2])
@pytest.mark.parametrize("cfg,scale", [(1, 0.02), (2, 0.1), (3, 0.1), (4, 0.01)])
def test_config_parity_both_grains(oracle, cfg, scale, grain):
    from dss_amd import _lib, geo, workload as W
    from dss_amd.store import EntityIndex
    _, q, qa, it, ia, now = W.config(cfg, scale=scale)
    ci = geo.cover_batch(it.kind, it.voff, it.lat, it.lng, it.radius_m)
    cq = geo.cover_batch(q.kind, q.voff, q.lat, q.lng, q.radius_m)
    tlo, thi = W.query_bounds(qa, now)
    ctx = _lib.context(0)
    ctx.set_tuning("index_grain", grain)
    try:
        idx = EntityIndex(ci.offs, ci.cells, ia.alt_lo, ia.alt_hi, ia.t0, ia.t1)
    finally:
        ctx.set_tuning("index_grain", 0)
    assert ctx.L.dssg_index_grain(idx.h) == (13 if grain == 1 else 12)
    if cfg == 3:
        gq, ge = idx.search_isas_batch(cq.offs, cq.cells, tlo, thi)
    else:
        gq, ge = idx.search_operations_batch(cq.offs, cq.cells, qa.alt_lo, qa.alt_hi, qa.t0, qa.t1, now)
    oq, oe = oracle.search(ci.offs, ci.cells, ia.alt_lo, ia.alt_hi, ia.t0, ia.t1, None, cq.offs, cq.cells, qa.alt_lo,
                           qa.alt_hi, tlo, thi)
    assert len(oq) > 0
    assert np.array_equal(_keys(gq, ge), _keys(oq, oe))


# The round-6 index / join options away from their defaults (4 altitude
# bands from 4096 postings per group and records in key order from 8192,
# which the small test airspaces never reach): bands off, 8 bands from 256
# postings, 4 from 64 and from 1024, records in query or in key order --
# identical pair sets to the oracle's.
@pytest.mark.parametrize("opts", [{"index_bands": 1}, {"index_bands": 8, "band_dense": 256}, {"band_dense": 64},
                                  {"band_dense": 1024}, {"record_order": 1}, {"record_order": 2},
                                  {"band_dense": 64, "record_order": 2}])
@pytest.mark.parametrize("cfg,scale", [(2, 0.1), (4, 0.01)])
def test_join_options_parity(oracle, cfg, scale, opts):
    from dss_amd import _lib, geo, workload as W
    from dss_amd.store import EntityIndex
    _, q, qa, it, ia, now = W.config(cfg, scale=scale)
    ci = geo.cover_batch(it.kind, it.voff, it.lat, it.lng, it.radius_m)
    cq = geo.cover_batch(q.kind, q.voff, q.lat, q.lng, q.radius_m)
    tlo, thi = W.query_bounds(qa, now)
    ctx = _lib.context(0)
    defaults = {"index_bands": 4, "band_dense": 4096, "record_order": 0}
    try:
        for k, v in opts.items():
            ctx.set_tuning(k, v)
        idx = EntityIndex(ci.offs, ci.cells, ia.alt_lo, ia.alt_hi, ia.t0, ia.t1)
        gq, ge = idx.search_operations_batch(cq.offs, cq.cells, qa.alt_lo, qa.alt_hi, qa.t0, qa.t1, now)
    finally:
        for k in opts:
            ctx.set_tuning(k, defaults[k])
    oq, oe = oracle.search(ci.offs, ci.cells, ia.alt_lo, ia.alt_hi, ia.t0, ia.t1, None, cq.offs, cq.cells, qa.alt_lo,
                           qa.alt_hi, tlo, thi)
    assert len(oq) > 0
    assert np.array_equal(_keys(gq, ge), _keys(oq, oe))
    # the per-request small join (<= 4096 queries) over the same index: each
    # band's m range searched separately
    k = 300
    sq, se = idx.search_operations_batch(cq.offs[:k + 1], cq.cells[:int(cq.offs[k])], qa.alt_lo[:k], qa.alt_hi[:k],
                                         qa.t0[:k], qa.t1[:k], now)
    sel = oq < k
    assert np.array_equal(_keys(sq, se), _keys(oq[sel], oe[sel]))
    idx.free()


def test_grain_picked_by_footprint_shape():
    """Auto grain: quads for metro footprints (~6 cells, ~2 per quad), cells
    for RID city blocks (~1.4 cells, ~1.2 per quad)."""
    from dss_amd import _lib, geo, workload as W
    from dss_amd.store import EntityIndex
    ctx = _lib.context(0)
    for cfg, want in ((1, 12), (3, 13)):
        _, q, qa, it, ia, now = W.config(cfg, scale=0.01)
        ci = geo.cover_batch(it.kind, it.voff, it.lat, it.lng, it.radius_m)
        idx = EntityIndex(ci.offs, ci.cells, ia.alt_lo, ia.alt_hi, ia.t0, ia.t1)
        assert ctx.L.dssg_index_grain(idx.h) == want, cfg


@pytest.fixture(scope="module")
def corridors_case(oracle):
    """configs[4] corridors at a scale with ~45k long x long occurrences."""
    from dss_amd import geo, workload as W
    _, q, qa, it, ia, now = W.config(4, scale=0.003)
    ci = geo.cover_batch(it.kind, it.voff, it.lat, it.lng, it.radius_m)
    cq = geo.cover_batch(q.kind, q.voff, q.lat, q.lng, q.radius_m)
    tlo, thi = W.query_bounds(qa, now)
    oq, oe = oracle.search(ci.offs, ci.cells, ia.alt_lo, ia.alt_hi, ia.t0, ia.t1, None, cq.offs, cq.cells, qa.alt_lo,
                           qa.alt_hi, tlo, thi)
    return ci, cq, qa, ia, now, _keys(oq, oe)


# tag_bucket_avg: 1024 (default buckets), 1 (hb capped by the pair count: tiny
# buckets), 2^40 (two buckets, each over the LDS set: the full-sort fallback
# for flagged buckets), 0 (the full-sort path)
@pytest.mark.parametrize("avg", [1024, 1, 1 << 40, 0])
def test_long_pair_dedupe_paths(corridors_case, avg, join_path):
    from dss_amd import _lib
    from dss_amd.store import EntityIndex
    ci, cq, qa, ia, now, want = corridors_case
    ctx = _lib.context(0)
    ctx.set_tuning("tag_bucket_avg", avg)
    try:
        idx = EntityIndex(ci.offs, ci.cells, ia.alt_lo, ia.alt_hi, ia.t0, ia.t1)
        gq, ge = idx.search_operations_batch(cq.offs, cq.cells, qa.alt_lo, qa.alt_hi, qa.t0, qa.t1, now)
    finally:
        ctx.set_tuning("tag_bucket_avg", 1024)
    got = _keys(gq, ge)
    assert len(got) > 0 and np.all(got[1:] != got[:-1])
    assert np.array_equal(got, want)


# lazy_sig_recs: 0 (every unit prefetches the posting signatures), 2^30 (every
# unit loads them per lane on first need) -- the same pairs either way
@pytest.mark.parametrize("lazy", [0, 1 << 30])
def test_lazy_signature_paths(corridors_case, lazy):
    from dss_amd import _lib
    from dss_amd.store import EntityIndex
    ci, cq, qa, ia, now, want = corridors_case
    ctx = _lib.context(0)
    ctx.set_tuning("lazy_sig_recs", lazy)
    try:
        idx = EntityIndex(ci.offs, ci.cells, ia.alt_lo, ia.alt_hi, ia.t0, ia.t1)
        gq, ge = idx.search_operations_batch(cq.offs, cq.cells, qa.alt_lo, qa.alt_hi, qa.t0, qa.t1, now)
    finally:
        ctx.set_tuning("lazy_sig_recs", 0)
    got = _keys(gq, ge)
    assert len(got) > 0 and np.all(got[1:] != got[:-1])
    assert np.array_equal(got, want)
