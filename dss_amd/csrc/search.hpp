// Host-side driver of the entity index and the 4D overlap join (search.hip).
#pragma once
#include "common.hpp"

// HBM-resident entity index.  One posting per (entity, group)
// of the cell range this index serves (a group: a quad or a level-13 cell, by
// gshift), sorted by
//   (slot, duration class, altitude band, m = min(t0, t1)):
// a group's postings are contiguous; within it the "regular" postings (entity
// duration |t1 - t0| <= dcap_thr) come first -- in one run, or in a dense
// group in n_bands runs by alt_lo quantile -- each run sorted by start time
// m, then the long-duration ones.  A query window [tlo, thi] can only meet a
// regular posting with m in [tlo - dcap, thi] -- one contiguous range per run
// (the band join of search.hip) -- and every long posting of the group.
struct dssg_index {
    int64_t n_e = 0;        // entities
    int64_t n_p = 0;        // postings held (unique (cell, entity) in range, ends_at not NULL)
    int64_t n_cells = 0;    // distinct cells with postings
    int64_t n_long = 0;     // postings of long-duration entities
    int64_t n_long_fp = 0;  // postings of long footprints (b_meta kMetaLongFp)
    int64_t max_cell_postings = 0;
    uint64_t cell_lo = 0, cell_hi = ~0ull;  // cell range of the postings held (shards)
    bool has_owner = false;
    // ---- cell -> slot ---------------------------------------------------------
    // valid level-13 ids: slot = (cell >> 35) - kmin when < n_dense; any other
    // id (the reference tests use invalid face-7 ids as opaque keys, Q12):
    // n_dense + its index in the sorted irr_cells.
    uint64_t kmin = 0;
    int64_t n_dense = 0;
    int64_t n_irr = 0;
    dss::DevBuf<uint64_t> irr_cells;  // n_irr, sorted
    dss::DevBuf<uint64_t> s_post;     // n_slots + 1: first posting of each slot
    dss::DevBuf<uint32_t> s_nreg;     // n_slots: regular-duration postings of the slot
    dss::DevBuf<uint8_t> s_lfp;       // n_slots: 1 = the slot holds a long-footprint posting (join variant)
    // altitude bands (n_bands > 1): a slot with >= band_dense postings keeps its
    // regular postings as n_bands runs by alt_lo (global quantiles), each in
    // m order; s_band[8 * slot + b] = start of band b relative to s_post[slot]
    // (band b ends where b + 1 starts, the last at s_nreg); other slots: one run
    dss::DevBuf<uint32_t> s_band;     // 8 * n_slots (n_bands > 1)
    int n_bands = 1;
    // ---- time --------------------------------------------------------------------
    int64_t dcap = 0;      // max duration of a regular posting's entity (us)
    int gshift = 37;       // posting groups: cell >> gshift (37: quads = level-12 cells, 35: level-13 cells)
    int64_t dcap_thr = 0;  // class threshold: duration <= dcap_thr is regular
    int64_t tbase = 0;     // query-order quantisation: (tlo - tbase) >> qshift
    int qshift = 0;
    // ---- postings ----------------------------------------------------------------
    dss::DevBuf<uint32_t> b_e;      // entity | kFirstBit (the cell is the entity's smallest)
    dss::DevBuf<uint8_t> b_meta;    // kMetaCompact | kMetaLongFp
    dss::DevBuf<float2> b_alt;      // (alt_lo, alt_hi)
    dss::DevBuf<longlong2> b_t;     // (t0, t1) microseconds
    dss::DevBuf<ulonglong2> b_sig;  // 2 per posting: 256-bit near-prefix signature
    dss::DevBuf<int32_t> b_owner;   // has_owner
    dss::DevBuf<uint32_t> b_mult;   // times (cell, entity) occurs in the stored array (has_mult)
    bool has_mult = false;
    // ---- entities ------------------------------------------------------------------
    dss::DevBuf<int64_t> e_offs;    // entity -> sorted unique cells (all of them, any range)
    dss::DevBuf<uint64_t> e_cells;
    dss::DevBuf<int64_t> e_t1;      // ends_at (us)
    dss::DevBuf<int32_t> e_owner;   // owner id (has_owner)
    dss::DevBuf<uint32_t> o_key;    // owner ^ 0x80000000, ascending (owner -> entities)
    dss::DevBuf<uint32_t> o_ent;    // entity ids in o_key order
    dss::DevBuf<int64_t> e_notify;  // notification_index counters
    // tombstones (write path, store.hip): bit e set = entity e is deleted or
    // superseded; the join and the subscription queries skip it
    dss::DevBuf<uint32_t> dead;
    bool has_dead = false;
    int device = 0;
    int64_t n_slots() const { return n_dense + n_irr; }
};

namespace dss {

class SearchEngine {
   public:
    SearchEngine() = default;
    SearchEngine(const SearchEngine &) = delete;
    SearchEngine &operator=(const SearchEngine &) = delete;
    ~SearchEngine()
    {
        if (mail_h_) (void)hipHostFree(mail_h_);
    }
    // Postings are kept only for cells in [cell_lo, cell_hi] (a cell-range
    // shard); entity cell lists stay whole, so the smallest-shared-cell rule
    // emits every pair on exactly one shard (long x long pairs: see search()).
    void build(dssg_index *idx, int64_t n, const int64_t *cell_offs, const uint64_t *cells, const float *alt_lo,
               const float *alt_hi, const int64_t *t0, const int64_t *t1, const int32_t *owner, uint64_t cell_lo,
               uint64_t cell_hi, hipStream_t s);
    // q cells must be sorted ascending and unique per query.  Output: every
    // matching (query, entity) pair once; out->n_tagged of them (the last
    // ones) are long x long pairs, deduplicated after the join (on a
    // cell-range shard: kept only by the shard of their smallest shared cell,
    // so each comes back once across shards).
    // nqc >= 0: the batch's cell count q_offs[nq], known to the caller (no
    // read back before the join).
    void search(const dssg_index *idx, int64_t nq, const int64_t *q_offs, const uint64_t *q_cells,
                const float *q_alt_lo, const float *q_alt_hi, const int64_t *q_tlo, const int64_t *q_thi,
                const int32_t *q_owner, hipStream_t s, dssg_pairs *out, int64_t nqc = -1);
    // Roofline accounting: postings scanned and distinct candidate entities
    // (predicate disabled), i.e. sum_q M_q and sum_q D_q of SURVEY s8(d).
    void stats(const dssg_index *idx, int64_t nq, const int64_t *q_offs, const uint64_t *q_cells, hipStream_t s,
               int64_t *matched, int64_t *distinct);
    // Postings of the distinct cells the batch touches, each once.
    int64_t touched(const dssg_index *idx, int64_t nq, const int64_t *q_offs, const uint64_t *q_cells, hipStream_t s);
    void set_timing(bool on) { timing_ = on; }
    // tuning: average tagged pairs per dedupe bucket (<= 0: the full-sort path)
    void set_tag_bucket_avg(int64_t v) { tag_bucket_avg_ = v; }
    // join units with at most this many records load the posting signatures
    // only for the lanes that need them (0: always prefetched)
    void set_lazy_sig_recs(int64_t v) { lazy_sig_recs_ = v; }
    // k_join's occupancy / pair-stage shape: 0 picks by the previous batch's
    // pass density, 1 forces 7 x 640, 2 forces 6 x 1024
    void set_join_shape(int v) { join_shape_ = v; }
    // posting grain of the next builds: 0 picks per build (quads when an
    // entity's cells fill them: >= 1.5 cells per (entity, quad)), 1 level-13
    // cells, 2 quads (level-12 cells)
    void set_grain(int v) { grain_ = v; }
    // altitude bands of the dense slots of later builds (1: none; 2..8) and the
    // slot size from which they apply
    void set_bands(int nb, int64_t dense)
    {
        bands_ = nb;
        band_dense_ = dense;
    }
    int bands() const { return bands_; }
    void set_rec_order(int v) { rec_order_ = v; }
    int64_t band_dense() const { return band_dense_; }
    double last_join_kernel_ms() const { return join_ms_; }
    int64_t last_units() const { return units_; }
    int64_t last_keys() const { return keys_; }
    int64_t last_tagged() const { return tagged_; }  // long x long pair occurrences before the dedupe
    void last_longs(int64_t *lq, int64_t *lp) const
    {
        *lq = long_queries_;
        *lp = long_postings_;
    }
    // Hands the engine-owned buffers holding `res` (the most recent result)
    // to the caller in exchange for (q, e), which later searches reuse: the
    // result then outlives the next search (the async sharded step's
    // alternating buffer sets).  false if `res` is not in the engine's buffers.
    bool adopt_output(const dssg_pairs &res, DevBuf<uint32_t> &q, DevBuf<uint32_t> &e)
    {
        auto give = [&](DevBuf<uint32_t> &a, DevBuf<uint32_t> &b) {
            if (res.q != a.p || res.e != b.p) return false;
            std::swap(a.p, q.p);
            std::swap(a.cap, q.cap);
            std::swap(b.p, e.p);
            std::swap(b.cap, e.cap);
            return true;
        };
        return give(oq_, oe_) || give(oq2_, oe2_);
    }
    void last_join_events(int64_t *flushes, int64_t *merges, int64_t *merge_lanes) const
    {
        *flushes = flushes_;
        *merges = merges_;
        *merge_lanes = merge_lanes_;
    }
    // runs = 0 (kept for the ABI); iters = record broadcasts (wave
    // iterations); tests = record x posting lane tests
    void last_work(int64_t *runs, int64_t *iters, int64_t *tests) const
    {
        *runs = runs_;
        *iters = iters_;
        *tests = tests_;
    }

    // batches of at most this many queries (and 16x as many cells) take the
    // one-launch small path (k_small_join); 0: never
    void set_small_max_q(int64_t v) { small_max_q_ = v; }

    // The one-launch small-batch join (k_small_join) with the batch's cell
    // count nqc known to the caller (no fetch of q_offs[nq]).
    void search_small(const dssg_index *idx, int64_t nq, const int64_t *q_offs, const uint64_t *q_cells,
                      const float *q_alt_lo, const float *q_alt_hi, const int64_t *q_tlo, const int64_t *q_thi,
                      const int32_t *q_owner, int64_t nqc, hipStream_t s, dssg_pairs *out);
    int64_t small_max_q() const { return small_max_q_; }

   private:
    int64_t small_max_q_ = 4096, small_cap_ = 0;
    DevBuf<unsigned long long> small_cnt_;
    DevBuf<unsigned char> tmp_, tmp2_;
    // query side
    DevBuf<uint32_t> cq_, dec_, okey_, okey2_, oval_, perm_, kkey_, kkey2_, rbeg_, bt_;
    DevBuf<int64_t> qcnt_, qoff_, rcnt_, roff_, ucnt_, uoff_, cnt64_;
    DevBuf<uint64_t> kv64_, kv64b_;  // query-cell keys' values: cell | quantised start << 32
    DevBuf<uint8_t> qlong_;
    DevBuf<unsigned char> rec_, rec2_, units_buf_, batch_buf_;  // rec2_: the records in key order
    DevBuf<unsigned long long> counter_, regcnt_;
    DevBuf<uint32_t> oq_, oe_, oq2_, oe2_, fills_;
    DevBuf<unsigned long long> work_;
    DevBuf<unsigned long long> tkey_, tkey2_;
    DevBuf<uint32_t> vpre_, qaux_;  // query cells: rank among the query's cells with postings; per query aux
    DevBuf<int64_t> tb_;   // tag buckets: starts, ends, distinct counts, offsets
    DevBuf<uint8_t> tovf_;  // tag buckets too large for the LDS set
    int n_cu_ = 0;
    int64_t out_rcap_ = 0;  // output slots per region
    int64_t tag_rcap_ = 0;  // tagged-key slots per region
    int64_t units_cap_hint_ = 0, units_cap_hint_l_ = 0;
    int64_t long_units_prev_ = INT64_MAX / 2;  // the previous batch's long-variant units (sizes its launch)
    // the join's control words, gathered into fine-grained host memory
    int64_t *mail_h_ = nullptr, *mail_d_ = nullptr;
    int64_t *mailbox();
    int occ_long_ = 0;                         // long-variant workgroups per CU
    bool timing_ = false;
    int64_t tag_bucket_avg_ = 2048;
    int64_t lazy_sig_recs_ = 0;
    bool dense_out_ = false;  // the previous batch's pass density was high: k_join's 6 x 1024-pair stage shape
    int join_shape_ = 0;      // 0: by dense_out_; 1: the sparse shape; 2: the dense shape (tests)
    int grain_ = 0;           // 0: auto; 1: cells; 2: quads
    int bands_ = 4;           // altitude bands of dense slots (1: none) -- DESIGN.md s4
    int rec_order_ = 0;        // join records: 0 auto (key order for indexes with groups >= 8192 postings), 1 query, 2 key
    int64_t band_dense_ = 4096;  // (1024 banded configs[1]'s ~3k-posting quads: k_join 0.90 -> 1.01 ms)
    double join_ms_ = 0;
    int64_t units_ = 0, keys_ = 0, runs_ = 0, iters_ = 0, tests_ = 0;
    int64_t flushes_ = 0, merges_ = 0, merge_lanes_ = 0, tagged_ = 0, long_queries_ = 0, long_postings_ = 0;
    hipEvent_t ev0_ = nullptr, ev1_ = nullptr;
    void timing_events();
};

// The counting build's per-lane-test outcome sums over every k_join launch
// since the last read (DSS_JOIN_PROFILE, search.hip); cleared by the read.
// Returns the number of counters written (0 in the shipped library); their
// names through join_profile_name(i).
int join_profile_read(int64_t *out, int n);
const char *join_profile_name(int i);

}  // namespace dss
