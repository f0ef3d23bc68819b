// Host-side driver of the entity index and the 4D overlap join (search.hip).
#pragma once
#include "common.hpp"

struct dssg_index {
    int64_t n_e = 0;      // entities
    int64_t n_p = 0;      // unique (cell, entity) postings
    int64_t n_reg = 0;    // of which on valid level-13 cells (dense lookup)
    int64_t n_cells = 0;  // distinct cells
    int64_t n_b = 0;      // time-bucketed postings (the join's working set)
    int64_t n_long_b = 0; // of which of long footprints (b_meta 0x40)
    uint64_t cell_lo = 0, cell_hi = ~0ull;  // cell range of the postings held (shards)
    bool has_owner = false;
    // ---- plain postings, sorted by (cell, entity); regular first -------------
    // A cell's "slot" is its dense slot (level-13 cells) or n_dense + its index
    // in the irregular side table.
    dss::DevBuf<uint64_t> p_cell;
    dss::DevBuf<uint32_t> p_e;  // bit 31: the cell is the entity's smallest cell
    dss::DevBuf<uint32_t> p_mult;  // times (cell, entity) occurs in the stored cell array (RID
                                   // `unnest(cells)` counts repeats, subscriptions.go:94-101)
    uint64_t kmin = 0;          // dense slot k <-> cell (kmin + k) << 35 | 1 << 34
    int64_t n_dense = 0;
    dss::DevBuf<uint32_t> dense;  // n_dense + 1 plain posting offsets
    int64_t n_irr = 0;
    dss::DevBuf<uint64_t> irr_cells;  // sorted, n_irr
    dss::DevBuf<uint32_t> irr_start;  // n_irr + 1, absolute plain offsets
    // entity -> sorted unique cells (smallest-shared-cell rule)
    dss::DevBuf<int64_t> e_offs;
    dss::DevBuf<uint64_t> e_cells;
    // ---- time buckets ---------------------------------------------------------
    // bucket(t) = clamp((t - tbase) >> shift, 0, nb - 1), nb <= 61; bucket 63
    // holds, once, the entities spanning more than kLongSpan buckets.
    int64_t tbase = 0;
    int shift = 0;
    int nb = 1;
    // ---- bucketed postings, sorted by (slot, bucket, entity) -----------------
    // Group g = one non-empty (slot, bucket); g = s_base[slot] +
    // popcount(s_mask[slot] & ((1 << bucket) - 1)); postings [bk_start[g], bk_start[g+1]).
    dss::DevBuf<unsigned long long> s_mask;  // n_slots
    dss::DevBuf<uint32_t> s_base;            // n_slots + 1
    dss::DevBuf<uint32_t> bk_start;          // n_groups + 1
    dss::DevBuf<uint64_t> g_key;             // n_groups: slot << 6 | bucket
    int64_t n_groups = 0;
    int64_t tiles_total = 0, tiles_max = 0;  // join-unit posting tiles (sum, max over groups)
    dss::DevBuf<uint32_t> b_e;               // entity | first bit
    dss::DevBuf<float2> b_alt;               // (alt_lo, alt_hi)
    dss::DevBuf<longlong2> b_t;              // (t0, t1) microseconds
    dss::DevBuf<uint8_t> b_meta;             // entity's first bucket | compact << 7
    dss::DevBuf<ulonglong2> b_sig;           // 2 per posting: 256-bit prefix signature
    dss::DevBuf<int32_t> b_owner;
    // ---- entity-level attributes (subscription-store queries, subs.hip) ------
    dss::DevBuf<int64_t> e_t1;     // ends_at (us)
    dss::DevBuf<int32_t> e_owner;  // owner id (has_owner)
    dss::DevBuf<uint32_t> o_key;   // owner ^ 0x80000000, ascending (owner -> entities)
    dss::DevBuf<uint32_t> o_ent;   // entity ids in o_key order
    dss::DevBuf<int64_t> e_notify; // notification_index counters
    // tombstones (write path, store.hip): bit e set = entity e is deleted or
    // superseded; the join and the subscription queries skip it
    dss::DevBuf<uint32_t> dead;
    bool has_dead = false;
    int device = 0;
};

namespace dss {

class SearchEngine {
   public:
    // Postings are kept only for cells in [cell_lo, cell_hi] (a cell-range
    // shard); entity cell lists stay whole, so the smallest-shared-cell rule
    // emits every pair on exactly one shard.
    void build(dssg_index *idx, int64_t n, const int64_t *cell_offs, const uint64_t *cells, const float *alt_lo,
               const float *alt_hi, const int64_t *t0, const int64_t *t1, const int32_t *owner, uint64_t cell_lo,
               uint64_t cell_hi, hipStream_t s);
    // q cells must be sorted ascending and unique per query.
    void search(const dssg_index *idx, int64_t nq, const int64_t *q_offs, const uint64_t *q_cells,
                const float *q_alt_lo, const float *q_alt_hi, const int64_t *q_tlo, const int64_t *q_thi,
                const int32_t *q_owner, hipStream_t s, dssg_pairs *out);
    // Roofline accounting: postings scanned and distinct candidate entities
    // (predicate disabled), i.e. sum_q M_q and sum_q D_q of SURVEY s8(d).
    void stats(const dssg_index *idx, int64_t nq, const int64_t *q_offs, const uint64_t *q_cells, hipStream_t s,
               int64_t *matched, int64_t *distinct);
    void set_timing(bool on) { timing_ = on; }
    double last_join_kernel_ms() const { return join_ms_; }
    int64_t last_units() const { return units_; }
    int64_t last_keys() const { return keys_; }
    // timing mode only: runs, wave iterations (records x tiles), useful lane tests
    // timing mode only: output flushes, exact list merges (events, lanes)
    int64_t last_tagged() const { return tagged_; }  // long x long pair occurrences before the dedupe
    // long queries in the last batch, long postings of its index (both > 0:
    // the join ran its long x long tagging variant)
    void last_longs(int64_t *lq, int64_t *lp) const { *lq = long_queries_; *lp = long_postings_; }
    void last_join_events(int64_t *flushes, int64_t *merges, int64_t *merge_lanes) const
    {
        *flushes = flushes_;
        *merges = merges_;
        *merge_lanes = merge_lanes_;
    }
    void last_work(int64_t *runs, int64_t *iters, int64_t *tests) const
    {
        *runs = runs_;
        *iters = iters_;
        *tests = tests_;
    }

   private:
    DevBuf<unsigned char> tmp_;
    DevBuf<uint64_t> k0_, k1_, uk_;
    DevBuf<uint32_t> v0_, v1_, v2_, v3_, ur_, up_, uq_, cq_, gb_, ge_, dec_;
    DevBuf<int64_t> c0_, c1_, rc_, rs_, nr_, uc_, uo_;
    DevBuf<unsigned long long> counter_;
    DevBuf<uint32_t> oq_, oe_, oq2_, oe2_;
    DevBuf<unsigned char> rec_;
    DevBuf<int32_t> own_;
    DevBuf<uint8_t> qlong_;
    DevBuf<unsigned long long> tkey_, tkey2_;  // tagged (long x long) pairs, deduplicated after the join
    DevBuf<uint32_t> work_;
    DevBuf<unsigned char> units_buf_;  // join unit descriptors
    int n_cu_ = 0;
    size_t out_cap_ = 0;
    bool timing_ = false;
    double join_ms_ = 0;
    int64_t units_ = 0, keys_ = 0, runs_ = 0, iters_ = 0, tests_ = 0;
    int64_t flushes_ = 0, merges_ = 0, merge_lanes_ = 0, tagged_ = 0, long_queries_ = 0, long_postings_ = 0;
    hipEvent_t ev0_ = nullptr, ev1_ = nullptr;
};

}  // namespace dss
