// Host-side driver of the entity index and the 4D overlap join (search.hip).
#pragma once
#include "common.hpp"

struct dssg_index {
    int64_t n_e = 0;      // entities
    int64_t n_p = 0;      // unique (cell, entity) postings
    int64_t n_reg = 0;    // postings whose cell is a valid level-13 id (dense lookup)
    bool has_owner = false;
    // postings sorted by (cell, entity); regular first, irregular after
    dss::DevBuf<uint64_t> p_cell;
    dss::DevBuf<uint32_t> p_e;      // bit 31: "cell is the entity's smallest cell"
    dss::DevBuf<float2> p_alt;      // (alt_lo, alt_hi)
    dss::DevBuf<longlong2> p_t;     // (t0, t1) microseconds
    dss::DevBuf<int32_t> p_owner;
    // entity -> sorted unique cells (canonical-cell dedupe)
    dss::DevBuf<int64_t> e_offs;
    dss::DevBuf<uint64_t> e_cells;
    // dense lookup over level-13 cells: key k = cell >> 35 in [kmin, kmin + n_dense)
    uint64_t kmin = 0;
    int64_t n_dense = 0;              // slots; dense has n_dense + 1 entries
    dss::DevBuf<uint32_t> dense;
    // irregular cells (not level 13 / invalid face): sorted unique + starts
    int64_t n_irr = 0;
    dss::DevBuf<uint64_t> irr_cells;
    dss::DevBuf<uint32_t> irr_start;  // n_irr + 1, absolute posting indices
    int device = 0;
};

namespace dss {

class SearchEngine {
   public:
    void build(dssg_index *idx, int64_t n, const int64_t *cell_offs, const uint64_t *cells, const float *alt_lo,
               const float *alt_hi, const int64_t *t0, const int64_t *t1, const int32_t *owner, hipStream_t s);
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

   private:
    DevBuf<unsigned char> tmp_;
    DevBuf<uint64_t> k0_, k1_;
    DevBuf<uint32_t> v0_, v1_;
    DevBuf<int64_t> c0_, c1_;
    DevBuf<uint8_t> fl_;
    DevBuf<unsigned long long> counter_;
    // tiled-join scratch
    DevBuf<uint32_t> sk_, sv_, uk_, tr_, tp_, tq_;
    DevBuf<int64_t> rc_, rs_, nr_, tc_, to_;
    DevBuf<uint32_t> oq_, oe_;
    size_t out_cap_ = 0;
    bool timing_ = false;
    double join_ms_ = 0;
    hipEvent_t ev0_ = nullptr, ev1_ = nullptr;
};

}  // namespace dss
