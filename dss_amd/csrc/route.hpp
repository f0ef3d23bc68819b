// Host-side driver of the cell-range shard routing kernels (route.hip).
#pragma once
#include "common.hpp"

namespace dss {

// One routed query: 32 bytes, the unit of the query all-to-all.
struct QRow {
    long long tlo, thi;  // time window (us), `now` already folded into tlo
    float alo, ahi;      // altitude band (f32, NULL -> -/+inf)
    uint32_t qid;        // index in the home rank's batch
    uint32_t ncells;     // length of the cell list that follows in the cells buffer
};
static_assert(sizeof(QRow) == 32, "QRow layout");
static_assert(sizeof(QRow) == DSSG_ROUTE_ROW_BYTES, "QRow size vs dssgpu.h");

class RouteEngine {
   public:
    static constexpr int kMaxParts = DSSG_MAX_PARTS;
    // pass 0: per-query destination masks, per-part row / cell counts (host)
    void plan(int64_t nq, const int64_t *offs, const uint64_t *cells, int np, const uint64_t *part_hi, hipStream_t s,
              int64_t *row_counts, int64_t *cell_counts);
    // pass 1: rows + cell lists into caller-owned part-major buffers
    void fill(int64_t nq, const int64_t *offs, const uint64_t *cells, const float *alo, const float *ahi,
              const int64_t *tlo, const int64_t *thi, hipStream_t s, void *rows, uint64_t *out_cells);
    void unpack(int64_t nrows, const void *rows, const uint64_t *cells, int np, const int64_t *src_rows, hipStream_t s,
                dssg_batch *out);
    void pairs_plan(const dssg_batch *b, const dssg_pairs *p, int np, hipStream_t s, int64_t *counts);
    void pairs_fill(const dssg_batch *b, const dssg_pairs *p, hipStream_t s, uint64_t *out);
    // routed pairs (home-local qid << 32 | entity) -> (q, e) arrays
    static void split_pairs(int64_t n, const uint64_t *in, uint32_t *q, uint32_t *e, hipStream_t s);

   private:
    DevBuf<unsigned char> tmp_;
    DevBuf<unsigned long long> mask_, acc_, pacc_;
    DevBuf<int64_t> base_, sbase_, pbase_, ncell_, tlo_, thi_, offs_;
    DevBuf<float> alo_, ahi_;
    DevBuf<uint32_t> home_, qid_;
    int64_t plan_nq_ = 0, pplan_n_ = 0;
    int plan_np_ = 0, pplan_np_ = 0;
    const int64_t *plan_offs_ = nullptr;
    const uint64_t *plan_cells_ = nullptr, *plan_part_hi_ = nullptr;
    const uint32_t *pplan_q_ = nullptr;
};

}  // namespace dss
