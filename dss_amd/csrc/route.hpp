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

// Bytes of one part's segment in the fused send buffer: its rows, then its
// cell lists, padded to 32 bytes.
int64_t route_segment_bytes(int64_t rows, int64_t cells);

// What the most recent sharded step on a context moved and how long its
// phases took (HIP events; timing on, else 0).  join_ms < 0: the one-rank
// identity route (no exchange).
struct ShardStats {
    double route_ms = 0, xq_ms = 0, join_ms = 0, pack_ms = 0, xp_ms = 0;
    int64_t q_bytes_sent = 0, q_bytes_recv = 0, p_bytes_sent = 0, p_bytes_recv = 0, rows = 0, shard_pairs = 0;
    int64_t cells = 0, touched = 0;  // routed query cells joined here; postings of their distinct cells (timing on)
};

class RouteEngine {
   public:
    static constexpr int kMaxParts = DSSG_MAX_PARTS;
    RouteEngine() = default;
    RouteEngine(const RouteEngine &) = delete;
    RouteEngine &operator=(const RouteEngine &) = delete;
    ~RouteEngine();
    // pass 0: per-query destination masks, per-part row / cell counts and
    // fused segment sizes (host)
    void plan(int64_t nq, const int64_t *offs, const uint64_t *cells, int np, const uint64_t *part_hi, hipStream_t s,
              int64_t *row_counts, int64_t *cell_counts, int64_t *seg_bytes);
    // pass 1: rows + cell lists into the caller-owned fused send buffer
    void fill(int64_t nq, const int64_t *offs, const uint64_t *cells, const float *alo, const float *ahi,
              const int64_t *tlo, const int64_t *thi, hipStream_t s, void *send);
    // received fused segments (src_rows / src_cells per source part) -> batch
    void unpack(const void *recv, int np, const int64_t *src_rows, const int64_t *src_cells, hipStream_t s,
                dssg_batch *out);
    // pair counts per home part; the send-buffer bases skip self_part (-1: none)
    void pairs_plan(const dssg_batch *b, const dssg_pairs *p, int np, int self_part, hipStream_t s, int64_t *counts);
    // other parts' pairs packed into `out`, the self part's to (self_q, self_e)
    void pairs_fill(const dssg_batch *b, const dssg_pairs *p, hipStream_t s, uint64_t *out, uint32_t *self_q,
                    uint32_t *self_e);
    // routed pairs (home-local qid << 32 | entity) -> (q, e) arrays
    static void split_pairs(int64_t n, const uint64_t *in, uint32_t *q, uint32_t *e, hipStream_t s);

   private:
    unsigned long long *host_words();
    DevBuf<unsigned char> tmp_;
    DevBuf<unsigned long long> mask_, acc_, pacc_;
    DevBuf<int64_t> base_, pbase_, ncell_, tlo_, thi_, offs_;
    DevBuf<uint64_t> cells_;
    DevBuf<float> alo_, ahi_;
    DevBuf<uint32_t> home_, qid_;
    // an H2D copy of host-written bases may still be pending (on any stream)
    // when the next plan rewrites them: the host waits for it first
    void wait_h2d(hipEvent_t &ev);
    void mark_h2d(hipEvent_t &ev, hipStream_t s);
    unsigned long long *h_counts_ = nullptr;  // pinned
    hipEvent_t h2d_plan_ = nullptr, h2d_pairs_ = nullptr;
    int64_t plan_nq_ = 0, pplan_n_ = 0, pplan_self_n_ = 0;
    int plan_np_ = 0, pplan_np_ = 0, pplan_self_ = -1;
    const int64_t *plan_offs_ = nullptr;
    const uint64_t *plan_cells_ = nullptr, *plan_part_hi_ = nullptr;
    const uint32_t *pplan_q_ = nullptr;
};

}  // namespace dss
