// Host-side write path over the entity index (store.hip): base + delta
// indexes, tombstones, compaction.
#pragma once
#include <vector>

#include "common.hpp"
#include "search.hpp"

namespace dss {

class Store {
   public:
    // delta folded into a new base past max(kMinDelta, base / kDeltaFrac)
    static constexpr int64_t kMinDelta = 4096;
    static constexpr int64_t kDeltaFrac = 16;

    Store(int device, bool with_owner) : device_(device), with_owner_(with_owner) {}
    ~Store();
    Store(const Store &) = delete;
    Store &operator=(const Store &) = delete;

    void upsert(SearchEngine &se, int64_t n, const uint32_t *ids, const int64_t *offs, const uint64_t *cells,
                const float *alo, const float *ahi, const int64_t *t0, const int64_t *t1, const int32_t *owner,
                hipStream_t s);
    void remove(SearchEngine &se, int64_t n, const uint32_t *ids, int32_t *found, hipStream_t s);
    void compact(SearchEngine &se, hipStream_t s);
    // Pairs (query << 32 | id), sorted.
    int64_t search(SearchEngine &se, int64_t nq, const int64_t *d_offs, const uint64_t *d_cells, const float *d_alo,
                   const float *d_ahi, const int64_t *d_tlo, const int64_t *d_thi, const int32_t *d_owner, hipStream_t s,
                   std::vector<uint64_t> &out);
    int64_t live() const { return live_; }
    int64_t base_size() const { return base_ ? base_->n_e : 0; }
    int64_t delta_size() const { return delta_ ? delta_->n_e : 0; }
    int64_t compactions() const { return compactions_; }
    bool with_owner() const { return with_owner_; }
    // the indexes a search covers (either may be null): every live row is in
    // exactly one of them (base rows rewritten since are tombstoned there)
    const dssg_index *base() const { return base_; }
    const dssg_index *delta() const { return delta_; }

   private:
    struct Row {
        bool live = false, in_delta = false;
        std::vector<uint64_t> cells;
        float alo = 0, ahi = 0;
        int64_t t0 = 0, t1 = 0;
        int32_t owner = 0;
    };
    void check_ids(int64_t n, const uint32_t *ids) const;
    void tomb(uint32_t id);
    void refresh(SearchEngine &se, hipStream_t s);
    dssg_index *build(SearchEngine &se, const std::vector<uint32_t> &ids, hipStream_t s, DevBuf<uint32_t> &map);

    int device_;
    bool with_owner_;
    std::vector<Row> rows_;   // by caller id
    std::vector<uint32_t> delta_list_;  // ids written since the base was built (in_delta set when listed)
    int64_t live_ = 0, compactions_ = 0;
    dssg_index *base_ = nullptr, *delta_ = nullptr;
    DevBuf<uint32_t> base_ids_, delta_ids_;  // dense index -> id
    std::vector<int64_t> base_pos_;          // id -> base index, -1 if none
    std::vector<uint32_t> dead_h_;           // base tombstones (host copy)
    bool dead_dirty_ = false;
    DevBuf<int64_t> u_offs_, u_t0_, u_t1_;
    DevBuf<uint64_t> u_cells_;
    DevBuf<float> u_lo_, u_hi_;
    DevBuf<int32_t> u_ow_;
};

}  // namespace dss
