// Host-side driver of the subscription-store queries (subs.hip).
#pragma once
#include "common.hpp"
#include "search.hpp"

namespace dss {

class SubsEngine {
   public:
    // out[q] (host) = max over the query's cells of the owner's unexpired
    // entities posted in the cell (repeats counted), 0 if none; the entities
    // of all `sides` (indexes over disjoint live entities: a store's base and
    // delta; null sides skipped) count together.
    void max_count(const dssg_index *const *sides, int nsides, int64_t nq, const int64_t *offs, const uint64_t *cells,
                   int64_t nqc, const int32_t *owner, int64_t now, hipStream_t s, int64_t *out);
    // Every entity of owner[q] with ends_at >= now; device outputs, count returned.
    int64_t owner_subs(const dssg_index *idx, int64_t nq, const int32_t *owner, int64_t now, hipStream_t s,
                       uint32_t **out_q, uint32_t **out_e);
    // Advances the index's notification counters for the (query, entity)
    // pairs p (distinct) in batch order; device outputs sorted by (entity,
    // query) with the value after each pair's increment.
    void notify(dssg_index *idx, const dssg_pairs *p, hipStream_t s, uint32_t **out_q, uint32_t **out_e, int64_t **out_v);

   private:
    DevBuf<unsigned char> tmp_;
    DevBuf<unsigned long long> cnt_, k0_, k1_;
    DevBuf<uint32_t> cq_, q_, e_;
    DevBuf<int64_t> c_, o_, v_;
};

}  // namespace dss
