// Device view of a dssg_index (search.hpp) shared by the kernels that read
// the index: the overlap join (search.hip) and the subscription-store
// queries (subs.hip).  Layout: DESIGN.md s3.
#pragma once
#include <hip/hip_runtime.h>

#include "search.hpp"

namespace dss {
namespace {

constexpr uint32_t kFirstBit = 0x80000000u;  // b_e: the cell is the entity's smallest cell
constexpr uint8_t kMetaCompact = 0x80;      // b_meta: every smaller cell of the entity is within +-7 cells
constexpr uint8_t kMetaLongFp = 0x40;       // b_meta: the entity's footprint is long (long_cells)
constexpr uint64_t kLsb13 = 1ull << 34;

__device__ __forceinline__ int64_t tid64() { return (int64_t)blockIdx.x * blockDim.x + threadIdx.x; }
__device__ __forceinline__ int64_t nthreads64() { return (int64_t)gridDim.x * blockDim.x; }
__host__ __device__ __forceinline__ bool is_regular(uint64_t c)
{
    return (c & ((kLsb13 << 1) - 1)) == kLsb13 && (c >> 61) < 6;  // level 13, valid face
}
__host__ __device__ __forceinline__ unsigned long long order_key(long long t)
{
    return (unsigned long long)t ^ 0x8000000000000000ull;  // signed order as unsigned
}
// Start of an entity's interval: the band join's sort key.
__host__ __device__ __forceinline__ long long tmin2(long long a, long long b) { return a < b ? a : b; }

// Device view of a dssg_index.
struct IndexView {
    uint64_t kmin;
    int64_t n_dense;
    int64_t n_irr;
    const uint64_t *irr_cells;
    const uint64_t *s_post;
    const uint32_t *s_nreg;
    const uint8_t *s_lfp;
    const uint32_t *b_e;
    const uint8_t *b_meta;
    const float2 *b_alt;
    const longlong2 *b_t;
    const ulonglong2 *b_sig;
    const int32_t *b_owner;  // nullptr: built without owners
    const uint32_t *b_mult;  // nullptr: every multiplicity is 1
    const int64_t *e_offs;
    const uint64_t *e_cells;
    const int64_t *e_t1;     // entity end time (us)
    const int32_t *e_owner;  // entity owner (nullptr: built without owners)
    const uint32_t *dead;    // tombstone bitmap (nullptr: none)
    long long dcap;
};

IndexView view_of(const dssg_index *idx)
{
    IndexView v{};
    v.kmin = idx->kmin;
    v.n_dense = idx->n_dense;
    v.n_irr = idx->n_irr;
    v.irr_cells = idx->irr_cells.p;
    v.s_post = idx->s_post.p;
    v.s_nreg = idx->s_nreg.p;
    v.s_lfp = idx->s_lfp.p;
    v.b_e = idx->b_e.p;
    v.b_meta = idx->b_meta.p;
    v.b_alt = idx->b_alt.p;
    v.b_t = idx->b_t.p;
    v.b_sig = idx->b_sig.p;
    v.b_owner = idx->has_owner ? idx->b_owner.p : nullptr;
    v.b_mult = idx->has_mult ? idx->b_mult.p : nullptr;
    v.e_offs = idx->e_offs.p;
    v.e_cells = idx->e_cells.p;
    v.e_t1 = idx->e_t1.p;
    v.e_owner = idx->has_owner ? idx->e_owner.p : nullptr;
    v.dead = idx->has_dead ? idx->dead.p : nullptr;
    v.dcap = idx->dcap;
    return v;
}

// Slot of cell c, or false if c is in neither table.
__device__ __forceinline__ bool find_slot(const IndexView &a, uint64_t c, uint32_t &slot)
{
    if (is_regular(c)) {
        uint64_t k = c >> 35;
        if (k < a.kmin || (int64_t)(k - a.kmin) >= a.n_dense) return false;
        slot = (uint32_t)(k - a.kmin);
        return true;
    }
    int64_t lo = 0, hi = a.n_irr;
    while (lo < hi) {
        int64_t mid = (lo + hi) >> 1;
        if (a.irr_cells[mid] < c) lo = mid + 1;
        else hi = mid;
    }
    if (lo < a.n_irr && a.irr_cells[lo] == c) {
        slot = (uint32_t)(a.n_dense + lo);
        return true;
    }
    return false;
}
__device__ __forceinline__ uint64_t cell_of_slot(const IndexView &a, uint32_t slot)
{
    if ((int64_t)slot < a.n_dense) return ((a.kmin + slot) << 35) | kLsb13;
    return a.irr_cells[slot - (uint32_t)a.n_dense];
}
// Postings of a slot: [s, e), the regular ones [s, s + nreg).
__device__ __forceinline__ void slot_range(const IndexView &a, uint32_t slot, uint64_t &s, uint64_t &e)
{
    s = a.s_post[slot];
    e = a.s_post[slot + 1];
}

__device__ __forceinline__ bool is_dead(const IndexView &a, uint32_t e)
{
    return a.dead && ((a.dead[e >> 5] >> (e & 31)) & 1u);
}

}  // namespace
}  // namespace dss
