// Device view of a dssg_index (search.hpp) shared by the kernels that read
// the index: the overlap join (search.hip) and the subscription-store
// queries (subs.hip).  Layout: DESIGN.md s3.
#pragma once
#include <hip/hip_runtime.h>

#include "search.hpp"

namespace dss {
namespace {

// Postings are per (entity, group): an index is built at one of two grains
// (dssg_index.gshift, chosen per build from the footprints' shape):
//   * quads (gshift 37): a group is a level-12 cell, the 2 x 2 level-13 cells
//     below it (ids contiguous in S2 order: a quad's cells are one run of a
//     sorted cell list); a posting carries the 4-bit mask of the entity's
//     cells in the quad (b_meta low bits, bit = the child position
//     (c >> 35) & 3);
//   * cells (gshift 35): a group is one level-13 cell, mask 1.
// An id that is not a valid level-13 cell (the reference tests use invalid
// face-7 ids as opaque keys, Q12) is a group of its own with mask 1, so it
// meets only an equal id.  "Quad" below means a group of either grain.
constexpr uint32_t kFirstBit = 0x80000000u;  // b_e: the quad is the entity's first (holds its smallest cell)
constexpr uint8_t kMetaCompact = 0x80;      // b_meta: every cell of the entity before the quad lies in its window
constexpr uint8_t kMetaLongFp = 0x40;       // b_meta: the entity's footprint is long (long_cells)
constexpr uint8_t kMetaMask = 0x0F;         // b_meta: the entity's cells in the quad (child bits)
constexpr uint64_t kLsb13 = 1ull << 34;
constexpr int kQuadShift = 37;              // group key of a level-13 id at the quad grain: c >> 37
constexpr int kCellShift = 35;              // ... at the cell grain: c >> 35

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
    const uint32_t *s_band;  // nullptr: one run per slot; else 8 band starts per slot (dssg_index.s_band)
    const uint32_t *b_e;
    const uint8_t *b_meta;
    const float2 *b_alt;
    const longlong2 *b_t;
    const ulonglong2 *b_sig;
    const int32_t *b_owner;  // nullptr: built without owners
    const uint32_t *b_mult;  // nullptr: every multiplicity is 1; else 8 bits per child (quads) or 32 (cells)
    const int64_t *e_offs;
    const uint64_t *e_cells;
    const int64_t *e_t1;     // entity end time (us)
    const int32_t *e_owner;  // entity owner (nullptr: built without owners)
    const uint32_t *dead;    // tombstone bitmap (nullptr: none)
    long long dcap;
    int gshift;              // group key = cell >> gshift (kQuadShift or kCellShift)
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
    v.s_band = idx->n_bands > 1 ? idx->s_band.p : nullptr;
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
    v.gshift = idx->gshift;
    return v;
}

// Child bit of a cell in its group (1 at the cell grain, and for an
// irregular id: its own group).
__host__ __device__ __forceinline__ uint32_t child_bit(uint64_t c, int gshift)
{
    return (gshift == kQuadShift && is_regular(c)) ? 1u << (uint32_t)((c >> 35) & 3u) : 1u;
}
// Two cells of one sorted list in the same group (irregular ids never share).
__host__ __device__ __forceinline__ bool same_quad(uint64_t a, uint64_t b, int gshift)
{
    return is_regular(a) && is_regular(b) && (a >> gshift) == (b >> gshift);
}

// Slot of the quad holding cell c, or false if it is in neither table.
__device__ __forceinline__ bool find_slot(const IndexView &a, uint64_t c, uint32_t &slot)
{
    if (is_regular(c)) {
        uint64_t k = c >> a.gshift;
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
// The smallest cell a slot's quad can hold (its child 0; an irregular id
// itself): "cells below the quad" are the cells < this one.
__device__ __forceinline__ uint64_t quad_first_cell(const IndexView &a, uint32_t slot)
{
    if ((int64_t)slot < a.n_dense) return ((a.kmin + slot) << a.gshift) | kLsb13;
    return a.irr_cells[slot - (uint32_t)a.n_dense];
}
// A posting's multiplicity for one child of its quad (the times (cell,
// entity) occurs in the stored array: 8 bits per child at the quad grain, the
// whole word at the cell grain -- b_mult).
__device__ __forceinline__ uint32_t child_mult(const IndexView &a, uint64_t p, uint32_t bit)
{
    if (!a.b_mult) return 1u;
    if (a.gshift == kCellShift) return a.b_mult[p];
    return (a.b_mult[p] >> (8u * (uint32_t)__builtin_ctz(bit))) & 0xffu;
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
