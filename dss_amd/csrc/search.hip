// Entity index + 4D overlap band join on gfx950.
//
// Replaces the CockroachDB side of the reference search:
//   scd_cells_operations PK (cell_id, operation_id) + scd_operations
//     (pkg/scd/store/cockroach/store.go:120-147) and the query at
//     pkg/scd/store/cockroach/operations.go:376-402;
//   RID `cells INT64[]` + INVERTED INDEX (pkg/rid/cockroach/store.go:122-151)
//     and the `cells && $n` queries (identification_service_area.go:170-180,
//     subscriptions.go:222-273).
//
// Index: one posting per (entity, quad) -- a quad is the
// level-12 parent of 2 x 2 level-13 cells, the posting carries the mask of the
// entity's cells in it -- sorted by (quad, duration class, altitude band,
// m = min(t0, t1)): a dense quad's regular postings form 4 runs by alt_lo
// quantile, each in m order; a quad's postings are found with one dense
// lookup (slot = cell >> 37 for level-13 ids; a sorted side table for any
// other id, each its own quad -- the reference tests use invalid face-7 ids,
// Q12).  A query and an entity meet in a quad where their masks intersect,
// and the pair is emitted in the quad holding their smallest shared cell (SQL
// DISTINCT).  Filter attributes (altitudes, times, a 256-bit "near prefix"
// signature) are inlined per posting, SoA.  No posting is copied: 2.2e9
// postings (configs[4], 50M corridors) fit one GPU.
//
// Search, a band join per quad:
//   * queries are ordered by start time (narrow windows first, wide ones
//     after), one 64-B record per (query, quad) emitted in that order, the
//     keys stably grouped by quad and the records permuted into that order,
//     so a quad's records are one contiguous run sorted by start;
//   * a join unit = one tile of <= 64 postings of a quad (one band of it) x
//     the quad's records whose start can meet the tile (k_units);
//   * one wavefront per unit, lane = posting (in registers): the records are
//     loaded 64 at a time, those meeting the tile's time hull (and a banded
//     tile's altitude hull) staged in LDS and broadcast; each lane ORs the
//     fused altitude/time/owner predicate into a 64-bit mask, ANDs the quad
//     cell masks, applies the smallest-shared-cell rule (SQL DISTINCT, Q13)
//     and the batch's pairs leave contiguously.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cmath>
#include <cstdio>
#include <cstring>
#include <vector>

#include "compact.cuh"
#include "index_view.cuh"
#include "radix.hpp"
#include "search.hpp"

namespace dss {
namespace {

constexpr unsigned kBlock = 256;
constexpr uint32_t kRank0 = 0x80000000u;     // record: the quad is the query's first (holds its smallest cell)
constexpr uint32_t kCompactQ = 0x40000000u;  // record: the query's cells before the quad lie in its window
constexpr uint32_t kLongQ = 0x20000000u;     // record: the query footprint is long (long_cells)
constexpr int kQMaskShift = 25;              // record: the query's cells in the quad (child bits 25..28)
constexpr uint32_t kQMask = 0xFu << kQMaskShift;
constexpr uint32_t kQFlags = kRank0 | kCompactQ | kLongQ | kQMask;
constexpr int64_t kMaxBatchQ = (int64_t)1 << kQMaskShift;  // queries per batch (ids below the flag bits)
constexpr uint32_t kNoDecode = 0xffffffffu;
constexpr uint32_t kNoSlot = 0xffffffffu;
// Query windows wider than a per-batch threshold T form their own per-cell
// runs (met by every tile of the cell); the narrow ones are met only by the
// tiles whose start range reaches [tlo - dcap, tlo + dqmax], dqmax the widest
// narrow window.  T = 2^b minimises narrow(b) (2^b + dcap) + wide(b) H over the
// batch's window histogram (k_qwin), H the index's time span (choose_wide_log).
// (A fixed T = 2^32 us let a few NULL-start queries near `now` set dqmax to
// 72 min on configs[2], whose windows are otherwise <= 30 min.)
constexpr int kWinBuckets = 65;  // ceil(log2(window)) in 0..64
constexpr int kOrderBits = 16;                          // query order key: quantised tlo (2 radix passes)
constexpr uint32_t kWideKey = (1u << kOrderBits) - 1u;  // quantised-start clamp
constexpr uint32_t kWideBit = 1u << kOrderBits;  // order key: a wide query (carried above the sorted bits)

// Work lists written from kRegions counters (spread 256 B apart; one
// same-address counter saturates at ~88 atomics/us, MI355X_MICROARCH.md
// "dequeue"): region r holds its items at [r * cap, r * cap + count(r)).
constexpr int kRegions = 8;
constexpr int kRegStride = 32;
struct Regions {
    unsigned long long *cnt;  // kRegions counters, kRegStride words apart
    int64_t cap;              // items per region
    __device__ __forceinline__ unsigned long long *counter(int r) const { return cnt + r * kRegStride; }
    // total items written and the region of virtual item u (u < total)
    __device__ __forceinline__ int64_t total(int64_t pre[kRegions + 1]) const
    {
        pre[0] = 0;
#pragma unroll
        for (int r = 0; r < kRegions; r++) pre[r + 1] = pre[r] + min((int64_t)cnt[r * kRegStride], cap);
        return pre[kRegions];
    }
    __device__ __forceinline__ int64_t slot_of(const int64_t pre[kRegions + 1], int64_t u) const
    {
        int r = 0;
#pragma unroll
        for (int k = 1; k < kRegions; k++) r += u >= pre[k] ? 1 : 0;
        return r * cap + (u - pre[r]);
    }
};

// k_join occupancy and its LDS pair stage, two shapes: sparse-output joins
// (configs[2]: ~6 pairs per staged record) run 7 workgroups per CU with a
// 640-pair stage per wave (k_join 3.45 -> 3.24 ms against 6 x 1024);
// dense-output joins (configs[3], RID 30-s windows: ~29 pairs per record,
// pass density 0.45) take 1024-pair stages at 3 workgroups per CU (round 6,
// on the 3-pipeline step: configs[3] 867 -> 973M q/s against 6, k_join 0.53
// -> 0.46 ms; 2 gave the step +3 % more with a slower join, profiles/r07z).
// The search picks the shape from the previous batch's pass density
// (dense_out_).
constexpr int kWaves = 4;  // waves per join workgroup
#ifndef DSS_JOIN_BPC_SPARSE
#define DSS_JOIN_BPC_SPARSE 7
#endif
#ifndef DSS_JOIN_BPC_DENSE
#define DSS_JOIN_BPC_DENSE 3
#endif
constexpr int kJoinBpcSparse = DSS_JOIN_BPC_SPARSE, kJoinBpcDense = DSS_JOIN_BPC_DENSE;
#ifndef DSS_STAGE_SPARSE
#define DSS_STAGE_SPARSE 640
#endif
constexpr int kStageSparse = DSS_STAGE_SPARSE, kStageDense = 1024;
#ifndef DSS_JOIN_LONG_WPE
#define DSS_JOIN_LONG_WPE 1
#endif
constexpr int kJoinLongWpe = DSS_JOIN_LONG_WPE;  // the long variant's register budget (waves per SIMD)
#ifndef DSS_EMIT_DENSITY
#define DSS_EMIT_DENSITY 2
#endif
constexpr int kEmitDensity = DSS_EMIT_DENSITY;

// Counting build of the join (-DDSS_JOIN_PROFILE through tools/variants.sh;
// never the shipped library): what becomes of every lane test -- which
// predicate rejects it, how many reach the smallest-shared-cell check, how
// many are kept -- plus the staging and emission shapes, summed over every
// k_join launch into g_jprof and read (and cleared) by dssg_join_profile.
// Slot meanings: kJProfNames in join_profile_read.
constexpr int kJProf = 22;
#ifdef DSS_JOIN_PROFILE
__device__ unsigned long long g_jprof[kJProf];
#define JPROF(i, v) (jp[i] += (unsigned long long)(v))
#else
#define JPROF(i, v) ((void)0)
#endif
// ---- level-13 decode + prefix signatures -----------------------------------
__device__ __forceinline__ int s2pos_to_ij(int o, int pos) { return (int)((0x874B78B4u >> (8 * o + 2 * pos)) & 3u); }
__device__ __forceinline__ int s2pos_to_orientation(int pos) { return (int)((0xC1u >> (2 * pos)) & 3u); }

// Level-13 (face, i, j) of a cell id (cellid.go faceIJOrientation, walked one
// level at a time), packed face << 26 | i << 13 | j; kNoDecode for ids that
// are not valid level-13 cells.
__device__ __forceinline__ uint32_t decode13(uint64_t c)
{
    if (!is_regular(c)) return kNoDecode;
    const int face = (int)(c >> 61);
    int o = face & 1, i = 0, j = 0;
#pragma unroll
    for (int l = 0; l < 13; l++) {
        const int pos = (int)((c >> (59 - 2 * l)) & 3);
        const int ij = s2pos_to_ij(o, pos);
        i = (i << 1) | (ij >> 1);
        j = (j << 1) | (ij & 1);
        o ^= s2pos_to_orientation(pos);
    }
    return (uint32_t)face << 26 | (uint32_t)i << 13 | (uint32_t)j;
}

// Near-prefix signature of a sorted cell list at a quad: one bit per
// (i mod 16, j mod 16) for every cell below the quad that lies on its face in
// the quad's 16 x 16 window (mod 16 is injective on it, so equal bits are
// equal cells); `compact` iff every cell below the quad is such a near cell.
// For two lists that meet in the quad:
//   * near bits overlap            -> they share a cell below it (exact);
//   * no overlap, one side compact -> they share no cell below it (exact: a
//     shared cell would lie in the compact side's window, so in both sets);
//   * otherwise both footprints are "long" (cells outside an 8 x 8 window,
//     long_cells): their pairs are tagged and deduplicated after the join.
struct Sig256 {
    unsigned long long w[4];
};
__device__ __forceinline__ void sig_set(Sig256 &sig, int i, int j)
{
    const int b = ((i & 15) << 4) | (j & 15);
    const unsigned long long bit = 1ull << (b & 63);
    const int wi = b >> 6;  // selects, not an indexed store: keeps sig in registers
    sig.w[0] |= wi == 0 ? bit : 0;
    sig.w[1] |= wi == 1 ? bit : 0;
    sig.w[2] |= wi == 2 ? bit : 0;
    sig.w[3] |= wi == 3 ? bit : 0;
}
// Signature of the decoded prefix dec[0..n) (the cells below the quad) at the
// quad of the decoded cell dc: the window is the 16 x
// 16 cells [i0 - 7, i0 + 8] x [j0 - 7, j0 + 8] around the quad's even anchor
// (i0, j0), so mod 16 stays injective; `compact` iff every cell of the prefix
// (the cells in earlier quads) lies in it.  Two lists meeting in the quad
// share a cell below it iff (when either is compact) their signatures
// overlap.  A footprint inside an 8 x 8 window is compact at each of its
// quads.
__device__ __forceinline__ void prefix_sig_quad(const uint32_t *dec, int64_t n, uint32_t dc, Sig256 &sig,
                                                bool &compact)
{
    sig.w[0] = sig.w[1] = sig.w[2] = sig.w[3] = 0;
    const bool v = dc != kNoDecode;
    compact = v;
    const int f = (int)(dc >> 26), i0 = (int)((dc >> 13) & 8190u), j0 = (int)(dc & 8190u);
    constexpr int kU = 8;  // prefix decodes loaded per round (4 or 2: k_qrecs 0.223 -> 0.233 / 0.247 ms, profiles/r07m)
    for (int64_t k0 = 0; k0 < n; k0 += kU) {
        uint32_t dd[kU];
#pragma unroll
        for (int u = 0; u < kU; u++) dd[u] = k0 + u < n ? dec[k0 + u] : 0u;
#pragma unroll
        for (int u = 0; u < kU; u++) {
            if (k0 + u >= n) break;
            const uint32_t d = dd[u];
            const int ci = (int)((d >> 13) & 8191u), cj = (int)(d & 8191u);
            const int di = ci - i0, dj = cj - j0;
            if (v && d != kNoDecode && (int)(d >> 26) == f && di >= -7 && di <= 8 && dj >= -7 && dj <= 8)
                sig_set(sig, ci, cj);
            else
                compact = false;
        }
    }
}

// A footprint is "long" unless all its cells are valid level-13 cells of one
// face inside an 8 x 8 window: then every prefix of it is compact at every
// one of its quads.
__device__ __forceinline__ bool long_cells_dec(const uint32_t *dec, int64_t n)
{
    int f0 = -1, imin = 0, imax = 0, jmin = 0, jmax = 0;
    for (int64_t k = 0; k < n; k++) {
        const uint32_t d = dec[k];
        if (d == kNoDecode) return true;
        const int f = (int)(d >> 26), i = (int)((d >> 13) & 8191u), j = (int)(d & 8191u);
        if (k == 0) {
            f0 = f;
            imin = imax = i;
            jmin = jmax = j;
        } else {
            if (f != f0) return true;
            imin = min(imin, i);
            imax = max(imax, i);
            jmin = min(jmin, j);
            jmax = max(jmax, j);
        }
    }
    return imax - imin > 7 || jmax - jmin > 7;
}

// True iff the query (cells qc[0..nq)) and the entity share no cell < c.
// Block merge: B cells of each list per step, all B x B pairs compared in
// registers, then the block with the smaller last cell advances (both on a
// tie).  Cells >= c never count.
template <int B>
__device__ __attribute__((noinline)) bool no_smaller_shared(const IndexView &a, uint32_t ent, uint64_t c, const uint64_t *qc, int64_t nq)
{
    const uint64_t *ec = a.e_cells + a.e_offs[ent];
    const int64_t ne = a.e_offs[ent + 1] - a.e_offs[ent];
    int64_t i = 0, j = 0;
    while (i < nq && j < ne) {
        uint64_t x[B], y[B];
#pragma unroll
        for (int t = 0; t < B; t++) {
            x[t] = i + t < nq ? qc[i + t] : c;
            y[t] = j + t < ne ? ec[j + t] : c;
        }
        if (x[0] >= c || y[0] >= c) break;
        bool hit = false;
#pragma unroll
        for (int p = 0; p < B; p++)
#pragma unroll
            for (int t = 0; t < B; t++) hit |= (x[p] == y[t]) & (x[p] < c);
        if (hit) return false;
        const uint64_t xl = x[B - 1], yl = y[B - 1];
        if (xl <= yl) i += B;
        if (yl <= xl) j += B;
    }
    return true;
}

__device__ __forceinline__ unsigned long long wave_or(unsigned long long x)
{
    for (int o = 32; o > 0; o >>= 1) x |= __shfl_xor(x, o);
    return x;
}
// One atomic per wave for a per-lane count.
__device__ __forceinline__ void wave_count(bool p, unsigned long long *cnt)
{
    const unsigned long long m = __ballot(p);
    if (m && (threadIdx.x & 63) == (unsigned)__builtin_ctzll(m)) atomicAdd(cnt, (unsigned long long)__popcll(m));
}

// ============================================================== build kernels
__global__ void k_expand(int64_t n, const int64_t *offs, uint32_t *val)
{
    const int64_t e = tid64();
    if (e >= n) return;
    for (int64_t k = offs[e]; k < offs[e + 1]; k++) val[k] = (uint32_t)e;
}

// Any entity whose cell list is not strictly increasing (then the build takes
// the general path: sort + unique with multiplicities).
__global__ void k_check_sorted(int64_t P, const uint32_t *ent, const uint64_t *cells, unsigned int *bad)
{
    const int64_t i = tid64();
    const bool b = i > 0 && i < P && ent[i] == ent[i - 1] && cells[i] <= cells[i - 1];
    if (__ballot(b) && (threadIdx.x & 63) == 0) atomicOr(bad, 1u);
}

// General path: e_offs from the entity ids of the (entity, cell)-sorted unique
// positions (entities without cells get empty ranges).
__global__ void k_offs_from_sorted(int64_t Pu, const uint32_t *pent, int64_t n, int64_t *e_offs)
{
    const int64_t r = tid64();
    if (r >= Pu) return;
    const int64_t lo = r == 0 ? 0 : (int64_t)pent[r - 1] + 1, hi = pent[r];
    for (int64_t e = lo; e <= hi; e++) e_offs[e] = r;
    if (r == Pu - 1)
        for (int64_t e = (int64_t)pent[r] + 1; e <= n; e++) e_offs[e] = Pu;
}

__global__ void k_decode(int64_t P, const uint64_t *cells, uint32_t *dec)
{
    const int64_t i = tid64();
    if (i < P) dec[i] = decode13(cells[i]);
}

__device__ __forceinline__ bool row_included(long long t1) { return t1 != INT64_MIN; }  // stored NULL end: never matches
// |t1 - t0| as unsigned; a NULL start (INT64_MIN) is unbounded.
__device__ __forceinline__ unsigned long long duration(long long t0, long long t1)
{
    if (t0 == INT64_MIN) return ~0ull;
    return t0 < t1 ? (unsigned long long)t1 - (unsigned long long)t0 : (unsigned long long)t0 - (unsigned long long)t1;
}

// Per entity: long-footprint flag, duration histogram (bit length of the
// duration; bin 64 = unbounded) and the range of interval starts m.
__global__ void k_entity_info(int64_t n, const int64_t *e_offs, const uint32_t *dec, const int64_t *t0,
                              const int64_t *t1, uint8_t *elong, unsigned long long *hist, unsigned long long *mm)
{
    __shared__ unsigned long long sh[65];
    for (int i = threadIdx.x; i < 65; i += blockDim.x) sh[i] = 0;
    __syncthreads();
    const int64_t e = tid64();
    unsigned long long lo = ~0ull, hi = 0;
    if (e < n) {
        elong[e] = long_cells_dec(dec + e_offs[e], e_offs[e + 1] - e_offs[e]) ? 1 : 0;
        const long long a = t0[e], b = t1[e];
        if (row_included(b)) {
            const unsigned long long d = duration(a, b);
            const int bin = d == ~0ull ? 64 : (d == 0 ? 0 : 64 - __builtin_clzll(d));
            atomicAdd(&sh[bin], 1ull);
            if (a != INT64_MIN) {
                lo = order_key(tmin2(a, b));
                hi = lo;
            }
        }
    }
    for (int o = 32; o > 0; o >>= 1) {
        lo = min(lo, __shfl_xor(lo, o));
        hi = max(hi, __shfl_xor(hi, o));
    }
    if ((threadIdx.x & 63) == 0 && hi) {
        atomicMin(&mm[0], lo);
        atomicMax(&mm[1], hi);
    }
    __syncthreads();
    for (int i = threadIdx.x; i < 65; i += blockDim.x)
        if (sh[i]) atomicAdd(&hist[i], sh[i]);
}

// dcap = the largest duration of a regular entity (duration <= thr).
__global__ void k_dcap(int64_t n, const int64_t *t0, const int64_t *t1, unsigned long long thr, unsigned long long *dmax)
{
    const int64_t e = tid64();
    unsigned long long d = 0;
    if (e < n && row_included(t1[e])) {
        const unsigned long long x = duration(t0[e], t1[e]);
        if (x <= thr) d = x;
    }
    for (int o = 32; o > 0; o >>= 1) d = max(d, __shfl_xor(d, o));
    if ((threadIdx.x & 63) == 0 && d) atomicMax(dmax, d);
}

// Range of the group keys (cell >> gshift) over the regular in-range cells of
// included rows.
__global__ void k_dense_range(int64_t P, const uint64_t *cells, const uint32_t *pent, const int64_t *t1, uint64_t lo,
                              uint64_t hi, int gshift, unsigned long long *mm, unsigned long long *n_irr)
{
    const int64_t i = tid64();
    unsigned long long kmn = ~0ull, kmx = 0;
    bool irr = false;
    if (i < P) {
        const uint64_t c = cells[i];
        if (c >= lo && c <= hi && row_included(t1[pent[i]])) {
            if (is_regular(c)) kmn = kmx = c >> gshift;
            else irr = true;
        }
    }
    for (int o = 32; o > 0; o >>= 1) {
        kmn = min(kmn, __shfl_xor(kmn, o));
        kmx = max(kmx, __shfl_xor(kmx, o));
    }
    if ((threadIdx.x & 63) == 0 && kmn != ~0ull) {
        atomicMin(&mm[0], kmn);
        atomicMax(&mm[1], kmx);
    }
    wave_count(irr, n_irr);
}

// Cells and quad heads (the first of an entity's cells in a quad) among the
// in-range cells of included rows: the grain choice of the build.
__global__ void k_grain_counts(int64_t P, const uint64_t *cells, const uint32_t *pent, const int64_t *t1, uint64_t lo,
                               uint64_t hi, unsigned long long *cnt)
{
    const int64_t i = tid64();
    bool in = false, head = false;
    if (i < P) {
        const uint64_t c = cells[i];
        in = c >= lo && c <= hi && row_included(t1[pent[i]]);
        head = in && (i == 0 || pent[i - 1] != pent[i] || !same_quad(cells[i - 1], c, kQuadShift));
    }
    wave_count(in, &cnt[0]);
    wave_count(head, &cnt[1]);
}

struct BuildCtx {
    const uint64_t *cells;  // e_cells
    const uint32_t *pent;   // entity of each e_cells position
    const int64_t *t0, *t1;
    uint64_t lo, hi;
    int gshift;
    // e_cells position i heads a posting: the first of its entity's cells in
    // its quad (a quad-aligned range holds all of them or none)
    __device__ bool posting(int64_t i) const
    {
        const uint64_t c = cells[i];
        if (!(c >= lo && c <= hi && row_included(t1[pent[i]]))) return false;
        return i == 0 || pent[i - 1] != pent[i] || !same_quad(cells[i - 1], c, gshift);
    }
    __device__ bool in_range(int64_t i) const
    {
        const uint64_t c = cells[i];
        return c >= lo && c <= hi && row_included(t1[pent[i]]);
    }
};

struct PredPosting {
    BuildCtx b;
    __device__ bool operator()(int64_t i) const { return b.posting(i); }
};
struct EmitPostingKey {  // (order_key(m), position)
    BuildCtx b;
    unsigned long long *key;
    uint32_t *val;
    __device__ void operator()(int64_t i, int64_t r) const
    {
        const uint32_t e = b.pent[i];
        key[r] = order_key(tmin2(b.t0[e], b.t1[e]));
        val[r] = (uint32_t)i;
    }
};
struct PredIrr {
    BuildCtx b;
    __device__ bool operator()(int64_t i) const { return b.in_range(i) && !is_regular(b.cells[i]); }
};
struct EmitIrr {
    const uint64_t *cells;
    uint64_t *out;
    __device__ void operator()(int64_t i, int64_t r) const { out[r] = cells[i]; }
};
struct PredRunStart64 {
    const uint64_t *k;
    __device__ bool operator()(int64_t i) const { return i == 0 || k[i] != k[i - 1]; }
};
struct EmitCopy64 {
    const uint64_t *k;
    uint64_t *out;
    __device__ void operator()(int64_t i, int64_t r) const { out[r] = k[i]; }
};
// General path: unique (entity, cell) runs -> e_cells, pent, multiplicity.
struct PredUniquePair {
    const uint32_t *ent;
    const uint64_t *cell;
    __device__ bool operator()(int64_t i) const { return i == 0 || ent[i] != ent[i - 1] || cell[i] != cell[i - 1]; }
};
struct EmitUniquePair {
    int64_t P;
    const uint32_t *ent;
    const uint64_t *cell;
    uint64_t *e_cells;
    uint32_t *pent;
    uint32_t *mult;
    unsigned long long *big;  // set when a multiplicity exceeds the quad grain's 8 bits per child
    __device__ void operator()(int64_t i, int64_t r) const
    {
        uint32_t m = 1;
        while (i + m < P && ent[i + m] == ent[i] && cell[i + m] == cell[i]) m++;
        e_cells[r] = cell[i];
        pent[r] = ent[i];
        mult[r] = m;
        if (m > 255u) atomicMax(big, (unsigned long long)m);
    }
};

__device__ __forceinline__ uint32_t slot_of(const IndexView &a, uint64_t c)
{
    uint32_t s = kNoSlot;
    find_slot(a, c, s);
    return s;
}

// Postings per slot (the altitude bands split the dense slots only).
__global__ void k_slot_hist(int64_t NP, IndexView a, const uint32_t *pos, const uint64_t *cells, uint32_t *scnt)
{
    const int64_t j = tid64();
    if (j >= NP) return;
    atomicAdd(&scnt[slot_of(a, cells[pos[j]])], 1u);
}

// Slots with at least `dense` postings (do any bands apply?).
__global__ void k_dense_slots(int64_t ns, const uint32_t *scnt, uint32_t dense, unsigned long long *cnt)
{
    const int64_t s = tid64();
    wave_count(s < ns && scnt[s] >= dense, cnt);
}

struct BandThr {
    float v[7];  // alt_lo quantile edges: band = #{v[b] <= alt_lo}
};

// Second sort key of every posting (already sorted by m): slot << 1 | long
// (kshift 1), or with altitude bands slot << 4 | long << 3 | band (kshift 4;
// band 0 unless the slot is dense and the posting regular).
__global__ void k_slot_keys(int64_t NP, IndexView a, const uint32_t *pos, const uint64_t *cells, const uint32_t *pent,
                            const int64_t *t0, const int64_t *t1, unsigned long long thr, int kshift,
                            const uint32_t *scnt, uint32_t dense, const float *alo, BandThr bt, int nb, uint32_t *key)
{
    const int64_t j = tid64();
    if (j >= NP) return;
    const uint32_t i = pos[j];
    const uint32_t e = pent[i];
    const bool lng = duration(t0[e], t1[e]) > thr;
    const uint32_t sl = slot_of(a, cells[i]);
    if (kshift == 1) {
        key[j] = sl << 1 | (lng ? 1u : 0u);
        return;
    }
    uint32_t band = 0;
    if (!lng && scnt[sl] >= dense) {
        const float x = alo[e];  // (NaN: band 0)
        for (int b = 0; b < nb - 1; b++) band += x >= bt.v[b] ? 1u : 0u;
    }
    key[j] = sl << 4 | (lng ? 8u : 0u) | band;
}

// Posting attributes in final order: the quad's cell mask (the entity's run
// of cells in the quad, <= 4), per-child multiplicities, the near-prefix
// signature of its cells below the quad.
__global__ void k_gather(int64_t NP, const uint32_t *pos, const uint32_t *pent, const int64_t *e_offs,
                         const uint64_t *e_cells, const uint32_t *dec, const uint8_t *elong, const float *alo,
                         const float *ahi, const int64_t *t0, const int64_t *t1, const int32_t *owner,
                         const uint32_t *mult, int gshift, uint32_t *b_e, uint8_t *b_meta, float2 *b_alt,
                         longlong2 *b_t, ulonglong2 *b_sig, int32_t *b_owner, uint32_t *b_mult,
                         unsigned long long *nlongfp)
{
    const int64_t j = tid64();
    bool lf = false;
    if (j < NP) {
        const uint32_t i = pos[j];
        const uint32_t e = pent[i];
        const int64_t o = e_offs[e], oe = e_offs[e + 1];
        const uint64_t c = e_cells[i];
        uint32_t mask = child_bit(c, gshift), mm = 0;
        // (quads: 8 bits per child -- the build takes the cell grain when a
        // multiplicity exceeds 255 -- cells: the whole word)
        if (mult) mm = gshift == kCellShift ? mult[i] : min(mult[i], 255u) << (8u * (uint32_t)__builtin_ctz(mask));
        for (int64_t r = (int64_t)i + 1; r < oe && r < (int64_t)i + 4; r++) {
            const uint64_t cr = e_cells[r];
            if (!same_quad(c, cr, gshift)) break;
            const uint32_t b = child_bit(cr, gshift);
            mask |= b;
            if (mult) mm |= min(mult[r], 255u) << (8u * (uint32_t)__builtin_ctz(b));
        }
        Sig256 sig;
        bool compact = false;
        prefix_sig_quad(dec + o, (int64_t)i - o, dec[i], sig, compact);
        lf = elong[e] != 0;
        b_e[j] = e | ((int64_t)i == o ? kFirstBit : 0u);
        b_meta[j] = (uint8_t)((compact ? kMetaCompact : 0) | (lf ? kMetaLongFp : 0) | mask);
        b_alt[j] = make_float2(alo[e], ahi[e]);
        b_t[j] = make_longlong2(t0[e], t1[e]);
        b_sig[2 * j] = make_ulonglong2(sig.w[0], sig.w[1]);
        b_sig[2 * j + 1] = make_ulonglong2(sig.w[2], sig.w[3]);
        if (owner) b_owner[j] = owner[e];
        if (mult) b_mult[j] = mm;
    }
    wave_count(lf, nlongfp);
}

// Slot boundaries of the sorted postings: first / end / end of the regular
// part (positions + 1; 0 = unset), band starts (bfirst, with bands), the
// distinct-cell count, long postings.
__global__ void k_slot_bounds(int64_t NP, const uint32_t *key, int kshift, uint32_t *sfirst, uint32_t *send,
                              uint32_t *sreg, uint32_t *bfirst, unsigned long long *stat)
{
    const int64_t j = tid64();
    bool run = false, lng = false;
    if (j < NP) {
        const uint32_t k = key[j], s = k >> kshift, lb = (uint32_t)kshift - 1u;
        const bool first = j == 0 || (key[j - 1] >> kshift) != s;
        const bool last = j == NP - 1 || (key[j + 1] >> kshift) != s;
        lng = ((k >> lb) & 1u) != 0;
        if (first) sfirst[s] = (uint32_t)j + 1u;
        if (last) send[s] = (uint32_t)j + 1u;
        if (!lng && (last || ((key[j + 1] >> lb) & 1u))) sreg[s] = (uint32_t)j + 1u;
        if (bfirst && !lng && (first || key[j - 1] != k)) bfirst[(int64_t)s * 8 + (k & 7u)] = (uint32_t)j + 1u;
        run = first;
    }
    wave_count(run, &stat[0]);
    wave_count(lng, &stat[1]);
}

__global__ void k_slot_counts(int64_t ns, const uint32_t *sfirst, const uint32_t *send, const uint32_t *sreg,
                              const uint32_t *bfirst, int64_t *cnt, uint32_t *nreg, uint32_t *sband,
                              unsigned long long *maxc)
{
    const int64_t s = tid64();
    unsigned long long c = 0;
    if (s < ns) {
        const uint32_t f = sfirst[s];
        c = f ? send[s] - f + 1 : 0;
        cnt[s] = (int64_t)c;
        const uint32_t nr = (f && sreg[s]) ? sreg[s] - f + 1 : 0;
        nreg[s] = nr;
        if (sband) {  // band starts relative to the slot; an empty band starts where the next one does
            uint32_t next = nr, rel[8];
            for (int b = 7; b >= 0; b--) {
                const uint32_t bf = bfirst[s * 8 + b];
                if (f && bf) next = bf - f;
                rel[b] = next;
            }
            uint4 *o = reinterpret_cast<uint4 *>(sband + s * 8);
            o[0] = make_uint4(rel[0], rel[1], rel[2], rel[3]);
            o[1] = make_uint4(rel[4], rel[5], rel[6], rel[7]);
        }
    }
    for (int o = 32; o > 0; o >>= 1) c = max(c, __shfl_xor(c, o));
    if ((threadIdx.x & 63) == 0 && c) atomicMax(maxc, c);
}

// Slots holding a long-footprint posting: their join units take the long
// join variant (the others' postings all have compact prefixes).
__global__ void k_slot_lfp(int64_t NP, const uint32_t *key, int kshift, const uint8_t *b_meta, uint8_t *s_lfp)
{
    const int64_t j = tid64();
    if (j < NP && (b_meta[j] & kMetaLongFp)) s_lfp[key[j] >> kshift] = 1;
}

// Every k-th alt_lo (the band quantiles are taken on the host from these).
__global__ void k_sample_f32(int64_t n, const float *x, int64_t ns, float *out)
{
    const int64_t k = tid64();
    if (k < ns) out[k] = x[(int64_t)((double)k * (double)n / (double)ns)];
}

__global__ void k_owner_keys(int64_t n, const int32_t *owner, uint32_t *key, uint32_t *val)
{
    const int64_t e = tid64();
    if (e >= n) return;
    key[e] = (uint32_t)owner[e] ^ 0x80000000u;  // signed order as unsigned
    val[e] = (uint32_t)e;
}

__global__ void k_u64_store(int64_t n, const int64_t *a, uint64_t *b)
{
    const int64_t k = tid64();
    if (k < n) b[k] = (uint64_t)a[k];
}

// ============================================================== search kernels
struct QueryView {
    int64_t nq;
    const int64_t *offs;
    const uint64_t *cells;
    const float *alo, *ahi;
    const int64_t *tlo, *thi;
    const int32_t *owner;
};

// Query record, one per query cell.
struct alignas(16) QRec {
    long long tlo, thi;
    float alo, ahi;
    uint32_t qv;   // query | kRank0 | kCompactQ | kLongQ | the query's cells in the quad << kQMaskShift
    int32_t own;   // owner filter (-1: any)
    unsigned long long sig[4];  // near-prefix signature of the query's cells before this one
};
static_assert(sizeof(QRec) == 64, "QRec layout");



// ceil(log2(thi - tlo)) of a non-empty window (0 for a point), -1 if empty.
__device__ __forceinline__ int win_bucket(long long tlo, long long thi)
{
    if (thi < tlo) return -1;
    const unsigned long long w = (unsigned long long)thi - (unsigned long long)tlo;
    return w <= 1ull ? (int)w : 64 - __clzll(w - 1ull);
}

// Histogram of the batch's window buckets (one LDS histogram per block).
__global__ __launch_bounds__(kBlock) void k_qwin(int64_t nq, const int64_t *tlo, const int64_t *thi,
                                                 unsigned long long *hist)
{
    __shared__ unsigned int h[kWinBuckets];
    for (int i = threadIdx.x; i < kWinBuckets; i += kBlock) h[i] = 0;
    __syncthreads();
    for (int64_t q = (int64_t)blockIdx.x * kBlock + threadIdx.x; q < nq; q += (int64_t)gridDim.x * kBlock) {
        const int b = win_bucket(tlo[q], thi[q]);
        if (b >= 0) atomicAdd(&h[b], 1u);
    }
    __syncthreads();
    for (int i = threadIdx.x; i < kWinBuckets; i += kBlock)
        if (h[i]) atomicAdd(&hist[i], (unsigned long long)h[i]);
}

// The wide threshold's log2 from the histogram: windows with bucket <= b are
// narrow.  A narrow record is loaded by the tiles of its cell whose starts lie
// within (dqmax + dcap) of its start, a wide one by every tile (the index's
// time span H); the cost of b is narrow(b) * (2^b + dcap) + wide(b) * H.
__device__ __forceinline__ int choose_wide_log(const unsigned long long *hist, double dcap, double span)
{
    double tot = 0;
    for (int i = 0; i < kWinBuckets; i++) tot += (double)hist[i];
    double nar = 0, best = 1e300;
    int bb = 64;
    for (int b = 0; b < kWinBuckets; b++) {
        nar += (double)hist[b];
        const double c = nar * (ldexp(1.0, b) + dcap) + (tot - nar) * span;
        if (c < best) {
            best = c;
            bb = b;
        }
    }
    return bb;
}

// Per query cell: its query, level-13 decode and slot (kNoSlot when the
// index holds no posting for the cell); per query the long flag
// (long_cells) from per-query LDS min/max/face-mask reductions.  One block
// per 256 queries: their cell offsets go to LDS, the block's cells are then
// visited coalesced, each finding its query by binary search in LDS.
// Per query cell: its query, decode and slot (kNoSlot unless the cell is the
// first of its query's cells in its quad -- the quad's record -- and the
// quad holds postings), and its rank among its query's records with postings
// (vpre[k] - qvb[q]); per query: the long flag and the count of records with
// postings.  One block per 256 queries, their cells in kBlock-wide steps.
__global__ __launch_bounds__(kBlock) void k_cell_query(IndexView a, int64_t nq, const int64_t *offs,
                                                       const uint64_t *cells, uint32_t *cq, uint32_t *dec,
                                                       uint32_t *cslot, uint8_t *qlong, uint32_t *vpre,
                                                       uint32_t *qvb, uint32_t *qvalid, unsigned long long *nlong)
{
    __shared__ int64_t so[kBlock + 1];
    __shared__ int s_imin[kBlock], s_imax[kBlock], s_jmin[kBlock], s_jmax[kBlock];
    __shared__ uint32_t s_face[kBlock];  // bit f: a cell on face f; bit 8: an undecodable cell
    __shared__ uint32_t s_cnt[kBlock];   // cells with postings per query
    __shared__ uint32_t s_wsum[kBlock / 64];
    const int64_t q0 = (int64_t)blockIdx.x * kBlock;
    const int nb = (int)(nq - q0 < (int64_t)kBlock ? nq - q0 : (int64_t)kBlock);
    const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
    for (int i = threadIdx.x; i <= nb; i += kBlock) so[i] = offs[q0 + i];
    s_imin[threadIdx.x] = s_jmin[threadIdx.x] = 1 << 30;
    s_imax[threadIdx.x] = s_jmax[threadIdx.x] = -1;
    s_face[threadIdx.x] = 0;
    s_cnt[threadIdx.x] = 0;
    __syncthreads();
    const int64_t k1 = so[nb];
    uint32_t carry = 0;  // cells with postings before this step (block-relative)
    for (int64_t base = so[0]; base < k1; base += kBlock) {
        const int64_t k = base + threadIdx.x;
        bool valid = false;
        int lo = 0;
        if (k < k1) {
            int hi = nb;  // so[lo] <= k < so[hi]
            while (hi - lo > 1) {
                const int mid = (lo + hi) >> 1;
                if (so[mid] <= k) lo = mid;
                else hi = mid;
            }
            cq[k] = (uint32_t)(q0 + lo);
            const uint64_t c = cells[k];
            const uint32_t d = decode13(c);
            dec[k] = d;
            // one record per (query, quad): the quad's first cell in the
            // query's sorted list carries it
            const bool head = k == so[lo] || !same_quad(cells[k - 1], c, a.gshift);
            uint32_t sl = kNoSlot;
            if (head && find_slot(a, c, sl) && a.s_post[sl + 1] == a.s_post[sl]) sl = kNoSlot;
            cslot[k] = sl;
            valid = sl != kNoSlot;
            if (valid) atomicAdd(&s_cnt[lo], 1u);
            if (d != kNoDecode) {
                atomicOr(&s_face[lo], 1u << (d >> 26));
                atomicMin(&s_imin[lo], (int)((d >> 13) & 8191u));
                atomicMax(&s_imax[lo], (int)((d >> 13) & 8191u));
                atomicMin(&s_jmin[lo], (int)(d & 8191u));
                atomicMax(&s_jmax[lo], (int)(d & 8191u));
            } else {
                atomicOr(&s_face[lo], 1u << 8);
            }
        }
        // block exclusive scan of the valid flags
        const unsigned long long m = __ballot(valid);
        if (lane == 0) s_wsum[wv] = (uint32_t)__popcll(m);
        __syncthreads();
        uint32_t pre = carry + __builtin_amdgcn_mbcnt_hi((uint32_t)(m >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)m, 0u)),
                 tot = 0;
#pragma unroll
        for (int i = 0; i < kBlock / 64; i++) {
            pre += i < wv ? s_wsum[i] : 0u;
            tot += s_wsum[i];
        }
        if (k < k1) {
            vpre[k] = pre;
            if (k == so[lo]) qvb[q0 + lo] = pre;
        }
        carry += tot;
        __syncthreads();
    }
    const int t = threadIdx.x;
    bool is_long = false;
    if (t < nb) {
        const uint32_t fm = s_face[t];
        // no cells: not long; else undecodable / multi-face / wide span
        is_long = fm != 0 && ((fm >> 8) != 0 || __popc(fm) > 1 || s_imax[t] - s_imin[t] > 7 ||
                              s_jmax[t] - s_jmin[t] > 7);
        qlong[q0 + t] = is_long ? 1 : 0;
        qvalid[q0 + t] = s_cnt[t];
    }
    wave_count(is_long, nlong);
}

// Quantised start: (t - tbase) >> qshift, clamped to [0, kWideKey - 1]
// (monotone, so a search on it brackets every record of a time range).
__device__ __forceinline__ uint32_t order_q(long long t, long long tbase, int qshift)
{
    const unsigned long long d = t <= tbase ? 0ull : ((unsigned long long)t - (unsigned long long)tbase) >> qshift;
    return d >= (unsigned long long)(kWideKey - 1) ? kWideKey - 1 : (uint32_t)d;
}

// Query order key: quantised tlo, | kWideBit for the wide windows; the
// widest narrow window of the batch -> *dqmax.  Every block derives the same
// threshold from the batch's window histogram (k_qwin).
__global__ __launch_bounds__(kBlock) void k_qorder(int64_t nq, const int64_t *tlo, const int64_t *thi, long long tbase,
                                                   int qshift, double dcap, const unsigned long long *whist,
                                                   uint32_t *key, uint32_t *val, unsigned long long *dqmax)
{
    __shared__ unsigned long long wmax[kBlock / 64];
    __shared__ int s_wb;
    if (threadIdx.x == 0) s_wb = choose_wide_log(whist, dcap, ldexp(1.0, kOrderBits + qshift));
    __syncthreads();
    const int wb = s_wb;
    const int64_t q = tid64();
    unsigned long long dq = 0;
    if (q < nq) {
        const long long a = tlo[q], b = thi[q];
        // wide queries are ordered by start too (kWideBit rides above the
        // sorted bits): a regular tile's wide records are then a prefix of
        // the cell's wide run, cut at the tile's latest possible end
        uint32_t k = order_q(a, tbase, qshift);
        if (win_bucket(a, b) <= wb) {  // narrow (or empty: matches nothing)
            if (b >= a) dq = (unsigned long long)b - (unsigned long long)a;
        } else {
            k |= kWideBit;
        }
        key[q] = k;
        val[q] = (uint32_t)q;
    }
    for (int o = 32; o > 0; o >>= 1) dq = max(dq, __shfl_xor(dq, o));
    if ((threadIdx.x & 63) == 0) wmax[threadIdx.x >> 6] = dq;
    __syncthreads();
    if (threadIdx.x == 0) {  // one atomic per block, on one of kRegions slots (readers take the max)
        unsigned long long m = 0;
        for (int i = 0; i < kBlock / 64; i++) m = max(m, wmax[i]);
        if (m) atomicMax(&dqmax[(blockIdx.x % kRegions) * kRegStride], m);
    }
}

// Per query (in order rank r): its cells with postings.
__global__ void k_qcount(int64_t nq, const uint32_t *perm, const uint32_t *qvalid, int64_t *cnt, uint32_t *rank)
{
    const int64_t r = tid64();
    if (r >= nq) return;
    const uint32_t q = perm[r];
    cnt[r] = qvalid[q];
    rank[q] = (uint32_t)r;
}

// One record per (query, group) with postings -- the group's first cell in
// the query's sorted list carries it -- written at its key's position w =
// off[rank of its query] + its rank among the query's records (the keys in
// query order, each query's groups in cell order): the key (slot << 1 |
// wide), its value (w | the query's quantised start << 32: after the sort by
// slot the unit-range searches probe one 8-B value per step and the join
// finds the record at the low word) and the 64-B record -- time window,
// altitudes, owner, flags, the query's cells in the group, and the
// near-prefix signature of its cells below the group (the prefix's decodes
// loaded 8 at a time).  (Round 5 fused the key emission into this pass and
// writes records only where a key points: half the cells of a quad-grain
// batch carry none.  Round 6: records at their cell index instead -- one
// coalesced store per block, k_qrecs 0.231 -> 0.215 ms -- left a sparse
// array whose gathers cost the join more: join phase +0.03 ms on configs[1]
// and [2], profiles/r06x.)
__global__ __launch_bounds__(kBlock) void k_qrecs(QueryView qv, int64_t nqc, const uint32_t *cq, const uint32_t *dec,
                                                  const uint32_t *cslot, const uint8_t *qlong, const uint32_t *vpre,
                                                  const uint32_t *qvb, const uint32_t *rank, const uint32_t *okey,
                                                  const int64_t *off, int gshift, uint32_t *key, uint64_t *val,
                                                  QRec *recs)
{
    const int64_t k = tid64();
    if (k >= nqc) return;
    const uint32_t sl = cslot[k];
    if (sl == kNoSlot) return;
    const uint32_t q = cq[k], r = rank[q], ok = okey[r];
    const int64_t w = off[r] + (int64_t)(vpre[k] - qvb[q]);
    key[w] = sl << 1 | ((ok & kWideBit) ? 1u : 0u);
    val[w] = (uint64_t)w | (uint64_t)(ok & (kWideBit - 1u)) << 32;
    const int64_t c0 = qv.offs[q], c1 = qv.offs[q + 1];
    const uint64_t c = qv.cells[k];
    uint32_t mask = child_bit(c, gshift);
    for (int64_t x = k + 1; x < c1 && x < k + 4; x++) {
        const uint64_t cx = qv.cells[x];
        if (!same_quad(c, cx, gshift)) break;
        mask |= child_bit(cx, gshift);
    }
    Sig256 sig;
    bool compact = false;
    prefix_sig_quad(dec + c0, k - c0, dec[k], sig, compact);
    QRec rec;
    rec.tlo = qv.tlo[q];
    rec.thi = qv.thi[q];
    rec.alo = qv.alo[q];
    rec.ahi = qv.ahi[q];
    rec.qv = q | (k == c0 ? kRank0 : 0u) | (compact ? kCompactQ : 0u) | (qlong[q] ? kLongQ : 0u) |
             (mask << kQMaskShift);
    rec.own = qv.owner ? qv.owner[q] : -1;
    rec.sig[0] = sig.w[0];
    rec.sig[1] = sig.w[1];
    rec.sig[2] = sig.w[2];
    rec.sig[3] = sig.w[3];
    const int4 *src = reinterpret_cast<const int4 *>(&rec);
    int4 *dst = reinterpret_cast<int4 *>(recs + w);
#pragma unroll
    for (int u = 0; u < 4; u++) dst[u] = src[u];
}

constexpr int64_t kRecPermuteMin = 8192;  // largest group (postings) from which records go in key order
// The records in key (slot) order: rec2[i] = recs[low word of sval[i]],
// four threads per 64-B record (16 B each, coalesced writes), over the
// device key count.  A join unit's records are then one contiguous run that
// every tile of the slot re-reads from L2, instead of 64-B gathers across the
// query-ordered array (round 6: those gathers were most of k_join's HBM reads).
__global__ void k_rec_permute(const int64_t *dnkeys, const uint64_t *sval, const QRec *recs, QRec *rec2)
{
    const int64_t t = tid64(), i = t >> 2;
    if (i >= *dnkeys) return;
    const int part = (int)(t & 3);
    const int4 *src = reinterpret_cast<const int4 *>(recs + (uint32_t)sval[i]);
    reinterpret_cast<int4 *>(rec2 + i)[part] = src[part];
}

// Lower / upper bound over a slot's regular postings (sorted by m).
__device__ __forceinline__ uint64_t lb_m(const longlong2 *bt, uint64_t lo, uint64_t hi, long long x)
{
    while (lo < hi) {  // first p with m(p) >= x
        const uint64_t mid = (lo + hi) >> 1;
        const longlong2 t = bt[mid];
        if (tmin2(t.x, t.y) < x) lo = mid + 1;
        else hi = mid;
    }
    return lo;
}
__device__ __forceinline__ uint64_t ub_m(const longlong2 *bt, uint64_t lo, uint64_t hi, long long x)
{
    while (lo < hi) {  // first p with m(p) > x
        const uint64_t mid = (lo + hi) >> 1;
        const longlong2 t = bt[mid];
        if (tmin2(t.x, t.y) <= x) lo = mid + 1;
        else hi = mid;
    }
    return lo;
}

// Inclusive prefix sum over the 64 lanes with DPP (no LDS round trips):
// row_shr 1/2/4/8 scan each 16-lane row, row_bcast 15 / 31 carry the row
// totals into the rows above (CDNA DPP; rows outside row_mask keep `old`=0).
__device__ __forceinline__ uint32_t wave_incl_scan(uint32_t x)
{
    x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x111, 0xf, 0xf, false);  // row_shr:1
    x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x112, 0xf, 0xf, false);  // row_shr:2
    x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x114, 0xf, 0xf, false);  // row_shr:4
    x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x118, 0xf, 0xf, false);  // row_shr:8
    x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x142, 0xa, 0xf, false);  // row_bcast:15 -> rows 1, 3
    x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x143, 0xc, 0xf, false);  // row_bcast:31 -> rows 2, 3
    return x;
}

// Wave maximum (lane 63 of a DPP max-scan; no LDS round trips).
__device__ __forceinline__ uint32_t wave_max(uint32_t x)
{
    x = max(x, (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x111, 0xf, 0xf, false));  // row_shr:1
    x = max(x, (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x112, 0xf, 0xf, false));  // row_shr:2
    x = max(x, (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x114, 0xf, 0xf, false));  // row_shr:4
    x = max(x, (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x118, 0xf, 0xf, false));  // row_shr:8
    x = max(x, (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x142, 0xa, 0xf, false));  // row_bcast:15
    x = max(x, (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x143, 0xc, 0xf, false));  // row_bcast:31
    return (uint32_t)__builtin_amdgcn_readlane((int)x, 63);
}

// Wave max / min of a float (no NaN) through an order-preserving u32 image.
__device__ __forceinline__ uint32_t f32_key(float x)
{
    const uint32_t u = __float_as_uint(x);
    return (u & 0x80000000u) ? ~u : (u | 0x80000000u);
}
__device__ __forceinline__ float f32_of_key(uint32_t k)
{
    return __uint_as_float((k & 0x80000000u) ? (k & 0x7fffffffu) : ~k);
}
__device__ __forceinline__ float wave_max_f(float x) { return f32_of_key(wave_max(f32_key(x))); }
__device__ __forceinline__ float wave_min_f(float x) { return f32_of_key(~wave_max(~f32_key(x))); }

// An upper bound (within 2^24 us) of the wave maximum of a 64-bit time, by a
// 32-bit DPP max of the times' top bits: the tile hull only needs to contain
// every posting's window (a looser hull stages a few more records; the
// per-lane tests stay exact).  ~8 VALU against ~32 for a 64-bit DPP max.
__device__ __forceinline__ long long wave_max_bound(long long x)
{
    const long long h = x >> 24;  // arithmetic: order preserving
    const int32_t c = h > (long long)INT32_MAX ? INT32_MAX : h < (long long)INT32_MIN ? INT32_MIN : (int32_t)h;
    const int32_t m = (int32_t)(wave_max((uint32_t)c ^ 0x80000000u) ^ 0x80000000u);
    return m == INT32_MAX ? LLONG_MAX : ((long long)m << 24) + ((1ll << 24) - 1);
}

__device__ __forceinline__ uint32_t lb_u32(const uint32_t *x, uint32_t lo, uint32_t hi, uint32_t v)
{
    while (lo < hi) {  // first index in [lo, hi) with x[i] >= v
        const uint32_t m = (lo + hi) >> 1;
        if (x[m] < v) lo = m + 1;
        else hi = m;
    }
    return lo;
}

// Join unit: one tile of <= 64 postings of one cell (a run of its regular
// postings in start order, or of its long-duration ones) x that cell's
// query records to test (positions in the sorted keys): narrow ones [n0, n1)
// -- for a regular tile the sub-range whose quantised start can meet the
// tile (unit_ranges) -- and wide ones [w0, w1); a long tile meets every
// record of the cell.  32 bytes.
constexpr uint32_t kUnitLong = 0x80000000u;  // np: long-duration tile
constexpr uint32_t kUnitBand = 0x40000000u;  // np: a tile of one altitude band (k_join stages by its altitude hull)
constexpr uint32_t kUnitFlags = kUnitLong | kUnitBand;
struct alignas(16) Unit {
    uint64_t p0;     // first posting
    uint32_t np;     // postings (1..64) | kUnitLong | kUnitBand
    uint32_t slot;
    uint32_t n0, n1;  // narrow records
    uint32_t w0, w1;  // wide records
};
static_assert(sizeof(Unit) == 32, "Unit layout");

// Narrow record sub-range of every regular tile: a narrow record (window <=
// dqmax) meets a posting only if tlo in [m - dqmax, max(t0, t1)], and over a
// start-sorted tile that is [m_first - dqmax, m_last + dcap]; the records'
// quantised starts (their order) bracket it by binary search, done by
// k_units as it writes each unit (round 4: one pass over the units fewer).
__device__ __forceinline__ uint32_t lb_q(const uint64_t *sv, uint32_t lo, uint32_t hi, uint32_t v)
{
    while (lo < hi) {  // first record in [lo, hi) with quantised start (sv's high word) >= v
        const uint32_t m = (lo + hi) >> 1;
        if ((uint32_t)(sv[m] >> 32) < v) lo = m + 1;
        else hi = m;
    }
    return lo;
}

// A banded slot's band starts relative to its first posting, rel[8] = the
// end of its regular part.
__device__ __forceinline__ void band_starts(const IndexView &a, uint32_t slot, uint32_t nreg, uint32_t rel[9])
{
    const uint4 *p = reinterpret_cast<const uint4 *>(a.s_band + (uint64_t)slot * 8);
    const uint4 x = p[0], y = p[1];
    rel[0] = x.x;
    rel[1] = x.y;
    rel[2] = x.z;
    rel[3] = x.w;
    rel[4] = y.x;
    rel[5] = y.y;
    rel[6] = y.z;
    rel[7] = y.w;
    rel[8] = nreg;
}

__device__ __forceinline__ void unit_ranges(const IndexView &a, Unit &d, const uint64_t *sq, long long dq, long long tbase,
                                            int qshift)
{
    if ((d.np & kUnitLong) || (d.n1 <= d.n0 && d.w1 <= d.w0)) return;
    {
        const longlong2 f = a.b_t[d.p0], l = a.b_t[d.p0 + d.np - 1];
        const long long m0 = tmin2(f.x, f.y), m1 = tmin2(l.x, l.y);
        const long long lo = m0 < LLONG_MIN + dq ? LLONG_MIN : m0 - dq;
        const long long hi = m1 > LLONG_MAX - a.dcap ? LLONG_MAX : m1 + a.dcap;
        const uint32_t qhi = order_q(hi, tbase, qshift) + 1u;
        if (d.n1 > d.n0) {
            const uint32_t n0 = lb_q(sq, d.n0, d.n1, order_q(lo, tbase, qshift));
            d.n1 = lb_q(sq, n0, d.n1, qhi);
            d.n0 = n0;
        }
        // wide records (start-ordered within the cell's wide run) starting
        // after every posting of the tile has ended meet none of them
        if (d.w1 > d.w0) d.w1 = lb_q(sq, d.w0, d.w1, qhi);
    }
}

// Join units, one wave per window of 64 sorted keys (grid-stride over the
// device key count): every lane that starts a cell (a run of equal slot)
// finds the cell's record ranges (within the window, or by binary search
// past it) and emits one unit per 64-posting tile of the cell's regular
// and long parts; slots come from one atomic per wave (region counters).
__global__ __launch_bounds__(kBlock) void k_units(IndexView a, const uint32_t *skey, const int64_t *dnkeys, Regions ur,
                                                  Unit *units, Regions url, Unit *units_l, uint32_t tp,
                                                  const uint64_t *sq, const unsigned long long *dqslots, long long tbase,
                                                  int qshift)
{
    __shared__ uint32_t s_xa[kBlock / 64][64];
    __shared__ uint64_t s_s0[kBlock / 64][64], s_sr[kBlock / 64][64], s_s1[kBlock / 64][64], s_bu[kBlock / 64][64];
    __shared__ uint4 s_par[kBlock / 64][64];  // ntr | lfp << 31, slot, first wide record, record end
    const int lane = threadIdx.x & 63;
    const uint32_t nkeys = (uint32_t)*dnkeys;
    const int64_t wave = (int64_t)blockIdx.x * (kBlock / 64) + (threadIdx.x >> 6);
    const int64_t nwaves = (int64_t)gridDim.x * (kBlock / 64);
    const int64_t nwin = ((int64_t)nkeys + 63) / 64;
    const int reg = (int)(blockIdx.x % kRegions);
    unsigned long long dqm = 0;
    for (int r = 0; r < kRegions; r++) dqm = max(dqm, dqslots[r * kRegStride]);
    const long long dq = (long long)min(dqm, 1ull << 62);
    for (int64_t win = wave; win < nwin; win += nwaves) {
        const uint32_t w0 = (uint32_t)(win * 64), wend = min(w0 + 64u, nkeys);
        const uint32_t p = w0 + (uint32_t)lane;
        const bool valid = p < nkeys;
        const uint32_t key = valid ? skey[p] : 0xffffffffu;
        const uint32_t prev = valid && p > 0 ? skey[p - 1] : 0xffffffffu;
        const bool cstart = valid && (p == 0 || (prev >> 1) != (key >> 1));
        const bool wstart = valid && (key & 1u) && (p == 0 || prev != key);
        const unsigned long long cm = __ballot(cstart), wm = __ballot(wstart);
        uint32_t nu = 0, rw = 0, re = 0, slot = key >> 1, ntr = 0;
        bool lfp = false;  // the cell holds long-footprint postings: its units go to the long queue
        uint64_t s0 = 0, sr = 0, s1 = 0;
        if (cstart) {
            const unsigned long long above = lane == 63 ? 0ull : (cm >> (lane + 1)) << (lane + 1);
            const uint32_t nxt = above ? w0 + (uint32_t)__builtin_ctzll(above) : 0xffffffffu;
            re = nxt != 0xffffffffu ? nxt : lb_u32(skey, wend, nkeys, (slot << 1 | 1u) + 1u);
            // the first wide record of the cell
            const unsigned long long wl = (wm >> lane) << lane;  // wide starts at or after this lane
            const uint32_t wpos = wl ? w0 + (uint32_t)__builtin_ctzll(wl) : 0xffffffffu;
            if (wpos < re) rw = wpos;
            else if (re <= wend) rw = re;
            else rw = lb_u32(skey, wend, re, slot << 1 | 1u);
            s0 = a.s_post[slot];
            s1 = a.s_post[slot + 1];
            sr = s0 + a.s_nreg[slot];
            if (a.s_band) {  // regular tiles per altitude band
                uint32_t rel[9];
                band_starts(a, slot, (uint32_t)(sr - s0), rel);
                int ne = 0;
                for (int b = 0; b < 8; b++) {
                    ntr += (rel[b + 1] - rel[b] + tp - 1) / tp;
                    ne += rel[b + 1] > rel[b] ? 1 : 0;
                }
                if (ne > 1) ntr |= kUnitBand;  // (a flag bit above any tile count)
            } else {
                ntr = (uint32_t)((sr - s0 + tp - 1) / tp);
            }
            nu = (ntr & ~kUnitBand) + (uint32_t)((s1 - sr + tp - 1) / tp);
            lfp = a.s_lfp[slot] != 0;
        }
        const uint32_t ns_ = lfp ? 0u : nu, nl_ = lfp ? nu : 0u;
        const uint32_t xs = wave_incl_scan(ns_), xl = wave_incl_scan(nl_);
        const uint32_t tots = (uint32_t)__builtin_amdgcn_readlane((int)xs, 63);
        const uint32_t totl = (uint32_t)__builtin_amdgcn_readlane((int)xl, 63);
        unsigned long long bs = 0, bl = 0;
        if (lane == 0 && tots) bs = atomicAdd(ur.counter(reg), (unsigned long long)tots);
        if (lane == 0 && totl) bl = atomicAdd(url.counter(reg), (unsigned long long)totl);
        bs = __shfl(bs, 0) + (xs - ns_);
        bl = __shfl(bl, 0) + (xl - nl_);
        // the wave's units written by all its lanes (a hot cell owns ~150
        // tiles: one lane per cell would loop that long while the rest idle):
        // each lane's cell parameters go to LDS, then lane u of every round
        // finds the cell of unit u by a search over the units' prefix
        const uint32_t xa = wave_incl_scan(nu);
        const uint32_t tot = (uint32_t)__builtin_amdgcn_readlane((int)xa, 63);
        const int wv = threadIdx.x >> 6;
        __builtin_amdgcn_wave_barrier();
        s_xa[wv][lane] = xa;
        s_s0[wv][lane] = s0;
        s_sr[wv][lane] = sr;
        s_s1[wv][lane] = s1;
        s_bu[wv][lane] = lfp ? bl : bs;
        s_par[wv][lane] = make_uint4(ntr | (lfp ? kUnitLong : 0u), slot, rw, re);
        __builtin_amdgcn_wave_barrier();
        for (uint32_t u = (uint32_t)lane; u < tot; u += 64) {
            int lo = 0, hi = 63;  // the first lane L with s_xa[L] > u
            while (lo < hi) {
                const int mid = (lo + hi) >> 1;
                if (s_xa[wv][mid] > u) hi = mid;
                else lo = mid + 1;
            }
            const uint32_t t = u - (lo ? s_xa[wv][lo - 1] : 0u);  // the unit's tile within its cell
            const uint4 pr = s_par[wv][lo];
            const uint32_t lntr = pr.x & ~kUnitFlags;
            const bool llfp = (pr.x & kUnitLong) != 0, lband = (pr.x & kUnitBand) != 0;
            const uint64_t l0 = s_s0[wv][lo], lr = s_sr[wv][lo], l1 = s_s1[wv][lo];
            Unit d;
            const bool lng = t >= lntr;
            uint64_t b = lng ? lr + (uint64_t)tp * (t - lntr) : l0 + (uint64_t)tp * t;
            uint64_t e = lng ? l1 : lr;
            if (!lng && a.s_band) {  // the tile's band: bands in order, each tiled from its start
                uint32_t rel[9];
                band_starts(a, pr.y, (uint32_t)(lr - l0), rel);
                uint32_t acc = 0;
                for (int k = 0; k < 8; k++) {
                    const uint32_t nt = (rel[k + 1] - rel[k] + tp - 1) / tp;
                    if (t < acc + nt) {
                        b = l0 + rel[k] + (uint64_t)tp * (t - acc);
                        e = l0 + rel[k + 1];
                        break;
                    }
                    acc += nt;
                }
            }
            d.p0 = b;
            d.np = (uint32_t)min((uint64_t)tp, e - b) | (lng ? kUnitLong : 0u);
            d.slot = pr.y;
            d.n0 = w0 + (uint32_t)lo;
            d.n1 = lng ? pr.w : pr.z;  // a long tile meets every record
            d.w0 = lng ? pr.w : pr.z;
            d.w1 = pr.w;
            unit_ranges(a, d, sq, dq, tbase, qshift);  // a regular tile's record sub-ranges
            if (lband && !lng) d.np |= kUnitBand;
            const unsigned long long wpos = s_bu[wv][lo] + t;
            const Regions &dr = llfp ? url : ur;
            Unit *du = llfp ? units_l : units;
            if ((int64_t)wpos < dr.cap) du[reg * dr.cap + (int64_t)wpos] = d;
        }
    }
}


__device__ __forceinline__ long long readlane64(long long v, int lane)
{
    const uint32_t lo = (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)v, lane);
    const uint32_t hi = (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)((unsigned long long)v >> 32), lane);
    return (long long)(((unsigned long long)hi << 32) | lo);
}

// Set bits of m below this lane.
__device__ __forceinline__ uint32_t mbcnt64(unsigned long long m)
{
    return __builtin_amdgcn_mbcnt_hi((uint32_t)(m >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)m, 0u));
}

// Output: pairs go straight to HBM in per-wave chunks of kOutChunk slots,
// each reserved with one atomic on the wave's region counter (kRegions
// counters: a single same-address counter saturates at ~88 atomics/us,
// MI355X_MICROARCH.md "dequeue").  The regions interleave at chunk
// granularity -- local chunk l of region r is global chunk l * kRegions + r
// -- so every region fills the bottom of the buffer: the holes below the
// total are only the waves' last, partly filled chunks and the few chunks of
// the regions' imbalance, which k_fix_* close.
constexpr int kOutChunkLog = 10, kOutChunk = 1 << kOutChunkLog, kRegionsLog = 3;  // (4096-pair chunks: no faster)
static_assert((1 << kOutChunkLog) == kOutChunk && (1 << kRegionsLog) == kRegions, "output layout");
struct OutStream {
    int64_t rcap;                  // slots per region (a multiple of kOutChunk)
    uint32_t *fills;               // per global chunk: entries written (0 = unreserved)
    unsigned long long *octr;      // kRegions reservation counters (local slots), kRegStride words apart
};
// Two streams: the pairs (q, e), final as written, and the long x long pairs
// the signatures cannot decide, as 64-bit keys (q << eb | e) << hbm | hbm
// hash bits of the pair, deduplicated after the join.
struct OutArgs {
    uint32_t *q, *e;
    OutStream ps;
    unsigned long long *tk;
    OutStream ts;
    int eb, hbm;
    unsigned long long *counter;   // [0] pairs [1] tagged keys [2] lane tests [3] broadcasts
};

__device__ __forceinline__ int uni32(int x) { return __builtin_amdgcn_readfirstlane(x); }
__device__ __forceinline__ unsigned long long uni64_lane0(unsigned long long x)
{
    return ((unsigned long long)(uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)(x >> 32), 0) << 32) |
           (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)x, 0);
}
__device__ __forceinline__ unsigned long long uni64(unsigned long long x)
{
    return ((unsigned long long)(uint32_t)__builtin_amdgcn_readfirstlane((int)(uint32_t)(x >> 32)) << 32) |
           (uint32_t)__builtin_amdgcn_readfirstlane((int)(uint32_t)x);
}

// Per-wave output state, wave-uniform by construction (readfirstlane keeps
// it in scalar registers: no exec-mask traffic around the chunk test).
struct WaveOut {
    unsigned long long base = 0;  // global slot of the current chunk
    int fill = kOutChunk;  // no chunk yet
    int have = 0;
    unsigned long long pairs = 0;  // wave-uniform
    // wave-uniform call: room for `total` (> 0) pairs.  The batch first fills
    // what is left of the current chunk, the rest goes to ceil(rest /
    // kOutChunk) fresh chunks of the region (kRegions global chunks apart);
    // pair i of the batch lands at at(i).
    struct Span {
        unsigned long long a0, g0;  // a0 + i for i < n0; else chunk-strided from g0
        int n0;
        __device__ __forceinline__ unsigned long long at(unsigned long long i) const
        {
            if (i < (unsigned long long)n0) return a0 + i;
            const unsigned long long j = i - (unsigned long long)n0;
            return g0 + ((j >> kOutChunkLog) << (kOutChunkLog + kRegionsLog)) + (j & (kOutChunk - 1));
        }
    };
    __device__ __forceinline__ Span reserve(const OutStream &o, int total)
    {
        pairs += (unsigned long long)total;
        Span sp;
        sp.a0 = base + (unsigned long long)fill;
        if (fill + total <= kOutChunk) {
            sp.n0 = total;
            sp.g0 = sp.a0;
            fill = uni32(fill + total);
            return sp;
        }
        sp.n0 = have ? kOutChunk - fill : 0;
        fill = kOutChunk;  // the current chunk is now full
        retire(o);
        const int rest = total - sp.n0;
        const int nch = (rest + kOutChunk - 1) / kOutChunk;
        const int reg = (int)(blockIdx.x % kRegions);
        unsigned long long b = 0;
        if ((threadIdx.x & 63) == 0)
            b = atomicAdd(&o.octr[reg * kRegStride], (unsigned long long)nch * (unsigned long long)kOutChunk);
        b = ((unsigned long long)(uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)(b >> 32), 0) << 32) |
            (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)b, 0);
        // else the region is full: counted, not written (rerun)
        have = uni32((int64_t)b + (int64_t)nch * kOutChunk <= o.rcap);
        const unsigned long long lc = b >> kOutChunkLog;  // first local chunk
        if (have)  // the chunks before the last are full
            for (int c = threadIdx.x & 63; c < nch - 1; c += 64)
                o.fills[((lc + (unsigned long long)c) << kRegionsLog) | (unsigned long long)reg] = (uint32_t)kOutChunk;
        sp.g0 = uni64(((lc << kRegionsLog) | (unsigned long long)reg) << kOutChunkLog);
        base = uni64((((lc + (unsigned long long)(nch - 1)) << kRegionsLog) | (unsigned long long)reg) << kOutChunkLog);
        fill = uni32(rest - (nch - 1) * kOutChunk);
        return sp;
    }
    __device__ __forceinline__ void retire(const OutStream &o)
    {
        if (have && (threadIdx.x & 63) == 0) o.fills[base >> kOutChunkLog] = (uint32_t)fill;
        have = 0;
    }
    __device__ __forceinline__ void finish(const OutStream &o, unsigned long long *counter)
    {
        retire(o);
        if ((threadIdx.x & 63) == 0 && pairs) atomicAdd(counter, pairs);
    }
};

__device__ __forceinline__ unsigned long long mix64(unsigned long long x)
{
    x ^= x >> 31;
    x *= 0x7fb5d329728ea185ull;
    x ^= x >> 27;
    x *= 0x81dadef4bc2dd44dull;
    x ^= x >> 33;
    return x;
}

// tagged-stream key of (q, e): the pair over hbm (3..24) bits of a cheap
// two-multiply hash of it (only bucketing: equal pairs, equal buckets)
__device__ __forceinline__ unsigned long long tag_key(uint32_t q, uint32_t e, int eb, int hbm)
{
    const unsigned long long pk = ((unsigned long long)q << eb) | e;
    const uint32_t h = (q * 0x9e3779b1u) ^ (e * 0x85ebca77u);
    return (pk << hbm) | (h >> (32 - hbm));
}

struct JoinArgs {
    IndexView ix;
    QueryView qv;
    Regions ur;                        // units (k_units)
    OutArgs out;
    uint32_t lazy_sig_recs;            // units with more records prefetch the posting signatures
    uint32_t rec_indirect;             // records in query order, found through sval (no k_rec_permute)
};

// One wavefront per unit, lane = posting (the tile stays in registers); the
// cell's relevant query records are staged in LDS 64 at a time and
// broadcast.  Narrow records: only those whose quantised start lies in
// [q(min m - widest window), q(max t1)] (64-ary cooperative search over the
// cell's start-sorted records); wide ones and long tiles: all.  Per record:
// the fused altitude/time/owner predicate is one wave mask; the
// smallest-shared-cell rule (SQL DISTINCT, Q13) compares the record's
// near-prefix signature (broadcast) with each lane's posting signature.
template <bool OWNER, bool LONG, bool DENSE, bool QUADS>
__global__ __launch_bounds__(64 * kWaves) __attribute__((amdgpu_waves_per_eu(LONG ? kJoinLongWpe : DENSE ? kJoinBpcDense : kJoinBpcSparse))) void k_join(JoinArgs a, const QRec *__restrict__ recs,
                                                      const uint64_t *__restrict__ sval,
                                                      const Unit *__restrict__ units,
                                                      unsigned long long *__restrict__ work)
{
    __shared__ longlong2 s_rt[kWaves][64];      // record (tlo, thi)
    __shared__ float4 s_ra[kWaves][64];         // record (alo, ahi, qv, own)
    __shared__ ulonglong2 s_rs[kWaves][2][64];  // record near-prefix signature
    constexpr int kOutStage = LONG ? 1 : DENSE ? kStageDense : kStageSparse;
    __shared__ uint16_t s_os[kWaves][kOutStage];  // a batch's pairs as (record slot << 6 | lane), staged
    __shared__ uint32_t s_pe[kWaves][64];         // each lane's posting entity (for the staged stores)
    const int lane = threadIdx.x & 63;
    const int w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const IndexView &ix = a.ix;
    WaveOut out, tout;  // pairs, tagged keys
    unsigned long long n_tests = 0, n_bcast = 0;
#ifdef DSS_JOIN_PROFILE
    unsigned long long jp[kJProf] = {};
#endif
    // units: kRegions queues (the unit regions), a wave starts on its own
    // region's and moves on when it is drained; grabs of g units per atomic
    int qreg = (int)(blockIdx.x % kRegions), visited = 0;
    int64_t qn = min((int64_t)a.ur.cnt[qreg * kRegStride], a.ur.cap);
    const int64_t wpr = max((int64_t)1, (int64_t)gridDim.x * kWaves / kRegions);  // waves per region
    int64_t ucur = 0, uend = 0;
    auto next_unit = [&]() -> int64_t {
        while (ucur >= uend) {
            const int64_t g = min((int64_t)32, max((int64_t)1, qn / (wpr * 8)));
            unsigned long long ub = 0;
            if (lane == 0) ub = atomicAdd(&work[qreg * kRegStride], (unsigned long long)g);
            // lane 0's grab into scalar registers: the unit loop's exits stay
            // wave-uniform, so its loop-carried state (output chunk, counters)
            // stays scalar too
            ub = ((unsigned long long)(uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)(ub >> 32), 0) << 32) |
                 (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)ub, 0);
            if ((int64_t)ub < qn) {
                ucur = (int64_t)ub;
                uend = min((int64_t)ub + g, qn);
                break;
            }
            if (++visited >= kRegions) return -1;
            qreg = (qreg + 1) % kRegions;
            qn = min((int64_t)a.ur.cnt[qreg * kRegStride], a.ur.cap);
        }
        return (int64_t)qreg * a.ur.cap + ucur++;
    };
    // software pipeline: the next unit's descriptor and postings are loaded
    // while this one's records are joined
    Unit dn{};
    longlong2 nt = make_longlong2(LLONG_MAX, LLONG_MIN);
    float2 na = make_float2(INFINITY, -INFINITY);
    uint32_t ne = 0, nmeta = 0;
    int32_t nown = 0;
    ulonglong2 ns01 = make_ulonglong2(0, 0), ns23 = make_ulonglong2(0, 0);
    bool nsig = false;
    // A unit with few records (the sparse case: a cell scanned for a handful
    // of queries) leaves the posting signatures (32 of the 61 bytes) to be
    // loaded later, only by the lanes that need the smallest-shared-cell test.
    auto prefetch = [&](int64_t u) {
        dn = units[u];
        nt = make_longlong2(LLONG_MAX, LLONG_MIN);
        na = make_float2(INFINITY, -INFINITY);
        ne = nmeta = 0;
        nown = 0;
        ns01 = ns23 = make_ulonglong2(0, 0);
        const uint32_t nrec = (dn.n1 > dn.n0 ? dn.n1 - dn.n0 : 0u) + (dn.w1 > dn.w0 ? dn.w1 - dn.w0 : 0u);
        nsig = nrec > a.lazy_sig_recs;
        if (nrec && (uint32_t)lane < (dn.np & ~kUnitFlags)) {  // a tile no record can meet is skipped unloaded
            const uint64_t p = dn.p0 + lane;
            ne = ix.b_e[p];
            nmeta = ix.b_meta[p];
            nt = ix.b_t[p];
            na = ix.b_alt[p];
            // (round 6: skipping the load for an entity's first quad, whose
            // pairs are all kept, made the load wait on b_e: 2.07 -> 2.10 ms)
            if (nsig) {
                ns01 = ix.b_sig[2 * p];
                ns23 = ix.b_sig[2 * p + 1];
            }
            if (OWNER) nown = ix.b_owner[p];
        }
    };
    int64_t un = next_unit();
    if (un >= 0) prefetch(un);
    while (un >= 0) {
        Unit d = dn;  // (a uniform load; made explicit for the compiler)
        d.np = (uint32_t)uni32((int)d.np);
        d.slot = (uint32_t)uni32((int)d.slot);
        d.n0 = (uint32_t)uni32((int)d.n0);
        d.n1 = (uint32_t)uni32((int)d.n1);
        d.w0 = (uint32_t)uni32((int)d.w0);
        d.w1 = (uint32_t)uni32((int)d.w1);
        const uint32_t np = d.np & ~kUnitFlags;
        // ---- this lane's posting
        const longlong2 pt = nt;
        const float2 pa = na;
        const uint32_t pe = ne, pmeta = nmeta;
        const int32_t pown = nown;
        ulonglong2 ps01 = ns01, ps23 = ns23;
        const bool usig = nsig;  // the signatures are loaded (else: per lane, on first need)
        bool lsig = false;
        const bool pv = (uint32_t)lane < np && !is_dead(ix, pe & ~kFirstBit);  // tombstones match nothing
        un = next_unit();
        if (un >= 0) prefetch(un);
        if (d.n1 <= d.n0 && d.w1 <= d.w0) continue;
        const uint32_t pent = pe & ~kFirstBit;
        s_pe[w][lane] = pent;  // (read after the wave barrier of the emission below)
        const unsigned long long vmask = __ballot(pv);
        if (!vmask) continue;  // (un, the next unit, is already in flight)
        JPROF(13, lane == 0);
        JPROF(19, lane == 0 ? __popcll(vmask) : 0);
        // tile time bounds (a regular tile is sorted by m = min(t0, t1)):
        // records whose window misses every posting are skipped (a long
        // tile: no bound)
        long long t0min = LLONG_MIN, t1max = LLONG_MAX;
        if (!(d.np & kUnitLong)) {
            const long long m = tmin2(pt.x, pt.y);
            t0min = readlane64(m, 0);  // <= every t0 of the tile
            t1max = wave_max_bound((uint32_t)lane < np ? (pt.x > pt.y ? pt.x : pt.y) : LLONG_MIN);
        }
        // a banded tile's altitude hull (its postings' [min alt_lo, max
        // alt_hi]; NaN altitudes meet nothing and are left out): records
        // outside it are not staged
        float hlo = -INFINITY, hhi = INFINITY;
        if (d.np & kUnitBand) {
            hlo = wave_min_f(pv && pa.x == pa.x ? pa.x : INFINITY);
            hhi = wave_max_f(pv && pa.y == pa.y ? pa.y : -INFINITY);
        }
        const uint32_t ra0 = d.n0, ra1 = d.n1, rb0 = d.w0, rb1 = d.w1;
        const bool pfirst = (pe & kFirstBit) != 0;                  // entity's smallest cell
        const bool pcompact = (pmeta & kMetaCompact) != 0;          // compact prefix
        const bool plong = LONG && (pmeta & kMetaLongFp) != 0;      // long footprint
        for (int part = 0; part < 2; part++) {
            const uint32_t x0 = part ? rb0 : ra0, x1 = part ? rb1 : ra1;
            for (uint32_t base = x0; base < x1; base += 64) {
                // stage the batch's records whose window meets the tile's time
                // hull (and a banded tile's altitude hull), compacted to slots
                // [0, nrel).  (Round 6: batches filled to 64 staged records
                // across loaded groups -- 35 % fewer batches on configs[2] --
                // made k_join slower, 2.22 -> 2.31 ms: each batch boundary
                // re-read a group through the dependent sval -> record loads.)
                const uint32_t r = base + (uint32_t)lane;
                bool rel = false;
                int4 h0 = make_int4(0, 0, 0, 0), h1 = h0;
                ulonglong2 g0 = make_ulonglong2(0, 0), g1 = g0;
                if (r < x1) {
                    const int4 *r4 = reinterpret_cast<const int4 *>(recs + (a.rec_indirect ? (uint32_t)sval[r] : r));
                    h0 = r4[0];
                    h1 = r4[1];
                    const long long tlo = ((long long)h0.y << 32) | (uint32_t)h0.x;
                    const long long thi = ((long long)h0.w << 32) | (uint32_t)h0.z;
                    rel = t1max >= tlo && t0min <= thi && __int_as_float(h1.y) >= hlo && __int_as_float(h1.x) <= hhi;
                    if (rel) {
                        g0 = reinterpret_cast<const ulonglong2 *>(r4)[2];
                        g1 = reinterpret_cast<const ulonglong2 *>(r4)[3];
                    }
                }
                const unsigned long long relm = __ballot(rel);
                const int nrel = uni32(__popcll(relm));
                JPROF(12, r < x1);
                if (!nrel) continue;
                JPROF(10, lane == 0);
                JPROF(11, lane == 0 ? nrel : 0);
                const uint32_t slot = mbcnt64(relm);
                __builtin_amdgcn_wave_barrier();
                if (rel) {
                    s_rt[w][slot] = make_longlong2(((long long)h0.y << 32) | (uint32_t)h0.x,
                                                   ((long long)h0.w << 32) | (uint32_t)h0.z);
                    s_ra[w][slot] = make_float4(__int_as_float(h1.x), __int_as_float(h1.y), __int_as_float(h1.z),
                                                __int_as_float(h1.w));
                    s_rs[w][0][slot] = g0;
                    s_rs[w][1][slot] = g1;
                }
                __builtin_amdgcn_wave_barrier();
                // record flags by slot, as wave-uniform masks
                const uint32_t qslot = (lane < nrel) ? (uint32_t)__float_as_int(s_ra[w][lane].z) : 0u;
                const unsigned long long R0 = __ballot((qslot & kRank0) != 0);
                const unsigned long long RC = __ballot((qslot & kCompactQ) != 0);
                const unsigned long long RL = LONG ? __ballot((qslot & kLongQ) != 0) : 0ull;
                // the records whose cells in the quad meet this posting's:
                // one ballot per child, ORed over the posting's children (at
                // the cell grain every mask is 1: all records meet)
                unsigned long long meets = ~0ull;
                if constexpr (QUADS) {  // (a template parameter: a runtime flag here cost the quad join ~3 %)
                    const unsigned long long Q0 = __ballot((qslot >> kQMaskShift) & 1u);
                    const unsigned long long Q1 = __ballot((qslot >> (kQMaskShift + 1)) & 1u);
                    const unsigned long long Q2 = __ballot((qslot >> (kQMaskShift + 2)) & 1u);
                    const unsigned long long Q3 = __ballot((qslot >> (kQMaskShift + 3)) & 1u);
                    meets = ((pmeta & 1u) ? Q0 : 0ull) | ((pmeta & 2u) ? Q1 : 0ull) | ((pmeta & 4u) ? Q2 : 0ull) |
                            ((pmeta & 8u) ? Q3 : 0ull);
                }
                n_bcast += (unsigned long long)nrel;
                n_tests += (unsigned long long)nrel * (unsigned long long)__popcll(vmask);
                // (1) this lane's posting against every staged record: a bit per
                // passing record.  COALESCE'd predicates of operations.go:394-402
                // (NULL -> sentinels).
                uint32_t mlo = 0, mhi = 0;
                const int nlo = nrel < 32 ? nrel : 32;
#pragma unroll 4
                for (int j = 0; j < nlo; j++) {
                    const longlong2 rt = s_rt[w][j];
                    const float4 ra = s_ra[w][j];
                    bool pass = (pt.y >= rt.x) & (pt.x <= rt.y) & (pa.y >= ra.x) & (pa.x <= ra.y);
                    if (OWNER) {
                        const int32_t own = __float_as_int(ra.w);
                        pass &= (own < 0) | (pown == own);
                    }
                    mlo |= (uint32_t)pass << j;
                }
#pragma unroll 4
                for (int j = 32; j < nrel; j++) {
                    const longlong2 rt = s_rt[w][j];
                    const float4 ra = s_ra[w][j];
                    bool pass = (pt.y >= rt.x) & (pt.x <= rt.y) & (pa.y >= ra.x) & (pa.x <= ra.y);
                    if (OWNER) {
                        const int32_t own = __float_as_int(ra.w);
                        pass &= (own < 0) | (pown == own);
                    }
                    mhi |= (uint32_t)pass << (j - 32);
                }
                const unsigned long long m = pv ? (((unsigned long long)mhi << 32) | mlo) & meets : 0ull;
#ifdef DSS_JOIN_PROFILE
                if (pv) {  // the first predicate (in this order) that rejects each test
                    unsigned long long ct = 0, ca = 0, co = 0;
                    for (int j = 0; j < nrel; j++) {
                        const longlong2 rt = s_rt[w][j];
                        const float4 ra = s_ra[w][j];
                        const bool tp = (pt.y >= rt.x) & (pt.x <= rt.y);
                        const bool ap = (pa.y >= ra.x) & (pa.x <= ra.y);
                        const int32_t own = __float_as_int(ra.w);
                        const bool op = !OWNER || (own < 0) | (pown == own);
                        ct += !tp;
                        ca += tp && !ap;
                        co += tp && ap && !op;
                    }
                    const unsigned long long pta = ((unsigned long long)mhi << 32) | mlo;
                    JPROF(0, nrel);
                    JPROF(1, ct);
                    JPROF(2, ca);
                    JPROF(3, co);
                    JPROF(4, __popcll(pta & ~meets));
                    JPROF(5, __popcll(m));
                }
#endif
                // (2) the quad of the smallest shared cell only (SQL DISTINCT,
                // Q13): a rank-0 record (the query's first quad) or a posting in
                // its entity's first quad has no cell below the quad on one
                // side; otherwise the near-prefix signatures of the cells below
                // the quad decide -- overlap: drop; none and either prefix
                // compact: keep (exact); both footprints long: keep, tagged (the
                // tagged set is deduplicated after the join); else exact merge.
                unsigned long long keep = pfirst ? m : (m & R0);
                unsigned long long need = m & ~keep;
#ifdef DSS_JOIN_PROFILE
                unsigned long long unc = 0;
                const unsigned long long need0 = need;
                JPROF(6, __popcll(keep));
                JPROF(7, __popcll(need0));
                {
                    const uint32_t wi = wave_max((uint32_t)__popcll(need0));
                    JPROF(14, lane == 0 ? wi : 0u);
                }
#endif
                if (!usig) {  // lazy signatures: the lanes that need them now
                    const bool want = need != 0ull && !lsig;
                    if (__ballot(want)) {
                        if (want) {
                            const uint64_t p = d.p0 + (uint64_t)lane;
                            ps01 = ix.b_sig[2 * p];
                            ps23 = ix.b_sig[2 * p + 1];
                            lsig = true;
                        }
                    }
                }
                // lane-major (each lane walks its own checks; round 6: record-major
                // -- one broadcast signature per record some lane needs -- made
                // k_join slower on configs[1] / [2] / [3]: 2.03 -> 2.14 ms on [2],
                // profiles/r07h)
                while (need) {
                    const int j = __builtin_ctzll(need);
                    need &= need - 1;
                    const ulonglong2 c0 = s_rs[w][0][j], c1 = s_rs[w][1][j];
                    if (((c0.x & ps01.x) | (c0.y & ps01.y) | (c1.x & ps23.x) | (c1.y & ps23.y)) != 0ull) continue;
                    // (without long postings every posting's prefix is compact:
                    // all of its entity's cells lie in an 8 x 8 window)
                    bool k = !LONG || pcompact || ((RC >> j) & 1ull) || (plong && ((RL >> j) & 1ull));
#ifdef DSS_JOIN_PROFILE
                    if (LONG && !(pcompact || ((RC >> j) & 1ull)) && plong && ((RL >> j) & 1ull)) unc |= 1ull << j;
#endif
                    if (LONG && !k) {  // neither prefix compact, not both long (rare; needs long postings)
                        const uint32_t q = (uint32_t)__float_as_int(s_ra[w][j].z) & ~kQFlags;
                        k = no_smaller_shared<2>(ix, pent, quad_first_cell(ix, d.slot), a.qv.cells + a.qv.offs[q],
                                                 a.qv.offs[q + 1] - a.qv.offs[q]);
                    }
                    if (k) keep |= 1ull << j;
                }
#ifdef DSS_JOIN_PROFILE
                JPROF(8, __popcll(need0 & ~keep));
                JPROF(9, __popcll(keep));
#endif
                // (3) emission, the batch's pairs contiguous per stream (pairs;
                // long x long keys): lane-major (each lane's pairs after the
                // lanes before it; iterations = the largest lane count) at low
                // pass density, else record-major (one coalesced row per record:
                // dense batches would scatter too many lane stores).  Both
                // streams' counts ride one scan (16-bit halves: <= 64 x 64).
                // long x long pairs are tagged (deduplicated after the join).
                // (Round 6: sending those kept in a first quad -- exactly their
                // smallest shared quad -- out untagged cut configs[4]'s tagged
                // occurrences 203M -> 173M at scale 0.2, but telling a tagged
                // pair whose smallest shared quad is a first quad needs list
                // searches per distinct pair: join phase 13.8 -> 69 ms.)
                const unsigned long long tagm = (LONG && plong) ? (keep & RL) : 0ull;
#ifdef DSS_JOIN_PROFILE
                JPROF(20, __popcll(tagm & ~need0));       // long x long kept in a first quad (exact)
                JPROF(21, __popcll(tagm & unc));          // long x long kept uncertain (neither prefix compact)
#endif
                const uint32_t cu = (uint32_t)__popcll(keep & ~tagm), ct = (uint32_t)__popcll(tagm);
                const uint32_t incl = wave_incl_scan(cu | (ct << 16));
                const uint32_t tot = (uint32_t)uni32(__builtin_amdgcn_readlane((int)incl, 63));
                const int total_u = (int)(tot & 0xffffu), total_t = LONG ? (int)(tot >> 16) : 0;
                JPROF(18, lane == 0 && !(total_u | total_t));
                if (!(total_u | total_t)) continue;
                WaveOut::Span su{}, st{};
                if (total_u) su = out.reserve(a.out.ps, total_u);
                if (LONG && total_t) st = tout.reserve(a.out.ts, total_t);
                const bool wu = out.have != 0, wt = LONG && tout.have != 0;  // else counted only (rerun)
                if ((int64_t)(total_u + total_t) * kEmitDensity <= (int64_t)nrel * __popcll(vmask)) {
#ifdef DSS_JOIN_PROFILE
                    {
                        const uint32_t wi = wave_max((uint32_t)__popcll(keep));
                        JPROF(15, lane == 0);
                        JPROF(17, lane == 0 ? wi : 0u);
                    }
#endif
                    // (one loop per stream: no divergent double bodies)
                    if (!LONG && wu && total_u <= kOutStage) {  // (long variants: direct, no VGPR headroom)
                        // each lane's pairs into the wave's LDS stage as 16-bit
                        // (record slot, lane) codes, then the batch leaves as
                        // runs of consecutive slots: full-width coalesced global
                        // stores instead of one scattered 4-B store per pair and
                        // array (configs[2] k_join 3.89 -> 3.70 ms against an
                        // 8-B (q, e) stage of a quarter the pairs)
                        uint32_t iu = (incl & 0xffffu) - cu;
                        unsigned long long kk = keep & ~tagm;
                        while (kk) {
                            const int j = __builtin_ctzll(kk);
                            kk &= kk - 1;
                            s_os[w][iu++] = (uint16_t)((uint32_t)j << 6 | (uint32_t)lane);
                        }
                        __builtin_amdgcn_wave_barrier();
                        // (the batch usually fits what is left of the wave's
                        // chunk: one contiguous run, no chunk-strided mapping)
                        if (su.n0 >= total_u) {
                            const unsigned long long a0 = uni64(su.a0);
                            for (int p = lane; p < total_u; p += 64) {
                                const uint32_t v = s_os[w][p];
                                a.out.q[a0 + p] = (uint32_t)__float_as_int(s_ra[w][v >> 6].z) & ~kQFlags;
                                a.out.e[a0 + p] = s_pe[w][v & 63u];
                            }
                        } else {
                            for (int p = lane; p < total_u; p += 64) {
                                const uint32_t v = s_os[w][p];
                                const uint32_t q = (uint32_t)__float_as_int(s_ra[w][v >> 6].z) & ~kQFlags;
                                const uint32_t e = s_pe[w][v & 63u];
                                const unsigned long long pos = su.at((unsigned long long)p);
                                a.out.q[pos] = q;
                                a.out.e[pos] = e;
                            }
                        }
                        __builtin_amdgcn_wave_barrier();
                    } else if (wu) {
                        unsigned long long iu = (incl & 0xffffu) - cu, kk = keep & ~tagm;
                        while (kk) {
                            const int j = __builtin_ctzll(kk);
                            kk &= kk - 1;
                            const uint32_t q = (uint32_t)__float_as_int(s_ra[w][j].z) & ~kQFlags;
                            const unsigned long long pos = su.at(iu++);
                            a.out.q[pos] = q;
                            a.out.e[pos] = pent;
                        }
                    }
                    if (LONG && wt) {
                        unsigned long long it = (incl >> 16) - ct, kk = tagm;
                        while (kk) {
                            const int j = __builtin_ctzll(kk);
                            kk &= kk - 1;
                            const uint32_t q = (uint32_t)__float_as_int(s_ra[w][j].z) & ~kQFlags;
                            a.out.tk[st.at(it++)] = tag_key(q, pent, a.out.eb, a.out.hbm);
                        }
                    }
                } else {
                    JPROF(16, lane == 0);
                    unsigned long long ou = 0, ot = 0;
                    for (int j = 0; j < nrel; j++) {
                        const unsigned long long kj = __ballot((keep >> j) & 1ull);
                        if (!kj) continue;
                        // (the lanes that tag record j: tagm, as the counts above)
                        const unsigned long long kt = LONG ? __ballot((tagm >> j) & 1ull) : 0ull, ku = kj & ~kt;
                        const uint32_t q =
                            (uint32_t)__builtin_amdgcn_readfirstlane(__float_as_int(s_ra[w][j].z)) & ~kQFlags;
                        if ((ku >> lane) & 1ull) {
                            const unsigned long long pos = su.at(ou + mbcnt64(ku));
                            if (wu) {
                                a.out.q[pos] = q;
                                a.out.e[pos] = pent;
                            }
                        }
                        if (LONG && ((kt >> lane) & 1ull)) {
                            const unsigned long long pos = st.at(ot + mbcnt64(kt));
                            if (wt) a.out.tk[pos] = tag_key(q, pent, a.out.eb, a.out.hbm);
                        }
                        ou += (unsigned long long)__popcll(ku);
                        ot += (unsigned long long)__popcll(kt);
                    }
                }
            }
        }
    }
    out.finish(a.out.ps, &a.out.counter[0]);
    if (LONG) tout.finish(a.out.ts, &a.out.counter[1]);
    if (lane == 0) {
        atomicAdd(&a.out.counter[2], n_tests);
        atomicAdd(&a.out.counter[3], n_bcast);
    }
#ifdef DSS_JOIN_PROFILE
    for (int i = 0; i < kJProf; i++)
        if (jp[i]) atomicAdd(&g_jprof[i], jp[i]);
#endif
}

// Closing the output holes: chunk c holds fills[c] pairs at c * kOutChunk
// (0 = never reserved); with n pairs in all, the holes below n are filled
// with the pairs at or above n, in order.  k_fix_counts: per chunk its holes
// below n and its pairs at or above n, and the list of chunks below n with
// holes (one ballot-aggregated atomic per wave; the order of the list is
// free: each chunk's sources follow from hoff alone).  k_fix_fill: a block
// per listed chunk, the sources found in an LDS window of the tail offsets.
__global__ void k_fix_counts(int64_t nch, const uint32_t *fills, int64_t n, int64_t *hole, int64_t *tail,
                             uint32_t *list, unsigned int *nlist)
{
    const int64_t c = tid64();
    bool listed = false;
    if (c < nch) {
        const int64_t s = c * kOutChunk, f = fills[c];
        const int64_t h0 = s + f, h1 = min(s + (int64_t)kOutChunk, n);  // holes below n
        const int64_t t0 = max(s, n), t1 = s + f;                        // pairs at or above n
        hole[c] = h1 > h0 ? h1 - h0 : 0;
        tail[c] = t1 > t0 ? t1 - t0 : 0;
        listed = h1 > h0;
    }
    const unsigned long long m = __ballot(listed);
    if (!m) return;
    const int lane = threadIdx.x & 63, leader = __builtin_ctzll(m);
    unsigned int b = 0;
    if (lane == leader) b = atomicAdd(nlist, (unsigned int)__popcll(m));
    b = (unsigned int)__shfl((int)b, leader);
    if (listed) list[b + mbcnt64(m)] = (uint32_t)c;
}
struct MovePairs {
    uint32_t *q, *e;
    __device__ void operator()(int64_t dst, int64_t src) const
    {
        q[dst] = q[src];
        e[dst] = e[src];
    }
};
struct MoveKeys {
    unsigned long long *k;
    __device__ void operator()(int64_t dst, int64_t src) const { k[dst] = k[src]; }
};
constexpr int kFixBlock = 256;
template <typename Move>
__global__ __launch_bounds__(kFixBlock) void k_fix_fill(int64_t nch, const uint32_t *list, const unsigned int *nlist,
                                                        const uint32_t *fills, int64_t n, const int64_t *hole,
                                                        const int64_t *hoff, const int64_t *toff, Move mv)
{
    __shared__ int64_t s_lo;
    __shared__ int64_t s_toff[kFixBlock + 1];  // toff[lo0 .. lo0 + kFixBlock]
    const int64_t nl = *nlist;
    for (int64_t i = blockIdx.x; i < nl; i += gridDim.x) {
        const int64_t c = list[i], h = hole[c], t0 = hoff[c];
        __syncthreads();
        if (threadIdx.x == 0) {  // tail chunk lo0 of the first source: toff[lo0] <= t0 < toff[lo0 + 1]
            int64_t lo = n / kOutChunk, hi = nch;
            while (hi - lo > 1) {
                const int64_t mid = (lo + hi) >> 1;
                if (toff[mid] <= t0) lo = mid;
                else hi = mid;
            }
            s_lo = lo;
        }
        __syncthreads();
        const int64_t lo0 = s_lo;
        for (int j = threadIdx.x; j <= kFixBlock; j += kFixBlock)
            s_toff[j] = lo0 + j < nch ? toff[lo0 + j] : INT64_MAX;
        __syncthreads();
        for (int64_t k = threadIdx.x; k < h; k += kFixBlock) {
            const int64_t t = t0 + k;  // its source: the t-th pair at or above n
            int64_t lo;
            if (t < s_toff[kFixBlock]) {  // inside the window (the usual case)
                int a = 0, b = kFixBlock;  // s_toff[a] <= t < s_toff[b]
                while (b - a > 1) {
                    const int mid = (a + b) >> 1;
                    if (s_toff[mid] <= t) a = mid;
                    else b = mid;
                }
                lo = lo0 + a;
            } else {  // past it: galloping in global memory
                int64_t step = 1;
                lo = lo0 + kFixBlock;
                while (lo + step < nch && toff[lo + step] <= t) {
                    lo += step;
                    step <<= 1;
                }
                int64_t hi = lo + step < nch ? lo + step : nch;
                while (hi - lo > 1) {
                    const int64_t mid = (lo + hi) >> 1;
                    if (toff[mid] <= t) lo = mid;
                    else hi = mid;
                }
            }
            const int64_t src = max(lo * kOutChunk, n) + (t - toff[lo]);
            mv(c * kOutChunk + fills[c] + k, src);
        }
    }
}

// Tagged (long x long) pairs after the join, which writes them as 64-bit keys
// ((q << eb | e) << hbm | hbm hash bits of the pair) to their own stream; a
// radix sort over hb <= hbm low hash bits only (ceil(hb / 8) passes instead
// of a full 40+-bit sort) groups equal pairs in one bucket of ~1024 keys
// (tunable), and
// one block per bucket removes the duplicates in an LDS hash set.  A bucket
// too large for the LDS set (never at the average) falls back to a full sort
// of its keys.
constexpr int kDedupBlock = 256, kDedupSlots = 4096;  // 32 KB of LDS: several blocks per CU
constexpr int64_t kDedupMax = kDedupSlots * 3 / 4;

struct PredRunU64 {
    const unsigned long long *k;
    __device__ bool operator()(int64_t i) const { return i == 0 || k[i] != k[i - 1]; }
};
struct EmitPairFromKey {  // key >> sh = q << eb | e
    const unsigned long long *k;
    uint32_t *q, *e;
    int64_t at;
    int eb, sh;
    __device__ void operator()(int64_t i, int64_t r) const
    {
        const unsigned long long pk = k[i] >> sh;
        q[at + r] = (uint32_t)(pk >> eb);
        e[at + r] = (uint32_t)(pk & ((1ull << eb) - 1));
    }
};

// bucket b's keys are [bs[b], be[b]) of the bucket-sorted keys (0, 0 if none)
__global__ void k_tag_bounds(int64_t n, const unsigned long long *__restrict__ k, int hb, int64_t *__restrict__ bs,
                             int64_t *__restrict__ be)
{
    const int64_t i = tid64();
    if (i >= n) return;
    const unsigned long long m = (1ull << hb) - 1, b = k[i] & m;
    if (i == 0 || (k[i - 1] & m) != b) bs[b] = i;
    if (i == n - 1 || (k[i + 1] & m) != b) be[b] = i + 1;
}

// One block per bucket: its distinct pairs (keys >> hbm) into stage[bs[b] ..),
// their count into cnt[b]; a bucket over kDedupMax keys is flagged instead.
__global__ __launch_bounds__(kDedupBlock) void k_tag_dedupe(const unsigned long long *__restrict__ k,
                                                             const int64_t *__restrict__ bs,
                                                             const int64_t *__restrict__ be, int hbm,
                                                             unsigned long long *__restrict__ stage,
                                                             int64_t *__restrict__ cnt, uint8_t *__restrict__ ovf,
                                                             unsigned long long *__restrict__ novf)
{
    __shared__ unsigned long long tab[kDedupSlots];
    __shared__ uint32_t nout;
    const int64_t b = blockIdx.x, lo = bs[b], hi = be[b];
    const int tid = threadIdx.x, lane = tid & 63;
    if (hi - lo > kDedupMax) {  // block-uniform
        if (tid == 0) {
            cnt[b] = 0;
            ovf[b] = 1;
            atomicAdd(novf, 1ull);
        }
        return;
    }
    if (tid == 0) ovf[b] = 0;
    if (hi == lo) {
        if (tid == 0) cnt[b] = 0;
        return;
    }
    // table: the smallest power of two >= 2x the bucket's keys (load <= 1/2)
    uint32_t slots = 256;
    while ((int64_t)slots < 2 * (hi - lo) && slots < (uint32_t)kDedupSlots) slots <<= 1;
    const uint32_t smask = slots - 1;
    constexpr unsigned long long kEmpty = ~0ull;
    for (uint32_t i = tid; i < slots; i += kDedupBlock) tab[i] = kEmpty;
    if (tid == 0) nout = 0;
    __syncthreads();
    for (int64_t i = lo + tid; i < hi; i += kDedupBlock) {
        const unsigned long long pk = k[i] >> hbm;
        uint32_t h = (uint32_t)mix64(pk ^ 0x9e3779b97f4a7c15ull) & smask;
        while (true) {  // fewer distinct keys than slots: a free slot always exists
            const unsigned long long prev = atomicCAS(&tab[h], kEmpty, pk);
            if (prev == kEmpty || prev == pk) break;
            h = (h + 1) & smask;
        }
    }
    __syncthreads();
    for (uint32_t i0 = 0; i0 < slots; i0 += kDedupBlock) {
        const unsigned long long v = i0 + tid < slots ? tab[i0 + tid] : kEmpty;
        const bool has = v != kEmpty;
        const unsigned long long m = __ballot(has);
        uint32_t base = 0;
        if (lane == 0 && m) base = atomicAdd(&nout, (uint32_t)__popcll(m));
        base = __shfl(base, 0);
        if (has) stage[lo + base + mbcnt64(m)] = v;
    }
    __syncthreads();
    if (tid == 0) cnt[b] = nout;
}

// bucket b's distinct pairs -> (q, e) at off[b]
__global__ void k_tag_emit(const unsigned long long *__restrict__ stage, const int64_t *__restrict__ bs,
                           const int64_t *__restrict__ cnt, const int64_t *__restrict__ off, int eb,
                           uint32_t *__restrict__ q, uint32_t *__restrict__ e)
{
    const int64_t b = blockIdx.x, c = cnt[b], lo = bs[b], o = off[b];
    const unsigned long long em = (1ull << eb) - 1;
    for (int64_t j = threadIdx.x; j < c; j += blockDim.x) {
        const unsigned long long pk = stage[lo + j];
        q[o + j] = (uint32_t)(pk >> eb);
        e[o + j] = (uint32_t)(pk & em);
    }
}

// Cell-range shards (dssg_index_build_range): a long x long pair can meet
// on several shards, and each keeps its own copy after the dedupe.  Only the
// shard owning the pair's smallest shared cell keeps it: a shard starting at
// cell_lo > 0 drops the pairs that also share a cell below cell_lo (a
// two-pointer walk over the two sorted lists' cells below cell_lo; both lists
// are whole on every shard).
// On a cell-range shard past the first: the distinct tagged (long x long)
// pairs sharing a cell below the shard's range are another shard's (exactly
// once across shards).
__global__ void k_tag_shard_keep(int64_t n, const uint32_t *__restrict__ q, const uint32_t *__restrict__ e,
                                 QueryView qv, IndexView ix, uint64_t cell_lo, uint8_t *__restrict__ keep)
{
    const int64_t i = tid64();
    if (i >= n) return;
    const uint32_t qq = q[i], ee = e[i];
    const uint64_t *a = qv.cells + qv.offs[qq], *b = ix.e_cells + ix.e_offs[ee];
    const int64_t na = qv.offs[qq + 1] - qv.offs[qq], nb = ix.e_offs[ee + 1] - ix.e_offs[ee];
    int64_t x = 0, y = 0;
    bool shared = false;
    while (x < na && y < nb) {
        const uint64_t ca = a[x], cb = b[y];
        if (ca >= cell_lo || cb >= cell_lo) break;
        if (ca == cb) {
            shared = true;
            break;
        }
        if (ca < cb) x++;
        else y++;
    }
    keep[i] = shared ? 0 : 1;
}
struct PredFlag8 {
    const uint8_t *f;
    __device__ bool operator()(int64_t i) const { return f[i] != 0; }
};
struct EmitPairCopy {
    const uint32_t *q, *e;
    uint32_t *q2, *e2;
    __device__ void operator()(int64_t i, int64_t r) const
    {
        q2[r] = q[i];
        e2[r] = e[i];
    }
};

struct PredOvf {  // keys of the flagged buckets
    const unsigned long long *k;
    const uint8_t *ovf;
    int hb;
    __device__ bool operator()(int64_t i) const { return ovf[k[i] & ((1ull << hb) - 1)] != 0; }
};
struct EmitShift {
    const unsigned long long *k;
    unsigned long long *out;
    int sh;
    __device__ void operator()(int64_t i, int64_t r) const { out[r] = k[i] >> sh; }
};

// Roofline accounting, predicate off: M = postings scanned query-cell by
// query-cell, D = pairs surviving the smallest-shared-cell rule (= distinct
// candidate entities per query, summed).
__global__ __launch_bounds__(kBlock) void k_stats(IndexView a, QueryView qv, unsigned long long *stat)
{
    const int lane = threadIdx.x & 63;
    const int64_t q = (int64_t)blockIdx.x * (kBlock / 64) + (threadIdx.x >> 6);
    unsigned long long my_m = 0, my_d = 0;
    if (q < qv.nq) {
        const int64_t c0 = qv.offs[q], c1 = qv.offs[q + 1];
        for (int64_t ci = c0; ci < c1; ci++) {
            const uint64_t c = qv.cells[ci];
            const uint32_t bit = child_bit(c, a.gshift);
            // the quad's first cell in the query also counts its pairs (the
            // query's cells in the quad: qmask)
            const bool head = ci == c0 || !same_quad(qv.cells[ci - 1], c, a.gshift);
            uint32_t qmask = bit;
            for (int64_t x = ci + 1; head && x < c1 && x < ci + 4 && same_quad(c, qv.cells[x], a.gshift); x++)
                qmask |= child_bit(qv.cells[x], a.gshift);
            uint32_t slot = 0;
            uint64_t s = 0, e = 0;
            if (find_slot(a, c, slot)) slot_range(a, slot, s, e);
            const uint64_t cq0 = s < e ? quad_first_cell(a, slot) : c;
            for (uint64_t base = s; base < e; base += 64) {
                const uint64_t p = base + lane;
                bool inc = false, pass = false;
                if (p < e) {
                    const uint32_t pm = a.b_meta[p];
                    inc = (pm & bit) != 0;  // a posting of this very cell (cell-level M)
                    if (head && (pm & qmask)) {
                        const uint32_t pe = a.b_e[p];
                        pass = ci == c0 || (pe & kFirstBit) ||
                               no_smaller_shared<8>(a, pe & ~kFirstBit, cq0, qv.cells + c0, ci - c0);
                    }
                }
                my_m += (unsigned long long)__popcll(__ballot(inc));
                my_d += (unsigned long long)__popcll(__ballot(pass));
            }
        }
    }
    if (lane == 0 && (my_m || my_d)) {
        atomicAdd(&stat[0], my_m);
        atomicAdd(&stat[1], my_d);
    }
}

// Small batches (the per-RPC path, pkg/scd/operations_handler.go:118-168:
// one covering and one search per request): kSmallSplit waves per query cell
// that opens a quad of the query, lanes over the quad's postings in the band
// [tlo - dcap, thi] (found by 64-ary wave searches) plus its long postings,
// the waves of one cell interleaved 64 postings apart; the cell-mask and fused
// altitude/time/owner filter, and the smallest-shared-cell rule (SQL
// DISTINCT, Q13) decided exactly by a merge of the two sorted cell lists
// below the quad -- no query ordering, units or dedupe pass: one launch, its
// pairs through one wave-aggregated atomic per 64 postings.  (Round 6: one
// wave per cell walked a hot quad's ~1.5k-posting band in ~24 dependent
// steps after two 14-step binary searches -- 0.10 -> 0.14 ms per batch of
// ~18 requests once quads doubled the postings per group, profiles/r06e.)
constexpr int kSmallBlock = 256;
constexpr int kSmallSplit = 4;  // waves per query cell

// First p in [lo, hi) with m(p) >= x (hi if none), the wave probing 64
// evenly spaced positions per round: ceil(log64) rounds of one load each
// instead of log2 dependent loads.  Wave-uniform.
__device__ __forceinline__ uint64_t wave_lb_m(const longlong2 *bt, uint64_t lo, uint64_t hi, long long x)
{
    const int lane = threadIdx.x & 63;
    while (hi - lo > 64) {
        const uint64_t step = (hi - lo + 63) / 64;
        const uint64_t p = lo + (uint64_t)lane * step;
        bool below = false;
        if (p < hi) {
            const longlong2 t = bt[p];
            below = tmin2(t.x, t.y) < x;
        }
        const int c = __popcll(__ballot(below));  // probes 0..c-1 lie below x (m is sorted)
        if (c == 0) return lo;
        const uint64_t nlo = lo + (uint64_t)(c - 1) * step + 1, nhi = lo + (uint64_t)c * step;
        lo = nlo;
        hi = nhi < hi ? nhi : hi;
    }
    const uint64_t p = lo + (uint64_t)lane;
    bool below = false;
    if (p < hi) {
        const longlong2 t = bt[p];
        below = tmin2(t.x, t.y) < x;
    }
    return lo + (uint64_t)__popcll(__ballot(below));
}

__global__ __launch_bounds__(kSmallBlock) void k_small_join(IndexView ix, QueryView qv, int64_t nqc, int64_t cap,
                                                             uint32_t *__restrict__ oq, uint32_t *__restrict__ oe,
                                                             unsigned long long *__restrict__ count)
{
    const int lane = threadIdx.x & 63;
    const int64_t wv = (int64_t)blockIdx.x * (kSmallBlock / 64) + (threadIdx.x >> 6);
    const int64_t k = wv / kSmallSplit;
    const uint64_t part = (uint64_t)(wv % kSmallSplit);
    if (k >= nqc) return;  // wave-uniform
    int64_t lo = 0, hi = qv.nq;  // the cell's query: offs[lo] <= k < offs[hi]
    while (hi - lo > 1) {
        const int64_t mid = (lo + hi) >> 1;
        if (qv.offs[mid] <= k) lo = mid;
        else hi = mid;
    }
    const uint32_t q = (uint32_t)lo;
    const int64_t c0 = qv.offs[q], c1 = qv.offs[q + 1];
    const uint64_t c = qv.cells[k];
    if (k > c0 && same_quad(qv.cells[k - 1], c, ix.gshift)) return;  // the quad's first cell in the query carries it
    uint32_t qmask = child_bit(c, ix.gshift);
    for (int64_t x = k + 1; x < c1 && x < k + 4; x++) {
        const uint64_t cx = qv.cells[x];
        if (!same_quad(c, cx, ix.gshift)) break;
        qmask |= child_bit(cx, ix.gshift);
    }
    uint32_t slot;
    if (!find_slot(ix, c, slot)) return;
    const uint64_t cq0 = quad_first_cell(ix, slot);
    const uint64_t s0 = ix.s_post[slot], s1 = ix.s_post[slot + 1], sr = s0 + ix.s_nreg[slot];
    const long long tlo = qv.tlo[q], thi = qv.thi[q];
    const float alo = qv.alo[q], ahi = qv.ahi[q];
    const int32_t own = qv.owner ? qv.owner[q] : -1;
    // a regular posting (|t1 - t0| <= dcap) meets [tlo, thi] only if its start m is in [tlo - dcap, thi]:
    // one range of each m-ordered run (the regular part, or each altitude band of it), then the long postings
    const long long mlo = tlo < LLONG_MIN + ix.dcap ? LLONG_MIN : tlo - ix.dcap;
    uint32_t rel[9];
    int nrun = 1;
    rel[0] = 0;
    rel[1] = (uint32_t)(sr - s0);
    if (ix.s_band) {
        band_starts(ix, slot, (uint32_t)(sr - s0), rel);
        nrun = 8;
    }
    for (int run = 0; run <= nrun; run++) {
        uint64_t r0 = sr, r1 = s1;  // (run == nrun: the long postings)
        if (run < nrun) {
            const uint64_t a0 = s0 + rel[run], a1 = s0 + rel[run + 1];
            if (a1 <= a0) continue;
            r0 = wave_lb_m(ix.b_t, a0, a1, mlo);
            // (ub: the first m > thi = the first m >= thi + 1; thi = LLONG_MAX: the run's end)
            r1 = thi == LLONG_MAX ? a1 : wave_lb_m(ix.b_t, r0, a1, thi + 1);
        }
        const uint64_t ntot = r1 - r0;
        for (uint64_t b = part * 64; b < ntot; b += kSmallSplit * 64) {
            const uint64_t t = b + (uint64_t)lane;
            bool keep = false;
            uint32_t ent = 0;
            if (t < ntot) {
                const uint64_t p = r0 + t;
                const longlong2 pt = ix.b_t[p];
                const float2 pa = ix.b_alt[p];
                const uint32_t pe = ix.b_e[p];
                ent = pe & ~kFirstBit;
                // COALESCE'd predicates of operations.go:394-402 (NULL -> sentinels)
                bool pass = (pt.y >= tlo) & (pt.x <= thi) & (pa.y >= alo) & (pa.x <= ahi) &
                            ((ix.b_meta[p] & qmask) != 0);
                if (own >= 0) pass &= ix.b_owner[p] == own;
                if (pass && !is_dead(ix, ent))
                    keep = k == c0 || (pe & kFirstBit) || no_smaller_shared<2>(ix, ent, cq0, qv.cells + c0, k - c0);
            }
            const unsigned long long m = __ballot(keep);
            if (!m) continue;
            unsigned long long base = 0;
            if (lane == 0) base = atomicAdd(count, (unsigned long long)__popcll(m));
            base = uni64_lane0(base);
            if (keep) {
                const unsigned long long pos = base + mbcnt64(m);
                if ((int64_t)pos < cap) {  // else counted only: the host regrows and reruns
                    oq[pos] = q;
                    oe[pos] = ent;
                }
            }
        }
    }
}

// Cell-level postings of the distinct cells a batch touches (each (cell,
// entity) once, as a per-cell index would hold them): the touched cells'
// child bits per quad, then per posting of a touched quad the touched cells
// among its own.
__global__ void k_touch_mark(IndexView a, int64_t nqc, const uint64_t *cells, uint32_t *mark)
{
    const int64_t k = tid64();
    if (k >= nqc) return;
    uint32_t s;
    if (find_slot(a, cells[k], s)) atomicOr(&mark[s], child_bit(cells[k], a.gshift));
}
__global__ void k_touch_sum(IndexView a, int64_t ns, const uint32_t *mark, unsigned long long *sum)
{
    const int64_t s = tid64();
    unsigned long long c = 0;
    if (s < ns && mark[s])
        for (uint64_t p = a.s_post[s]; p < a.s_post[s + 1]; p++) c += (unsigned long long)__popc(a.b_meta[p] & mark[s]);
    for (int o = 32; o > 0; o >>= 1) c += __shfl_xor(c, o);
    if ((threadIdx.x & 63) == 0 && c) atomicAdd(sum, c);
}

int bits_for(int64_t n)
{
    int b = 1;
    while (b < 63 && ((int64_t)1 << b) <= n) b++;
    return b;
}

template <typename T>
T fetch(const T *p, hipStream_t s)
{
    T v{};
    DSS_HIP(hipMemcpyAsync(&v, p, sizeof(T), hipMemcpyDeviceToHost, s));
    DSS_HIP(hipStreamSynchronize(s));
    return v;
}

}  // namespace

// the join's timing events, created on first use by either join path
void SearchEngine::timing_events()
{
    if (timing_ && !ev0_) {
        DSS_HIP(hipEventCreate(&ev0_));
        DSS_HIP(hipEventCreate(&ev1_));
    }
}

// ============================================================ small batches
void SearchEngine::search_small(const dssg_index *idx, int64_t nq, const int64_t *q_offs, const uint64_t *q_cells,
                                const float *q_alt_lo, const float *q_alt_hi, const int64_t *q_tlo,
                                const int64_t *q_thi, const int32_t *q_owner, int64_t nqc, hipStream_t s,
                                dssg_pairs *out)
{
    timing_events();  // (the batcher calls this directly, not through search())
    const IndexView ix = view_of(idx);
    const QueryView qv{nq, q_offs, q_cells, q_alt_lo, q_alt_hi, q_tlo, q_thi, q_owner};
    unsigned long long *count = small_cnt_.ensure(1);
    if (small_cap_ == 0) small_cap_ = std::max<int64_t>(1 << 16, 64 * qv.nq);
    for (int attempt = 0; attempt < 4; attempt++) {
        uint32_t *oq = oq_.ensure(small_cap_ + 1), *oe = oe_.ensure(small_cap_ + 1);
        DSS_HIP(hipMemsetAsync(count, 0, sizeof(unsigned long long), s));
        if (timing_) DSS_HIP(hipEventRecord(ev0_, s));
        hipLaunchKernelGGL(k_small_join, dim3(grid_for(nqc * kSmallSplit, kSmallBlock / 64)), dim3(kSmallBlock), 0, s,
                           ix, qv, nqc,
                           small_cap_, oq, oe, count);
        if (timing_) DSS_HIP(hipEventRecord(ev1_, s));
        const int64_t n = (int64_t)fetch(count, s);
        if (n > small_cap_) {  // counted, not all written: regrow and rerun
            small_cap_ = n + n / 4 + 1024;
            continue;
        }
        if (timing_) {
            float ms = 0;
            DSS_HIP(hipEventElapsedTime(&ms, ev0_, ev1_));
            join_ms_ = ms;
        }
        out->q = oq;
        out->e = oe;
        out->n = n;
        out->n_tagged = 0;
        units_ = keys_ = runs_ = iters_ = tests_ = tagged_ = long_queries_ = 0;
        long_postings_ = idx->n_long_fp;
        return;
    }
    throw Error(DSSG_ERR_DEVICE, "search: output size did not converge");
}

// ================================================================== build
void SearchEngine::build(dssg_index *idx, int64_t n, const int64_t *cell_offs, const uint64_t *cells,
                         const float *alt_lo, const float *alt_hi, const int64_t *t0, const int64_t *t1,
                         const int32_t *owner, uint64_t cell_lo, uint64_t cell_hi, hipStream_t s)
{
    // a cell-range shard holds whole quads: ranges cut at quad boundaries
    constexpr uint64_t kQuadSpan = (1ull << kQuadShift) - 1;  // the low bits of every id under one quad
    if ((cell_lo != 0 && (cell_lo & kQuadSpan) != 0) || (cell_hi != ~0ull && (cell_hi & kQuadSpan) != kQuadSpan))
        throw Error(DSSG_ERR_INVALID, "index: a cell range must start and end at quad (level-12 cell) boundaries");
    idx->cell_lo = cell_lo;
    idx->cell_hi = cell_hi;
    idx->n_e = n;
    idx->has_owner = owner != nullptr;
    if (n >= (int64_t)0x7fffffff) throw Error(DSSG_ERR_INVALID, "index: more than 2^31 - 1 entities");
    const int64_t P = n > 0 ? fetch(cell_offs + n, s) : 0;
    if (P >= (int64_t)0xffffffffll) throw Error(DSSG_ERR_INVALID, "index: more than 2^32 - 1 cells in one build");
    DevBuf<unsigned long long> stat_b;
    unsigned long long *stat = stat_b.ensure(80);  // [0..64] hist, 65..66 m range, 67 dcap, 68..69 dense range,
                                                   // 70 n_irr, 71 nlongfp, 72..73 runs/long, 74 max cell,
                                                   // 75..76 grain counts, 77 largest multiplicity > 255
    DSS_HIP(hipMemsetAsync(stat, 0, 80 * sizeof(unsigned long long), s));
    {
        const unsigned long long init[2] = {~0ull, 0ull};
        DSS_HIP(hipMemcpyAsync(stat + 65, init, sizeof(init), hipMemcpyHostToDevice, s));
        DSS_HIP(hipMemcpyAsync(stat + 68, init, sizeof(init), hipMemcpyHostToDevice, s));
    }
    // (1) entity -> sorted unique cells; the position -> entity map
    DevBuf<uint32_t> pent_b;
    DevBuf<uint32_t> mult_b;
    int64_t Pu = P;
    uint32_t *pent = pent_b.ensure(P + 1);
    if (n) hipLaunchKernelGGL(k_expand, dim3(grid_for(n, kBlock)), dim3(kBlock), 0, s, n, cell_offs, pent);
    unsigned int *bad = (unsigned int *)(stat + 79);
    if (P) hipLaunchKernelGGL(k_check_sorted, dim3(grid_for(P, kBlock)), dim3(kBlock), 0, s, P, pent, cells, bad);
    stage_check(s, "index build: expand");
    const bool general = P > 0 && fetch(bad, s) != 0;
    int64_t *e_offs = idx->e_offs.ensure_exact(n + 1);
    uint64_t *e_cells = idx->e_cells.ensure_exact(P + 1);
    const uint32_t *mult = nullptr;
    if (!general) {
        device_copy(e_offs, cell_offs, sizeof(int64_t) * (n + 1), s);
        device_copy(e_cells, cells, sizeof(uint64_t) * P, s);
    } else {  // sort by cell, then stably by entity; unique (entity, cell) runs with multiplicity
        DevBuf<uint64_t> ka, kb;
        DevBuf<uint32_t> va, vb;
        uint64_t *k0 = ka.ensure(P + 1), *k1 = kb.ensure(P + 1);
        uint32_t *v0 = va.ensure(P + 1), *v1 = vb.ensure(P + 1);
        radix_sort_pairs_packed(cells, (uint64_t *)k1, (const uint32_t *)pent, v1, P, 64, tmp_, s);
        radix_sort_pairs(v1, v0, k1, k0, P, bits_for(n), tmp_, s);  // (entity, cell)
        uint32_t *m = mult_b.ensure(P + 1);
        int64_t *dtot = (int64_t *)(stat + 78);
        compact_if(P, PredUniquePair{v0, k0}, EmitUniquePair{P, v0, k0, e_cells, pent, m, stat + 77}, tmp_, tmp2_, s,
                   dtot, &Pu);
        hipLaunchKernelGGL(k_offs_from_sorted, dim3(grid_for(Pu, kBlock)), dim3(kBlock), 0, s, Pu, pent, n, e_offs);
        if (Pu == 0) DSS_HIP(hipMemsetAsync(e_offs, 0, sizeof(int64_t) * (n + 1), s));
        mult = m;
    }
    stage_check(s, "index build: entity cells");
    idx->has_mult = general;
    // (2) decodes, per-entity long flags, duration classes, time range
    DevBuf<uint32_t> dec_b;
    DevBuf<uint8_t> elong_b;
    uint32_t *dec = dec_b.ensure(Pu + 1);
    uint8_t *elong = elong_b.ensure(n + 1);
    if (Pu) hipLaunchKernelGGL(k_decode, dim3(grid_for(Pu, kBlock)), dim3(kBlock), 0, s, Pu, e_cells, dec);
    if (n)
        hipLaunchKernelGGL(k_entity_info, dim3(grid_for(n, kBlock)), dim3(kBlock), 0, s, n, e_offs, dec, t0, t1, elong,
                           stat, stat + 65);
    stage_check(s, "index build: entity info");
    unsigned long long h[80];
    DSS_HIP(hipMemcpyAsync(h, stat, sizeof(h), hipMemcpyDeviceToHost, s));
    DSS_HIP(hipStreamSynchronize(s));
    // class threshold: the smallest power of two covering >= 99.9 % of the
    // rows' durations (the rest -- and unbounded ones -- are "long", scanned
    // by every record of their cell)
    unsigned long long rows = 0;
    for (int b = 0; b <= 64; b++) rows += h[b];
    unsigned long long thr = 0, acc = 0;
    for (int b = 0; b <= 62; b++) {
        acc += h[b];
        thr = b == 0 ? 0 : ((1ull << b) - 1);
        if (rows && acc * 1000 >= rows * 999) break;
    }
    idx->dcap_thr = (int64_t)thr;
    DSS_HIP(hipMemsetAsync(stat + 67, 0, sizeof(unsigned long long), s));
    if (n) hipLaunchKernelGGL(k_dcap, dim3(grid_for(n, kBlock)), dim3(kBlock), 0, s, n, t0, t1, thr, stat + 67);
    // query-order quantisation over the rows' start range
    {
        const long long mlo = h[66] ? (long long)(h[65] ^ 0x8000000000000000ull) : 0;
        const long long mhi = h[66] ? (long long)(h[66] ^ 0x8000000000000000ull) : 0;
        const unsigned long long span = (unsigned long long)mhi - (unsigned long long)mlo + (1ull << 33);
        int sh = 0;
        while (sh < 62 && (span >> sh) >= (1ull << (kOrderBits - 1))) sh++;
        idx->tbase = mlo;
        idx->qshift = sh;
    }
    // (3) the grain: quads when an entity's cells fill them (>= 1.5 cells
    // per (entity, quad): metro footprints, corridors), else level-13 cells
    // (city blocks of 1-4 cells, whose quads would add candidates without
    // saving postings)
    int gshift = grain_ == 1 ? kCellShift : kQuadShift;
    if (grain_ == 0 && Pu) {
        hipLaunchKernelGGL(k_grain_counts, dim3(grid_for(Pu, kBlock)), dim3(kBlock), 0, s, Pu, e_cells, pent, t1, cell_lo,
                           cell_hi, stat + 75);
        unsigned long long g[2];
        DSS_HIP(hipMemcpyAsync(g, stat + 75, sizeof(g), hipMemcpyDeviceToHost, s));
        DSS_HIP(hipStreamSynchronize(s));
        gshift = 2 * g[0] >= 3 * g[1] ? kQuadShift : kCellShift;
    }
    // a (cell, entity) repeated more than 255 times in a stored array (RID
    // unnest(cells) multiplicities, MaxSubscriptionCount) does not fit the
    // quad grain's 8 bits per child: the cell grain keeps the full 32 bits
    if (general && h[77] != 0) gshift = kCellShift;
    idx->gshift = gshift;
    // (4) slots: dense range and the irregular side table
    const BuildCtx bc{e_cells, pent, t0, t1, cell_lo, cell_hi, gshift};
    if (Pu)
        hipLaunchKernelGGL(k_dense_range, dim3(grid_for(Pu, kBlock)), dim3(kBlock), 0, s, Pu, e_cells, pent, t1, cell_lo,
                           cell_hi, gshift, stat + 68, stat + 70);
    DSS_HIP(hipMemcpyAsync(h + 67, stat + 67, 4 * sizeof(unsigned long long), hipMemcpyDeviceToHost, s));
    DSS_HIP(hipStreamSynchronize(s));
    idx->dcap = (int64_t)h[67];
    idx->kmin = h[68] == ~0ull ? 0 : h[68];
    idx->n_dense = h[68] == ~0ull ? 0 : (int64_t)(h[69] - h[68] + 1);
    idx->n_irr = 0;
    if (h[70]) {
        DevBuf<uint64_t> ia, ib;
        uint64_t *i0 = ia.ensure(h[70] + 1), *i1 = ib.ensure(h[70] + 1);
        int64_t *dtot = (int64_t *)(stat + 78), nirr_p = 0, nu = 0;
        compact_if(Pu, PredIrr{bc}, EmitIrr{e_cells, i0}, tmp_, tmp2_, s, dtot, &nirr_p);
        radix_sort_keys(i0, i1, nirr_p, 64, tmp_, s);
        uint64_t *irr = idx->irr_cells.ensure_exact(nirr_p + 1);
        compact_if(nirr_p, PredRunStart64{i1}, EmitCopy64{i1, irr}, tmp_, tmp2_, s, dtot, &nu);
        idx->n_irr = nu;
    } else {
        idx->irr_cells.ensure_exact(1);
    }
    const int64_t ns = idx->n_slots();
    if (ns >= (int64_t)0x7fffffff) throw Error(DSSG_ERR_INVALID, "index: more than 2^31 - 1 cell slots");
    // (5) postings: the first in-range position of each (entity, group) of
    // included rows, sorted by m, then stably by (slot, long) -> (slot, class, m)
    int64_t NP = 0;
    DevBuf<uint32_t> pos_b;
    uint32_t *pos = nullptr;
    {
        DevBuf<unsigned long long> ka, kb;
        DevBuf<uint32_t> va;
        unsigned long long *k0 = ka.ensure(Pu + 1), *k1 = kb.ensure(Pu + 1);
        uint32_t *v0 = va.ensure(Pu + 1);
        pos = pos_b.ensure(Pu + 1);
        int64_t *dtot = (int64_t *)(stat + 78);
        compact_if(Pu, PredPosting{bc}, EmitPostingKey{bc, k0, v0}, tmp_, tmp2_, s, dtot, &NP);
        radix_sort_pairs(k0, k1, v0, pos, NP, 64, tmp_, s);
    }
    stage_check(s, "index build: posting sort");
    idx->n_p = NP;
    IndexView pv = view_of(idx);  // slots only (postings not built yet)
    DevBuf<uint32_t> key_b, key2_b, pos2_b;
    uint32_t *key = key_b.ensure(NP + 1), *key2 = key2_b.ensure(NP + 1), *pos2 = pos2_b.ensure(NP + 1);
    // altitude bands (tools/band_sim.py): the regular postings
    // of slots with >= band_dense_ of them split into bands_ runs by alt_lo
    // quantile, so a 64-posting tile's altitude hull excludes the records of
    // other altitudes (configs[2]: 38 % of the lane tests failed on altitude)
    int nb = 1, kshift = 1;
    BandThr bt{};
    DevBuf<uint32_t> scnt_b;
    const uint32_t *scnt = nullptr;
    const uint32_t dense = (uint32_t)std::min<int64_t>(band_dense_, 0xffffffffll);
    if (bands_ > 1 && NP && n && ns < ((int64_t)1 << 27)) {
        uint32_t *sc = scnt_b.ensure(ns + 1);
        DSS_HIP(hipMemsetAsync(sc, 0, sizeof(uint32_t) * (ns + 1), s));
        hipLaunchKernelGGL(k_slot_hist, dim3(grid_for(NP, kBlock)), dim3(kBlock), 0, s, NP, pv, pos, e_cells, sc);
        unsigned long long *nd = stat + 77;  // (the multiplicity word is consumed)
        DSS_HIP(hipMemsetAsync(nd, 0, sizeof(unsigned long long), s));
        hipLaunchKernelGGL(k_dense_slots, dim3(grid_for(ns, kBlock)), dim3(kBlock), 0, s, ns, sc, dense, nd);
        constexpr int64_t kSamples = 8192;
        const int64_t m = std::min<int64_t>(kSamples, n);
        DevBuf<float> smp_b;
        float *smp = smp_b.ensure(m + 1);
        hipLaunchKernelGGL(k_sample_f32, dim3(grid_for(m, kBlock)), dim3(kBlock), 0, s, n, alt_lo, m, smp);
        std::vector<float> hs((size_t)m);
        unsigned long long ndense = 0;
        DSS_HIP(hipMemcpyAsync(hs.data(), smp, sizeof(float) * m, hipMemcpyDeviceToHost, s));
        DSS_HIP(hipMemcpyAsync(&ndense, nd, sizeof(ndense), hipMemcpyDeviceToHost, s));
        DSS_HIP(hipStreamSynchronize(s));
        hs.erase(std::remove_if(hs.begin(), hs.end(), [](float x) { return x != x; }), hs.end());
        std::sort(hs.begin(), hs.end());
        if (ndense > 0 && !hs.empty() && hs.front() < hs.back()) {
            nb = std::min(bands_, 8);
            kshift = 4;
            for (int b = 0; b < nb - 1; b++) bt.v[b] = hs[(size_t)((b + 1) * hs.size() / (size_t)nb)];
            scnt = sc;
        }
    }
    idx->n_bands = nb;
    if (NP)
        hipLaunchKernelGGL(k_slot_keys, dim3(grid_for(NP, kBlock)), dim3(kBlock), 0, s, NP, pv, pos, e_cells, pent, t0, t1,
                           thr, kshift, scnt, dense, alt_lo, bt, nb, key);
    radix_sort_pairs(key, key2, pos, pos2, NP, bits_for(ns) + kshift, tmp_, s);
    scnt_b.release();
    key_b.release();
    pos_b.release();
    tmp_.release();  // the sort's alternate buffers
    // (6) posting attributes in final order
    uint32_t *b_e = idx->b_e.ensure_exact(NP + 1);
    uint8_t *b_meta = idx->b_meta.ensure_exact(NP + 1);
    float2 *b_alt = idx->b_alt.ensure_exact(NP + 1);
    longlong2 *b_t = idx->b_t.ensure_exact(NP + 1);
    ulonglong2 *b_sig = idx->b_sig.ensure_exact(2 * (NP + 1));
    int32_t *b_owner = idx->b_owner.ensure_exact(owner ? NP + 1 : 1);
    uint32_t *b_mult = idx->b_mult.ensure_exact(mult ? NP + 1 : 1);
    if (NP)
        hipLaunchKernelGGL(k_gather, dim3(grid_for(NP, kBlock)), dim3(kBlock), 0, s, NP, pos2, pent, e_offs, e_cells,
                           dec, elong, alt_lo, alt_hi, t0, t1, owner, mult, gshift, b_e, b_meta, b_alt, b_t, b_sig,
                           b_owner, b_mult, stat + 71);
    stage_check(s, "index build: gather");
    pos2_b.release();
    dec_b.release();
    // (7) slot table: s_post (first posting per slot, scan of counts), s_nreg
    {
        DevBuf<uint32_t> f_b, e_b, r_b, bf_b;
        uint32_t *sf = f_b.ensure(ns + 1), *se = e_b.ensure(ns + 1), *sr = r_b.ensure(ns + 1);
        uint32_t *bfirst = nullptr, *sband = nullptr;
        DSS_HIP(hipMemsetAsync(sf, 0, sizeof(uint32_t) * (ns + 1), s));
        DSS_HIP(hipMemsetAsync(se, 0, sizeof(uint32_t) * (ns + 1), s));
        DSS_HIP(hipMemsetAsync(sr, 0, sizeof(uint32_t) * (ns + 1), s));
        if (nb > 1) {
            bfirst = bf_b.ensure(8 * (ns + 1));
            DSS_HIP(hipMemsetAsync(bfirst, 0, sizeof(uint32_t) * 8 * (ns + 1), s));
            sband = idx->s_band.ensure_exact(8 * (ns + 1));
        } else {
            idx->s_band.release();
        }
        if (NP)
            hipLaunchKernelGGL(k_slot_bounds, dim3(grid_for(NP, kBlock)), dim3(kBlock), 0, s, NP, key2, kshift, sf, se,
                               sr, bfirst, stat + 72);
        DevBuf<int64_t> c_b, o_b;
        int64_t *cnt = c_b.ensure(ns + 1), *off = o_b.ensure(ns + 2);
        uint32_t *nreg = idx->s_nreg.ensure_exact(ns + 1);
        if (ns)
            hipLaunchKernelGGL(k_slot_counts, dim3(grid_for(ns, kBlock)), dim3(kBlock), 0, s, ns, sf, se, sr,
                               (const uint32_t *)bfirst, cnt, nreg, sband, stat + 74);
        exclusive_scan_i64(cnt, off, ns, tmp2_, s);
        uint64_t *sp = idx->s_post.ensure_exact(ns + 1);
        hipLaunchKernelGGL(k_u64_store, dim3(grid_for(ns + 1, kBlock)), dim3(kBlock), 0, s, ns + 1, off, sp);
        uint8_t *lfp = idx->s_lfp.ensure_exact(ns + 1);
        DSS_HIP(hipMemsetAsync(lfp, 0, ns + 1, s));
        if (NP)
            hipLaunchKernelGGL(k_slot_lfp, dim3(grid_for(NP, kBlock)), dim3(kBlock), 0, s, NP, key2, kshift, b_meta, lfp);
    }
    stage_check(s, "index build: slot table");
    // (8) entity-level attributes: ends_at, owner, owner -> entities, counters
    int64_t *et1 = idx->e_t1.ensure_exact(n + 1);
    device_copy(et1, t1, sizeof(int64_t) * n, s);
    int64_t *notify = idx->e_notify.ensure_exact(n + 1);
    DSS_HIP(hipMemsetAsync(notify, 0, sizeof(int64_t) * (n + 1), s));
    if (owner) {
        int32_t *eo = idx->e_owner.ensure_exact(n + 1);
        device_copy(eo, owner, sizeof(int32_t) * n, s);
        DevBuf<uint32_t> kb, vb;
        uint32_t *k0 = kb.ensure(n + 1), *v0 = vb.ensure(n + 1);
        uint32_t *ok = idx->o_key.ensure_exact(n + 1), *oe = idx->o_ent.ensure_exact(n + 1);
        if (n) hipLaunchKernelGGL(k_owner_keys, dim3(grid_for(n, kBlock)), dim3(kBlock), 0, s, n, owner, k0, v0);
        radix_sort_pairs(k0, ok, v0, oe, n, 32, tmp_, s);
    }
    DSS_HIP(hipMemcpyAsync(h + 70, stat + 70, 5 * sizeof(unsigned long long), hipMemcpyDeviceToHost, s));
    DSS_HIP(hipStreamSynchronize(s));
    idx->n_long_fp = (int64_t)h[71];
    idx->n_cells = (int64_t)h[72];
    idx->n_long = (int64_t)h[73];
    idx->max_cell_postings = (int64_t)h[74];
    tmp_.release();
    tmp2_.release();
}

// ================================================================== search
void SearchEngine::stats(const dssg_index *idx, int64_t nq, const int64_t *q_offs, const uint64_t *q_cells, hipStream_t s,
                         int64_t *matched, int64_t *distinct)
{
    unsigned long long *cnt = counter_.ensure(8);
    DSS_HIP(hipMemsetAsync(cnt, 0, 4 * sizeof(unsigned long long), s));
    QueryView qv{nq, q_offs, q_cells, nullptr, nullptr, nullptr, nullptr, nullptr};
    if (nq > 0) hipLaunchKernelGGL(k_stats, dim3(grid_for(nq, kBlock / 64)), dim3(kBlock), 0, s, view_of(idx), qv, cnt);
    unsigned long long h[4];
    DSS_HIP(hipMemcpyAsync(h, cnt, sizeof(h), hipMemcpyDeviceToHost, s));
    DSS_HIP(hipStreamSynchronize(s));
    *matched = (int64_t)h[0];
    *distinct = (int64_t)h[1];
}

int64_t SearchEngine::touched(const dssg_index *idx, int64_t nq, const int64_t *q_offs, const uint64_t *q_cells,
                              hipStream_t s)
{
    if (nq <= 0) return 0;
    const int64_t nqc = fetch(q_offs + nq, s), ns = idx->n_slots();
    DevBuf<uint32_t> mark_b;
    uint32_t *mark = mark_b.ensure(ns + 1);
    DSS_HIP(hipMemsetAsync(mark, 0, sizeof(uint32_t) * (ns + 1), s));
    unsigned long long *sum = counter_.ensure(8) + 4;
    DSS_HIP(hipMemsetAsync(sum, 0, sizeof(unsigned long long), s));
    const IndexView a = view_of(idx);
    if (nqc) hipLaunchKernelGGL(k_touch_mark, dim3(grid_for(nqc, kBlock)), dim3(kBlock), 0, s, a, nqc, q_cells, mark);
    if (ns) hipLaunchKernelGGL(k_touch_sum, dim3(grid_for(ns, kBlock)), dim3(kBlock), 0, s, a, ns, mark, sum);
    return (int64_t)fetch(sum, s);
}

// The words of the join's control block the host reads after the join --
// per region the unit, long-unit, pair and tagged-key counters, and misc
// words 0..5 -- gathered into fine-grained host memory (one small launch
// instead of a copy of the whole block).
static_assert(kRegions == 8, "k_ctl_mail gathers 8 region counters per kind");
__global__ void k_ctl_mail(const unsigned long long *ctl, int units, int units_l, int out, int tout, int misc,
                           int stride, int64_t *mail)
{
    const int t = threadIdx.x;
    if (t < 32) {
        const int base = t < 8 ? units : t < 16 ? units_l : t < 24 ? out : tout;
        mail[t] = (int64_t)ctl[base + (t & 7) * stride];
    } else if (t < 38) {
        mail[t] = (int64_t)ctl[misc + (t - 32)];
    }
}

int64_t *SearchEngine::mailbox()
{
    if (!mail_h_) {
        DSS_HIP(hipHostMalloc((void **)&mail_h_, 64 * sizeof(int64_t), hipHostMallocMapped | hipHostMallocCoherent));
        DSS_HIP(hipHostGetDevicePointer((void **)&mail_d_, mail_h_, 0));
    }
    return mail_d_;
}

void SearchEngine::search(const dssg_index *idx, int64_t nq, const int64_t *q_offs, const uint64_t *q_cells,
                          const float *q_alt_lo, const float *q_alt_hi, const int64_t *q_tlo, const int64_t *q_thi,
                          const int32_t *q_owner, hipStream_t s, dssg_pairs *out, int64_t nqc_known)
{
    if (q_owner && !idx->has_owner) throw Error(DSSG_ERR_INVALID, "search by owner on an index built without owners");
    if (nq >= kMaxBatchQ) throw Error(DSSG_ERR_INVALID, "search: more than 2^25 queries per batch");
    timing_events();
    const IndexView ix = view_of(idx);
    const QueryView qv{nq, q_offs, q_cells, q_alt_lo, q_alt_hi, q_tlo, q_thi, q_owner};
    auto empty = [&]() {
        out->q = oq_.ensure(1);
        out->e = oe_.ensure(1);
        out->n = 0;
        out->n_tagged = 0;
        units_ = keys_ = runs_ = iters_ = tests_ = tagged_ = 0;
        join_ms_ = 0;
    };
    if (nq <= 0 || idx->n_p == 0) return empty();
    // the batch's cell count sizes the per-cell buffers and bounds every
    // later device count: from the caller (a covering it just ran), else the
    // one host sync before the join
    const int64_t nqc = nqc_known >= 0 ? nqc_known : fetch(q_offs + nq, s);
    if (nqc >= (int64_t)0xffffffffll) throw Error(DSSG_ERR_CAPACITY, "search: more than 2^32 - 1 query cells per batch");
    if (nqc == 0) return empty();
    if (nq <= small_max_q_ && nqc <= 16 * small_max_q_)
        return search_small(idx, nq, q_offs, q_cells, q_alt_lo, q_alt_hi, q_tlo, q_thi, q_owner, nqc, s, out);
    // one control block (a single memset to start, one copy back per join):
    // dqmax slots, unit region counters (short / long queues), misc counters ([0] pairs [1] tagged
    // [2] lane tests [3] broadcasts [5] long queries [9] scratch), unit queue
    // heads, output region counters -- kRegStride words between counters
    constexpr int kR = kRegions * kRegStride;
    // (the unit counters come before the misc words: each join attempt
    // zeroes everything from misc word 6 on)
    constexpr int kCtlDq = 0, kCtlUnits = kR, kCtlUnitsL = 2 * kR, kCtlMisc = 3 * kR, kCtlQueue = 3 * kR + 16,
                  kCtlQueueL = 4 * kR + 16, kCtlOut = 5 * kR + 16, kCtlTOut = 6 * kR + 16, kCtlWin = 7 * kR + 16,
                  kCtlWords = 7 * kR + 16 + kWinBuckets;
    unsigned long long *ctl = counter_.ensure(kCtlWords);
    unsigned long long *cnt = ctl + kCtlMisc;
    DSS_HIP(hipMemsetAsync(ctl, 0, kCtlWords * sizeof(unsigned long long), s));
    // (1) per query cell: query, decode, slot; per query: long flag
    uint32_t *cq = cq_.ensure(nqc + 1), *dec = dec_.ensure(nqc + 1), *cslot = bt_.ensure(nqc + 1);
    uint32_t *vpre = vpre_.ensure(nqc + 1), *qaux = qaux_.ensure(3 * (nq + 1));
    uint32_t *qvb = qaux, *qvalid = qaux + (nq + 1), *qrank = qaux + 2 * (nq + 1);
    uint8_t *qlong = qlong_.ensure(nq + 1);
    hipLaunchKernelGGL(k_cell_query, dim3(grid_for(nq, kBlock)), dim3(kBlock), 0, s, ix, nq, q_offs, q_cells, cq, dec,
                       cslot, qlong, vpre, qvb, qvalid, cnt + 5);
    // (2) query order: narrow windows by start time, wide ones last
    uint32_t *ok0 = okey_.ensure(nq + 1), *ok1 = okey2_.ensure(nq + 1), *ov0 = oval_.ensure(nq + 1),
             *perm = perm_.ensure(nq + 1);
    hipLaunchKernelGGL(k_qwin, dim3((unsigned)std::min<int64_t>(grid_for(nq, kBlock), 1024)), dim3(kBlock), 0, s, nq,
                       q_tlo, q_thi, ctl + kCtlWin);
    hipLaunchKernelGGL(k_qorder, dim3(grid_for(nq, kBlock)), dim3(kBlock), 0, s, nq, q_tlo, q_thi, (long long)idx->tbase,
                       idx->qshift, (double)idx->dcap, (const unsigned long long *)(ctl + kCtlWin), ok0, ov0,
                       ctl + kCtlDq);
    // (round 6: a one-pass counting sort here -- ties need no order -- took
    // 0.6 ms: the clamped NULL starts of ~2.5 % of the queries share one
    // counter, and same-address atomics serialise; the 2-pass radix sort's
    // per-tile histograms do not)
    radix_sort_pairs(ok0, ok1, ov0, perm, nq, kOrderBits, tmp_, s);
    // (3) keys (slot << 1 | wide, query cell) in that order; records per cell
    int64_t *qc = qcnt_.ensure(nq + 1), *qo = qoff_.ensure(nq + 2);
    hipLaunchKernelGGL(k_qcount, dim3(grid_for(nq, kBlock)), dim3(kBlock), 0, s, nq, perm, qvalid, qc, qrank);
    exclusive_scan_i64(qc, qo, nq, tmp2_, s);
    uint32_t *key = kkey_.ensure(nqc + 1), *skey = kkey2_.ensure(nqc + 1);
    uint64_t *val = kv64_.ensure(nqc + 1), *sval = kv64b_.ensure(nqc + 1);
    QRec *recs = (QRec *)rec_.ensure(sizeof(QRec) * (nqc + 1));
    hipLaunchKernelGGL(k_qrecs, dim3(grid_for(nqc, kBlock)), dim3(kBlock), 0, s, qv, nqc, cq, dec, cslot, qlong, vpre,
                       qvb, qrank, ok1, qo, idx->gshift, key, val, recs);
    // (4) group the keys by cell (stable: each cell's records stay in query
    // order), over the device key count qo[nq] (<= nqc)
    const int64_t *dnkeys = qo + nq;
    radix_sort_pairs_dn(key, skey, val, sval, nqc, dnkeys, bits_for(idx->n_slots()) + 1, tmp_, s);
    const uint64_t *sq = sval;  // (quantised starts in the high words)
    // the records in key order when the index holds groups whose record runs
    // outgrow L2 (configs[2]'s hotspot quads: k_join 2.22 -> 2.05 ms for a
    // 0.094-ms permutation); with only moderate groups (configs[1]'s ~3k
    // postings per quad) the gathers through sval hit L2 and the permutation
    // would cost more than it saves
    const bool key_order = rec_order_ == 2 || (rec_order_ == 0 && idx->max_cell_postings >= kRecPermuteMin);
    QRec *recs_k = recs;
    if (key_order) {
        recs_k = (QRec *)rec2_.ensure(sizeof(QRec) * (nqc + 1));
        hipLaunchKernelGGL(k_rec_permute, dim3(grid_for(4 * nqc, kBlock)), dim3(kBlock), 0, s, dnkeys,
                           (const uint64_t *)sval, (const QRec *)recs, recs_k);
    }
    // (5) join units = 64-posting tiles of every cell the batch meets, each
    // with the records it can meet
    if (n_cu_ == 0) {
        int dev = 0, ncu = 0;
        DSS_HIP(hipGetDevice(&dev));
        DSS_HIP(hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, dev));
        n_cu_ = ncu > 0 ? ncu : 256;
    }
    int64_t ucap = std::max<int64_t>(units_cap_hint_, 1024);  // per region
    // units of cells with long-footprint postings (idx->s_lfp) go to a second
    // set of queues joined by the long variant; the rest by the short one
    const bool any_long = idx->n_long_fp > 0;
    int64_t ucap_l = any_long ? std::max<int64_t>(units_cap_hint_l_, 1024) : 0;
    Unit *units = nullptr, *units_l = nullptr;
    const unsigned ugrid = (unsigned)std::min<int64_t>((nqc + 63) / 64 / (kBlock / 64) + 1, (int64_t)n_cu_ * 16);
    bool ctl_fresh = true;  // the control block as the opening memset left it (the first build and join skip theirs)
    auto build_units = [&]() {
        units = (Unit *)units_buf_.ensure(sizeof(Unit) * (kRegions * (ucap + ucap_l) + 1));
        units_l = units + kRegions * ucap;
        if (!ctl_fresh) {
            DSS_HIP(hipMemsetAsync(ctl + kCtlUnits, 0, kR * sizeof(unsigned long long), s));
            DSS_HIP(hipMemsetAsync(ctl + kCtlUnitsL, 0, kR * sizeof(unsigned long long), s));
        }
        hipLaunchKernelGGL(k_units, dim3(ugrid), dim3(kBlock), 0, s, ix, skey, dnkeys, Regions{ctl + kCtlUnits, ucap},
                           units, Regions{ctl + kCtlUnitsL, ucap_l}, units_l, 64u, sq,
                           (const unsigned long long *)(ctl + kCtlDq), (long long)idx->tbase, idx->qshift);
    };
    build_units();
    // (6) join; grow the output (and the units) and rerun if too small
    JoinArgs ja{};
    ja.ix = ix;
    ja.qv = qv;
    ja.lazy_sig_recs = (uint32_t)std::max<int64_t>(0, std::min<int64_t>(lazy_sig_recs_, 0xffffffffll));
    ja.rec_indirect = key_order ? 0u : 1u;
    const bool dense = join_shape_ == 0 ? dense_out_ : join_shape_ == 2;
    const unsigned nblocks = (unsigned)n_cu_ * (dense ? kJoinBpcDense : kJoinBpcSparse);
    if (out_rcap_ == 0) out_rcap_ = ((int64_t)nq * 16 / kRegions / kOutChunk + 2) * kOutChunk;
    if (any_long && tag_rcap_ == 0) tag_rcap_ = ((int64_t)nq * 4 / kRegions / kOutChunk + 2) * kOutChunk;
    const int qb = bits_for(nq), eb = bits_for(idx->n_e);
    const int hbm = std::min(24, 64 - qb - eb);  // qb <= 25 (kMaxBatchQ), eb <= 32: 7 <= hbm <= 24
    // closing the holes of partly filled / unreserved chunks below n with the
    // entries at or above n
    auto close_holes = [&](int64_t nch, const uint32_t *fills, int64_t n, auto mover) {
        const int64_t nbelow = std::min<int64_t>(nch, (n + kOutChunk - 1) / kOutChunk);
        int64_t *hole = cnt64_.ensure(5 * (nch + 2)), *tail = hole + (nch + 2);
        int64_t *hoff = tail + (nch + 2), *toff = hoff + (nch + 2);
        uint32_t *list = reinterpret_cast<uint32_t *>(toff + (nch + 2));
        unsigned int *nlist = reinterpret_cast<unsigned int *>(cnt + 12);  // (zeroed with the control block)
        DSS_HIP(hipMemsetAsync(nlist, 0, sizeof(unsigned int), s));
        hipLaunchKernelGGL(k_fix_counts, dim3(grid_for(nch, kBlock)), dim3(kBlock), 0, s, nch, fills, n, hole, tail,
                           list, nlist);
        exclusive_scan_i64(hole, hoff, nch, tmp2_, s);
        exclusive_scan_i64(tail, toff, nch, tmp2_, s);
        if (nbelow > 0)
            hipLaunchKernelGGL(k_fix_fill<decltype(mover)>, dim3((unsigned)std::min<int64_t>(nbelow, (int64_t)n_cu_ * 8)),
                               dim3(kFixBlock), 0, s, nch, (const uint32_t *)list, (const unsigned int *)nlist, fills, n,
                               hole, hoff, toff, mover);
    };
    // the overflow pair buffers of an earlier batch (whose output this batch
    // replaces) go before the primary ones regrow to take their place: one
    // context never holds both at their full size
    oq2_.release();
    oe2_.release();
    for (int attempt = 0; attempt < 6; attempt++) {
        const int64_t cap = kRegions * out_rcap_, nch = cap / kOutChunk;
        uint32_t *oq = oq_.ensure(cap + 1), *oe = oe_.ensure(cap + 1);
        const int64_t tcap = any_long ? kRegions * tag_rcap_ : 0, tnch = tcap / kOutChunk;
        uint32_t *fills = fills_.ensure(nch + tnch + 1), *tfills = fills + nch;
        unsigned long long *tk = any_long ? tkey_.ensure(tcap + 1) : nullptr;
        DSS_HIP(hipMemsetAsync(fills, 0, sizeof(uint32_t) * (nch + tnch), s));
        // (misc word 5, the long-query count of k_cell_query, survives; on the
        // first attempt nothing has written these words since the opening
        // memset but k_qwin's histogram, which nothing reads after k_qorder)
        if (!ctl_fresh) {
            DSS_HIP(hipMemsetAsync(ctl + kCtlMisc, 0, 5 * sizeof(unsigned long long), s));
            DSS_HIP(hipMemsetAsync(ctl + kCtlMisc + 6, 0, (kCtlWords - kCtlMisc - 6) * sizeof(unsigned long long), s));
        }
        ctl_fresh = false;
        ja.ur = Regions{ctl + kCtlUnits, ucap};
        ja.out = OutArgs{oq, oe, OutStream{out_rcap_, fills, ctl + kCtlOut}, tk, OutStream{tag_rcap_, tfills, ctl + kCtlTOut},
                         eb, hbm, cnt};
        if (timing_) DSS_HIP(hipEventRecord(ev0_, s));
        const bool quads = idx->gshift == kQuadShift;
        auto kshort = quads ? (dense ? (q_owner ? k_join<true, false, true, true> : k_join<false, false, true, true>)
                                     : (q_owner ? k_join<true, false, false, true> : k_join<false, false, false, true>))
                            : (dense ? (q_owner ? k_join<true, false, true, false> : k_join<false, false, true, false>)
                                     : (q_owner ? k_join<true, false, false, false> : k_join<false, false, false, false>));
        hipLaunchKernelGGL(kshort, dim3(nblocks), dim3(64 * kWaves), 0, s, ja, (const QRec *)recs_k,
                           (const uint64_t *)sval, (const Unit *)units, ctl + kCtlQueue);
        if (any_long) {  // the same output streams, continued
            auto klong = quads ? (q_owner ? k_join<true, true, false, true> : k_join<false, true, false, true>)
                               : (q_owner ? k_join<true, true, false, false> : k_join<false, true, false, false>);
            JoinArgs jl = ja;
            jl.ur = Regions{ctl + kCtlUnitsL, ucap_l};
            // sized by the previous batch's long units (>= ~8 per wave), at
            // most what fits at the variant's occupancy: its waves loop over
            // the queue until it is drained, and every idle wave still visits
            // the 8 region counters -- a full-chip launch over a few
            // thousand units cost configs[2] ~0.2 ms
            if (occ_long_ == 0) {
                int occ = 0;
                DSS_HIP(hipOccupancyMaxActiveBlocksPerMultiprocessor(&occ, reinterpret_cast<const void *>(klong),
                                                                     64 * kWaves, 0));
                occ_long_ = std::max(1, occ);
            }
            const int64_t want = (long_units_prev_ + 8 * kWaves - 1) / (8 * kWaves);
            const unsigned lblocks = (unsigned)std::max<int64_t>(
                std::min<int64_t>((int64_t)n_cu_ * occ_long_, std::max<int64_t>(want, n_cu_)), 1);
            hipLaunchKernelGGL(klong, dim3(lblocks), dim3(64 * kWaves), 0, s, jl, (const QRec *)recs_k,
                               (const uint64_t *)sval, (const Unit *)units_l, ctl + kCtlQueueL);
        }
        if (timing_) DSS_HIP(hipEventRecord(ev1_, s));
        unsigned long long h[kCtlWords];
        {
            int64_t *mail = mailbox();
            hipLaunchKernelGGL(k_ctl_mail, dim3(1), dim3(64), 0, s, (const unsigned long long *)ctl, kCtlUnits,
                               kCtlUnitsL, kCtlOut, kCtlTOut, kCtlMisc, kRegStride, mail);
            DSS_HIP(hipStreamSynchronize(s));
            volatile const int64_t *mh = mail_h_;
            for (int r = 0; r < kRegions; r++) {
                h[kCtlUnits + r * kRegStride] = (unsigned long long)mh[r];
                h[kCtlUnitsL + r * kRegStride] = (unsigned long long)mh[8 + r];
                h[kCtlOut + r * kRegStride] = (unsigned long long)mh[16 + r];
                h[kCtlTOut + r * kRegStride] = (unsigned long long)mh[24 + r];
            }
            for (int m = 0; m < 6; m++) h[kCtlMisc + m] = (unsigned long long)mh[32 + m];
        }
        int64_t nu = 0, umax = 0, umax_l = 0, omax = 0, tmax = 0;
        for (int r = 0; r < kRegions; r++) {
            const int64_t u = (int64_t)h[kCtlUnits + r * kRegStride], ul = (int64_t)h[kCtlUnitsL + r * kRegStride];
            nu += u + ul;
            umax = std::max(umax, u);
            umax_l = std::max(umax_l, ul);
            omax = std::max(omax, (int64_t)h[kCtlOut + r * kRegStride]);
            tmax = std::max(tmax, (int64_t)h[kCtlTOut + r * kRegStride]);
        }
        if (umax > ucap || umax_l > ucap_l) {  // the units did not fit: regrow, rebuild them, rerun the join
            if (umax > ucap) ucap = umax + umax / 4 + 1024;
            if (umax_l > ucap_l) ucap_l = umax_l + umax_l / 4 + 1024;
            build_units();
            continue;
        }
        int64_t nul = 0;
        for (int r = 0; r < kRegions; r++) nul += (int64_t)h[kCtlUnitsL + r * kRegStride];
        long_units_prev_ = nul;
        units_cap_hint_ = std::max<int64_t>(units_cap_hint_, umax + umax / 8);
        units_cap_hint_l_ = std::max<int64_t>(units_cap_hint_l_, umax_l + umax_l / 8);
        bool rerun = false;
        if (omax > out_rcap_) {  // an output region filled up: regrow (per region) and rerun
            out_rcap_ = ((omax + omax / 8) / kOutChunk + 2) * kOutChunk;
            rerun = true;
        }
        if (any_long && tmax > tag_rcap_) {  // the same for the tagged keys
            tag_rcap_ = ((tmax + tmax / 8) / kOutChunk + 2) * kOutChunk;
            rerun = true;
        }
        if (rerun) continue;
        const int64_t n = (int64_t)h[kCtlMisc + 0], nt = (int64_t)h[kCtlMisc + 1];
        if (timing_) {
            float ms = 0;
            DSS_HIP(hipEventElapsedTime(&ms, ev0_, ev1_));
            join_ms_ = ms;
            keys_ = (int64_t)fetch(dnkeys, s);
        }
        runs_ = 0;
        units_ = nu;
        tests_ = (int64_t)h[kCtlMisc + 2];
        // the next batch's join shape: dense output (pairs above a quarter of
        // the lane tests) takes the wider stage
        if (tests_ > 0) dense_out_ = 4 * n > tests_;
        iters_ = (int64_t)h[kCtlMisc + 3];
        long_queries_ = (int64_t)h[kCtlMisc + 5];
        long_postings_ = idx->n_long_fp;
        tagged_ = nt;
        close_holes(nch, fills, n, MovePairs{oq, oe});
        if (nt == 0) {
            out->q = oq;
            out->e = oe;
            out->n = n;
            out->n_tagged = 0;
            return;
        }
        // long x long keys: contiguous, grouped by hash bucket, unique,
        // appended after the pairs (in place when the pair buffer has room;
        // the next batch's buffer is sized for it)
        close_holes(tnch, tfills, nt, MoveKeys{tk});
        uint32_t *fq = oq, *fe = oe;
        if (n + nt > cap) {
            fq = oq2_.ensure(n + nt + 1);
            fe = oe2_.ensure(n + nt + 1);
            device_copy(fq, oq, sizeof(uint32_t) * n, s);
            device_copy(fe, oe, sizeof(uint32_t) * n, s);
            out_rcap_ = std::max<int64_t>(out_rcap_, ((n + nt) / kRegions / kOutChunk + 2) * kOutChunk);
        }
        unsigned long long *k1 = tk, *k2 = tkey2_.ensure(nt + 1);
        int64_t *dtot = (int64_t *)(cnt + 9);
        int64_t nuq = 0;
        if (tag_bucket_avg_ <= 0) {  // one full sort of the keys
            radix_sort_keys(k1, k2, nt, 64, tmp_, s);
            compact_if(nt, PredRunU64{k2}, EmitPairFromKey{k2, fq, fe, n, eb, hbm}, tmp_, tmp2_, s, dtot, &nuq);
        } else {
            int hb = 1;
            while (hb < hbm && (nt >> hb) > tag_bucket_avg_) hb++;
            radix_sort_keys(k1, k2, nt, hb, tmp_, s);
            const int64_t nb = (int64_t)1 << hb;
            int64_t *bs = tb_.ensure(4 * nb + 2), *be = bs + nb, *bc = be + nb, *bo = bc + nb;
            uint8_t *ovf = tovf_.ensure(nb + 1);
            DSS_HIP(hipMemsetAsync(bs, 0, 2 * nb * sizeof(int64_t), s));
            hipLaunchKernelGGL(k_tag_bounds, dim3(grid_for(nt, kBlock)), dim3(kBlock), 0, s, nt, k2, hb, bs, be);
            hipLaunchKernelGGL(k_tag_dedupe, dim3((unsigned)nb), dim3(kDedupBlock), 0, s, k2, bs, be, hbm, k1, bc, ovf,
                               cnt + 10);
            // distinct pairs of the regular buckets (the scan total) and the
            // flagged buckets' count, through the host mailbox
            int64_t *mail = mailbox();
            exclusive_scan_i64(bc, bo, nb, tmp2_, s, mail + 40);
            hipLaunchKernelGGL(k_tag_emit, dim3((unsigned)nb), dim3(256), 0, s, k1, bs, bc, bo, eb, fq + n, fe + n);
            mail_counters(reinterpret_cast<const unsigned int *>(cnt + 10), nullptr, nullptr, mail + 41, s);
            DSS_HIP(hipStreamSynchronize(s));
            volatile const int64_t *mh = mail_h_;
            nuq = mh[40];
            if (mh[41]) {  // flagged buckets: full sort of their keys
                int64_t no = 0, nov = 0;
                compact_if(nt, PredOvf{k2, ovf, hb}, EmitShift{k2, k1, hbm}, tmp_, tmp2_, s, dtot, &no);
                radix_sort_keys(k1, k2, no, qb + eb, tmp_, s);
                compact_if(no, PredRunU64{k2}, EmitPairFromKey{k2, fq, fe, n + nuq, eb, 0}, tmp_, tmp2_, s, dtot, &nov);
                nuq += nov;
            }
        }
        if (idx->cell_lo > 0 && nuq > 0) {  // a cell-range shard past the first: exactly-once across shards
            uint8_t *keep = tovf_.ensure(nuq + 1);  // (the bucket flags are consumed)
            hipLaunchKernelGGL(k_tag_shard_keep, dim3(grid_for(nuq, kBlock)), dim3(kBlock), 0, s, nuq, fq + n, fe + n,
                               qv, ix, (uint64_t)idx->cell_lo, keep);
            uint32_t *tq = reinterpret_cast<uint32_t *>(k2), *te = tq + nuq;  // k2 holds >= 2 nuq words
            int64_t nk = 0;
            compact_if(nuq, PredFlag8{keep}, EmitPairCopy{fq + n, fe + n, tq, te}, tmp_, tmp2_, s, dtot, &nk);
            device_copy(fq + n, tq, sizeof(uint32_t) * nk, s);
            device_copy(fe + n, te, sizeof(uint32_t) * nk, s);
            nuq = nk;
        }
        out->q = fq;
        out->e = fe;
        out->n = n + nuq;
        out->n_tagged = nuq;
        return;
    }
    throw Error(DSSG_ERR_DEVICE, "search: output size did not converge");
}

static const char *const kJProfNames[kJProf] = {
    "lane_tests", "time_fail", "altitude_fail", "owner_fail", "quad_mask_fail", "pass",
    "kept_first_group", "distinct_checks", "distinct_drops", "kept", "staged_batches", "staged_records",
    "loaded_records", "units_with_work", "distinct_wave_iters", "emit_lane_major_batches",
    "emit_record_major_batches", "emit_lane_major_wave_iters", "batches_without_pairs", "posting_lanes",
    "long_pairs_kept_first_quad", "long_pairs_kept_uncertain"};

const char *join_profile_name(int i) { return i >= 0 && i < kJProf ? kJProfNames[i] : nullptr; }

int join_profile_read(int64_t *out, int n)
{
#ifdef DSS_JOIN_PROFILE
    unsigned long long h[kJProf] = {};
    DSS_HIP(hipDeviceSynchronize());
    DSS_HIP(hipMemcpyFromSymbol(h, HIP_SYMBOL(g_jprof), sizeof(h), 0, hipMemcpyDeviceToHost));
    const unsigned long long z[kJProf] = {};
    DSS_HIP(hipMemcpyToSymbol(HIP_SYMBOL(g_jprof), z, sizeof(z), 0, hipMemcpyHostToDevice));
    const int k = n < kJProf ? n : kJProf;
    for (int i = 0; i < k; i++) out[i] = (int64_t)h[i];
    return k;
#else
    (void)out;
    (void)n;
    return 0;
#endif
}

}  // namespace dss
