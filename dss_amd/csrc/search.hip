// Entity index + 4D overlap join on gfx950.
//
// Replaces the CockroachDB side of the reference search:
//   scd_cells_operations PK (cell_id, operation_id) + scd_operations
//     (pkg/scd/store/cockroach/store.go:120-147) and the query at
//     pkg/scd/store/cockroach/operations.go:376-402;
//   RID `cells INT64[]` + INVERTED INDEX (pkg/rid/cockroach/store.go:122-151)
//     and the `cells && $n` queries (identification_service_area.go:170-180,
//     subscriptions.go:222-273).
//
// Index layout in HBM (built once, resident):
//  * plain postings sorted by (cell, entity) -- the cell -> entity map the
//    SQL index holds; level-13 cells found with one dense lookup (slot =
//    cell >> 35, a 29-bit face+Hilbert prefix), any other id (the reference
//    tests use invalid face-7 ids as opaque keys, Q12) via a sorted side table;
//  * time-bucketed postings: each posting is copied into every time bucket
//    its [t0, t1] touches (entities spanning more than kLongSpan buckets go,
//    once, to the "long" bucket 63), sorted by (slot, bucket, entity), SoA
//    with the filter attributes and a 256-bit "prefix signature" inlined.
//
// Join: the batch's (query cell, bucket) keys are radix-sorted
// so every non-empty (slot, bucket) group meets all its queries at once; one
// wavefront owns 64 postings of a group (one per lane, loaded once) and
// sweeps the group's query records with scalar loads, applying the fused
// altitude/time/owner predicate.  A pair is kept exactly once -- at the
// smallest cell the query and the entity share and in their first common
// bucket -- which is the SQL DISTINCT (Q13) without a dedupe pass.
#include <hip/hip_runtime.h>

#include <hipcub/hipcub.hpp>

#include <algorithm>
#include <cmath>
#include <cstring>
#include <type_traits>
#include <utility>
#include <vector>

#include "index_view.cuh"
#include "radix.hpp"
#include "search.hpp"

namespace dss {
namespace {

constexpr unsigned kBlock = 256;
constexpr int kLongBucket = 63;
constexpr int kLongSpan = 8;     // entities touching more buckets go to kLongBucket
#ifndef DSS_MAX_BUCKETS
#define DSS_MAX_BUCKETS 61
#endif
constexpr int kMaxBuckets = DSS_MAX_BUCKETS;  // regular buckets 0..nb-1 (<= 62: bucket 63 is the long one)
static_assert(kMaxBuckets <= 62, "bucket 63 is reserved");
constexpr int kWaves = 4;        // join units per workgroup
constexpr int kQChunk = 1024;    // query records per join unit
#ifndef DSS_JOIN_EXPERIMENT
#define DSS_JOIN_EXPERIMENT 0
#endif
#ifndef DSS_JOIN_LONG
#define DSS_JOIN_LONG 1  // 0: experiments only (long x long pairs would be deduplicated wrongly)
#endif
// k_join<OWNER, LONG>: LONG = false when the batch holds no long query or
// the index no long posting (no long x long pair can exist): the tagging
// code is compiled out of the record loop.
#ifndef DSS_JOIN_SPECIALISE
#define DSS_JOIN_SPECIALISE 1  // record loop specialised on the unit's slot count
#endif
#ifndef DSS_JOIN_SIG_AHEAD
#define DSS_JOIN_SIG_AHEAD 0  // 1: posting signatures in the one-unit-ahead prefetch too
#endif
#ifndef DSS_JOIN_PREFETCH
#define DSS_JOIN_PREFETCH 1  // posting heads loaded one unit ahead
#endif
#ifndef DSS_JOIN_DIAG
#define DSS_JOIN_DIAG 0  // 1: count flushes / exact merges (same-address atomics: slows the join)
#endif
#ifndef DSS_JOIN_STAGE
#define DSS_JOIN_STAGE 1024
#endif
#ifndef DSS_JOIN_GRAB
#define DSS_JOIN_GRAB 4
#endif
constexpr int kStage = DSS_JOIN_STAGE;  // pairs staged per wave in LDS
constexpr int kGrab = DSS_JOIN_GRAB;    // join units a persistent wave takes per queue access
#ifndef DSS_JOIN_BPC
#define DSS_JOIN_BPC 4
#endif
constexpr int kJoinBlocksPerCU = DSS_JOIN_BPC;  // persistent workgroups per CU (LDS: 40 KiB each)
#ifndef DSS_JOIN_WAVES
#define DSS_JOIN_WAVES 4
#endif
#if DSS_JOIN_WAVES > 0
#define DSS_JOIN_OCC __attribute__((amdgpu_waves_per_eu(DSS_JOIN_WAVES)))
#else
#define DSS_JOIN_OCC
#endif
constexpr uint32_t kRank0 = 0x80000000u;    // record: the cell is the query's first cell
constexpr uint32_t kCompact = 0x40000000u;  // record: the query's prefix is compact
constexpr uint32_t kLong = 0x20000000u;     // record: the query is a long footprint (long_cells)
constexpr uint32_t kQFlags = kRank0 | kCompact | kLong;
constexpr uint32_t kTag = 0x80000000u;      // output: a long x long pair, deduplicated after the join

// ---- level-13 decode + prefix signatures -----------------------------------
__device__ __forceinline__ int s2pos_to_ij(int o, int pos) { return (int)((0x874B78B4u >> (8 * o + 2 * pos)) & 3u); }
__device__ __forceinline__ int s2pos_to_orientation(int pos) { return (int)((0xC1u >> (2 * pos)) & 3u); }

// Level-13 (face, i, j) of a cell id (cellid.go faceIJOrientation, walked one
// level at a time); false for ids that are not valid level-13 cells.
__device__ __forceinline__ bool decode13(uint64_t c, int &face, int &i, int &j)
{
    if (!is_regular(c)) return false;
    face = (int)(c >> 61);
    int o = face & 1;
    i = j = 0;
#pragma unroll
    for (int l = 0; l < 13; l++) {
        int pos = (int)((c >> (59 - 2 * l)) & 3);
        int ij = s2pos_to_ij(o, pos);
        i = (i << 1) | (ij >> 1);
        j = (j << 1) | (ij & 1);
        o ^= s2pos_to_orientation(pos);
    }
    return true;
}

// Prefix signature of a sorted cell list at cell c ("near-only"): one bit
// per (i mod 16, j mod 16) for every cell < c that lies on c's face within
// +-7 cells of c (mod 16 is injective on that window, so equal bits are
// equal cells); `compact` iff every cell < c is such a near cell.  For two
// lists that meet at c:
//   * near bits overlap           -> they share a cell < c (exact);
//   * no overlap, one side compact -> they share no cell < c (exact: a shared
//     cell < c lies in the compact side's window, so in both near sets);
//   * otherwise both sides are "long" footprints (cells outside an 8 x 8
//     window, see long_cells), which the join never tests (tagged pairs).
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
__device__ __forceinline__ void prefix_sig(const uint64_t *cells, int64_t n, uint64_t c, Sig256 &sig, bool &compact)
{
    int fc = 0, ic = 0, jc = 0;
    const bool cvalid = decode13(c, fc, ic, jc);
    sig.w[0] = sig.w[1] = sig.w[2] = sig.w[3] = 0;
    compact = cvalid;
    for (int64_t k = 0; k < n; k++) {
        uint64_t x = cells[k];
        if (x >= c) break;
        int f, i, j;
        if (cvalid && decode13(x, f, i, j)) {
            const int di = i - ic, dj = j - jc;
            if (f == fc && di >= -7 && di <= 7 && dj >= -7 && dj <= 7) sig_set(sig, i, j);
            else compact = false;
        } else {
            compact = false;  // position unknown
        }
    }
}

// A footprint is "long" unless all its cells are valid level-13 cells of one
// face inside an 8 x 8 window: then every prefix of it is compact at every
// one of its cells.  Two long footprints' pairs skip the signature test.
__device__ __forceinline__ bool long_cells(const uint64_t *cells, int64_t n)
{
    int f0 = -1, imin = 0, imax = 0, jmin = 0, jmax = 0;
    for (int64_t k = 0; k < n; k++) {
        int f, i, j;
        if (!decode13(cells[k], f, i, j)) return true;
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
// Block merge: B cells of each list per step (independent loads, all B x B
// pairs compared in registers), then the block with the smaller last cell
// advances (both on a tie) -- every common element meets its twin in some
// step.  Cells >= c never count (padding with c keeps them out).
template <int B>
__device__ bool no_smaller_shared(const IndexView &a, uint32_t ent, uint64_t c, const uint64_t *qc, int64_t nq)
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

// ============================================================== build kernels
__global__ void k_expand(int64_t n, const int64_t *offs, uint32_t *val)
{
    int64_t e = tid64();
    if (e >= n) return;
    for (int64_t k = offs[e]; k < offs[e + 1]; k++) val[k] = (uint32_t)e;
}

// keep: first of its (cell, entity) run (entity cell lists, always whole);
// reg / irr: kept postings in this index's cell range [lo, hi] (a cell-range
// shard holds only those), split regular level-13 / other ids.
__global__ void k_keep_flags(int64_t P, const uint64_t *key, const uint32_t *val, uint64_t lo, uint64_t hi, int64_t *keep,
                             int64_t *reg, int64_t *irr)
{
    int64_t i = tid64();
    if (i >= P) return;
    bool k = i == 0 || key[i] != key[i - 1] || val[i] != val[i - 1];
    bool in = key[i] >= lo && key[i] <= hi;
    bool r = is_regular(key[i]);
    keep[i] = k;
    reg[i] = k && in && r;
    irr[i] = k && in && !r;
}

__global__ void k_scatter_unique(int64_t P, const uint64_t *key, const uint32_t *val, const int64_t *keep,
                                 const int64_t *kpos, uint64_t *ukey, uint32_t *uval)
{
    int64_t i = tid64();
    if (i >= P || !keep[i]) return;
    ukey[kpos[i]] = key[i];
    uval[kpos[i]] = val[i];
}

__global__ void k_scatter_part(int64_t P, const uint64_t *key, const uint32_t *val, const int64_t *reg,
                               const int64_t *rpos, const int64_t *irr, const int64_t *ipos, int64_t n_reg,
                               uint64_t *p_cell, uint32_t *p_e, uint32_t *p_mult)
{
    int64_t i = tid64();
    if (i >= P || !(reg[i] || irr[i])) return;
    uint32_t m = 1;  // run length of this (cell, entity) in the sorted input
    while (i + m < P && key[i + m] == key[i] && val[i + m] == val[i]) m++;
    const int64_t w = reg[i] ? rpos[i] : n_reg + ipos[i];
    p_cell[w] = key[i];
    p_e[w] = val[i];
    p_mult[w] = m;
}

__global__ void k_owner_keys(int64_t n, const int32_t *owner, uint32_t *key, uint32_t *val)
{
    int64_t e = tid64();
    if (e >= n) return;
    key[e] = (uint32_t)owner[e] ^ 0x80000000u;  // signed order as unsigned
    val[e] = (uint32_t)e;
}

__global__ void k_count_by_entity(int64_t P, const uint32_t *e, unsigned long long *cnt)
{
    int64_t i = tid64();
    if (i < P) atomicAdd(&cnt[e[i]], 1ull);
}

__global__ void k_u64_to_i64(int64_t n, const unsigned long long *a, int64_t *b)
{
    int64_t k = tid64();
    if (k < n) b[k] = (int64_t)a[k];
}

__global__ void k_i64_to_u32(int64_t n, const int64_t *a, uint32_t *b)
{
    int64_t k = tid64();
    if (k < n) b[k] = (uint32_t)a[k];
}

__global__ void k_first_flags(int64_t P, const uint64_t *p_cell, uint32_t *p_e, const int64_t *e_offs,
                              const uint64_t *e_cells, unsigned long long *n_cells)
{
    int64_t i = tid64();
    if (i >= P) return;
    uint32_t e = p_e[i];
    if (e_cells[e_offs[e]] == p_cell[i]) p_e[i] = e | kFirstBit;
    if (i == 0 || p_cell[i] != p_cell[i - 1]) atomicAdd(n_cells, 1ull);
}

__global__ void k_dense_hist(int64_t n_reg, const uint64_t *p_cell, uint64_t kmin, unsigned long long *cnt)
{
    int64_t i = tid64();
    if (i < n_reg) atomicAdd(&cnt[(p_cell[i] >> 35) - kmin], 1ull);
}

__global__ void k_irr_runs(int64_t n_irr_p, const uint64_t *cells, int64_t *flag)
{
    int64_t i = tid64();
    if (i < n_irr_p) flag[i] = (i == 0 || cells[i] != cells[i - 1]) ? 1 : 0;
}
__global__ void k_irr_scatter(int64_t n_irr_p, const uint64_t *cells, const int64_t *flag, const int64_t *pos,
                              int64_t n_reg, uint64_t *irr_cells, uint32_t *irr_start)
{
    int64_t i = tid64();
    if (i < n_irr_p && flag[i]) {
        irr_cells[pos[i]] = cells[i];
        irr_start[pos[i]] = (uint32_t)(n_reg + i);
    }
}

// Time span of the rows that can match (stored NULL ends never do, Q9), and
// the sum / count of the bounded rows' durations (bucket width, build step 5).
__global__ void k_time_range(int64_t n, const int64_t *t0, const int64_t *t1, unsigned long long *mm, double *dsum)
{
    unsigned long long lo = ~0ull, hi = 0, cnt = 0;
    double sum = 0;
    for (int64_t e = tid64(); e < n; e += (int64_t)gridDim.x * blockDim.x) {
        long long a = t0[e], b = t1[e];
        if (b == INT64_MIN) continue;
        long long x = a < b ? a : b, y = a < b ? b : a;
        if (x != INT64_MIN) {
            lo = min(lo, order_key(x));
            if (y != INT64_MAX) {
                sum += (double)y - (double)x;
                cnt++;
            }
        }
        hi = max(hi, order_key(y));
    }
    for (int o = 32; o > 0; o >>= 1) {
        lo = min(lo, __shfl_xor(lo, o));
        hi = max(hi, __shfl_xor(hi, o));
        cnt += __shfl_xor(cnt, o);
        sum += __shfl_xor(sum, o);
    }
    if ((threadIdx.x & 63) == 0) {
        atomicMin(&mm[0], lo);
        atomicMax(&mm[1], hi);
        atomicAdd(&mm[2], cnt);
        atomicAdd(dsum, sum);
    }
}

// Entity bucket range [lo, hi] of [min(t0,t1), max(t0,t1)].
__device__ __forceinline__ void entity_buckets(long long t0, long long t1, const Buckets &bk, int &lo, int &hi)
{
    lo = bucket_of(t0 < t1 ? t0 : t1, bk);
    hi = bucket_of(t0 < t1 ? t1 : t0, bk);
}

__global__ void k_plain_slot(int64_t P, const uint64_t *p_cell, IndexView a, uint32_t *pslot)
{
    int64_t i = tid64();
    if (i >= P) return;
    uint32_t s = 0;
    find_slot(a, p_cell[i], s);  // always found: the tables are built from p_cell
    pslot[i] = s;
}

template <int PASS>
__global__ void k_bucket_copies(int64_t P, const uint32_t *p_e, const uint32_t *pslot, const int64_t *t0,
                                const int64_t *t1, Buckets bk, int64_t *cnt, const int64_t *off, uint64_t *key,
                                uint32_t *val)
{
    int64_t i = tid64();
    if (i >= P) return;
    uint32_t e = p_e[i] & ~kFirstBit;
    long long a = t0[e], b = t1[e];
    if (b == INT64_MIN) {  // stored NULL end: never matches
        if (!PASS) cnt[i] = 0;
        return;
    }
    int lo, hi;
    entity_buckets(a, b, bk, lo, hi);
    bool lng = hi - lo + 1 > kLongSpan;
    if (!PASS) {
        cnt[i] = lng ? 1 : hi - lo + 1;
        return;
    }
    uint64_t sk = (uint64_t)pslot[i] << 6;
    int64_t w = off[i];
    if (lng) {
        key[w] = sk | kLongBucket;
        val[w] = (uint32_t)i;
        return;
    }
    for (int b2 = lo; b2 <= hi; b2++, w++) {
        key[w] = sk | (uint64_t)b2;
        val[w] = (uint32_t)i;
    }
}

__global__ void k_bucket_gather(int64_t NB, const uint32_t *sval, const uint64_t *p_cell, const uint32_t *p_e,
                                const int64_t *e_offs, const uint64_t *e_cells, const float *alo, const float *ahi,
                                const int64_t *t0, const int64_t *t1, const int32_t *owner, Buckets bk, uint32_t *b_e,
                                float2 *b_alt, longlong2 *b_t, uint8_t *b_meta, ulonglong2 *b_sig, int32_t *b_owner)
{
    int64_t j = tid64();
    if (j >= NB) return;
    uint32_t i = sval[j];
    uint32_t pe = p_e[i];
    uint32_t e = pe & ~kFirstBit;
    long long a = t0[e], b = t1[e];
    int lo, hi;
    entity_buckets(a, b, bk, lo, hi);
    Sig256 sig;
    bool compact = false;
    if (!(pe & kFirstBit))
        prefix_sig(e_cells + e_offs[e], e_offs[e + 1] - e_offs[e], p_cell[i], sig, compact);
    else
        sig.w[0] = sig.w[1] = sig.w[2] = sig.w[3] = 0;
    b_e[j] = pe;
    b_alt[j] = make_float2(alo[e], ahi[e]);
    b_t[j] = make_longlong2(a, b);
    const bool lng = long_cells(e_cells + e_offs[e], e_offs[e + 1] - e_offs[e]);
    b_meta[j] = (uint8_t)(lo | (lng ? 0x40 : 0) | (compact ? 0x80 : 0));
    b_sig[2 * j] = make_ulonglong2(sig.w[0], sig.w[1]);
    b_sig[2 * j + 1] = make_ulonglong2(sig.w[2], sig.w[3]);
    if (owner) b_owner[j] = owner[e];
}

__global__ void k_group_mask(int64_t ng, const uint64_t *gkey, unsigned long long *s_mask)
{
    int64_t g = tid64();
    if (g < ng) atomicOr(&s_mask[gkey[g] >> 6], 1ull << (gkey[g] & 63));
}
__global__ void k_slot_pop(int64_t ns, const unsigned long long *s_mask, int64_t *cnt)
{
    int64_t s = tid64();
    if (s < ns) cnt[s] = __popcll(s_mask[s]);
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

// Query record, one per query cell: what one predicate sweep needs.
struct alignas(64) QRec {
    long long tlo, thi;
    float alo, ahi;
    uint32_t qv;   // query | kRank0 | kCompact
    int32_t bq0;   // first bucket of [min(tlo,thi), max(tlo,thi)]
    unsigned long long sig[4];  // prefix signature of the query's cells before this one
};
static_assert(sizeof(QRec) == 64, "QRec layout");

// Owner query and level-13 (face, i, j) of every query cell, the latter
// packed face << 26 | i << 13 | j, or kNoDecode for ids that are not valid
// level-13 cells.  One block per 256 queries: their cell offsets go to LDS,
// then the block's cells are visited coalesced, each finding its query by
// binary search in LDS.
constexpr uint32_t kNoDecode = 0xffffffffu;
// The same pass sets each query's long flag (long_cells semantics): an
// undecodable cell, cells on more than one face, or an (i, j) span wider than
// 7 -- from per-query LDS min/max/face-mask reductions.
__global__ __launch_bounds__(kBlock) void k_cell_query(int64_t nq, const int64_t *offs, const uint64_t *cells,
                                                       uint32_t *cq, uint32_t *dec, uint8_t *qlong,
                                                       unsigned long long *nlong)
{
    __shared__ int64_t so[kBlock + 1];
    __shared__ int s_imin[kBlock], s_imax[kBlock], s_jmin[kBlock], s_jmax[kBlock];
    __shared__ uint32_t s_face[kBlock];  // bit f: a cell on face f; bit 8: an undecodable cell
    const int64_t q0 = (int64_t)blockIdx.x * kBlock;
    const int nb = (int)(nq - q0 < (int64_t)kBlock ? nq - q0 : (int64_t)kBlock);
    for (int i = threadIdx.x; i <= nb; i += kBlock) so[i] = offs[q0 + i];
    s_imin[threadIdx.x] = s_jmin[threadIdx.x] = 1 << 30;
    s_imax[threadIdx.x] = s_jmax[threadIdx.x] = -1;
    s_face[threadIdx.x] = 0;
    __syncthreads();
    const int64_t k1 = so[nb];
    for (int64_t k = so[0] + threadIdx.x; k < k1; k += kBlock) {
        int lo = 0, hi = nb;  // so[lo] <= k < so[hi]
        while (hi - lo > 1) {
            const int mid = (lo + hi) >> 1;
            if (so[mid] <= k) lo = mid;
            else hi = mid;
        }
        cq[k] = (uint32_t)(q0 + lo);
        int f = 0, i = 0, j = 0;
        const bool ok = decode13(cells[k], f, i, j);
        dec[k] = ok ? ((uint32_t)f << 26 | (uint32_t)i << 13 | (uint32_t)j) : kNoDecode;
        if (ok) {
            atomicOr(&s_face[lo], 1u << f);
            atomicMin(&s_imin[lo], i);
            atomicMax(&s_imax[lo], i);
            atomicMin(&s_jmin[lo], j);
            atomicMax(&s_jmax[lo], j);
        } else {
            atomicOr(&s_face[lo], 1u << 8);
        }
    }
    __syncthreads();
    const int t = threadIdx.x;
    bool is_long = false;
    if (t < nb) {
        const uint32_t fm = s_face[t];
        // no cells: not long; else undecodable / multi-face / wide span
        is_long = fm != 0 && ((fm >> 8) != 0 || __popc(fm) > 1 || s_imax[t] - s_imin[t] > 7 ||
                              s_jmax[t] - s_jmin[t] > 7);
        qlong[q0 + t] = is_long ? 1 : 0;
    }
    const unsigned long long m = __ballot(is_long);
    if (m && (threadIdx.x & 63) == __builtin_ctzll(m)) atomicAdd(nlong, (unsigned long long)__popcll(m));
}

// Long postings of the index (b_meta bit 0x40).
__global__ void k_count_long(int64_t NB, const uint8_t *b_meta, unsigned long long *cnt)
{
    const int64_t j = tid64();
    const bool l = j < NB && (b_meta[j] & 0x40) != 0;
    const unsigned long long m = __ballot(l);
    if (m && (threadIdx.x & 63) == __builtin_ctzll(m)) atomicAdd(cnt, (unsigned long long)__popcll(m));
}

// Groups (non-empty (slot, bucket) runs of the index) query cell k meets:
// the buckets of [min(tlo,thi), max(tlo,thi)] plus the long bucket.
__device__ __forceinline__ unsigned long long cell_groups(const IndexView &a, uint64_t cell, long long tlo,
                                                          long long thi, uint32_t &slot)
{
    if (!find_slot(a, cell, slot)) return 0;
    const int bq0 = bucket_of(tlo < thi ? tlo : thi, a.bk), bq1 = bucket_of(tlo < thi ? thi : tlo, a.bk);
    const unsigned long long range = ((1ull << (bq1 + 1)) - 1ull) & ~((1ull << bq0) - 1ull);
    const unsigned long long m0 = a.s_mask[slot];
    return (m0 & range) | (m0 & (1ull << kLongBucket));
}

// (1) one thread per query cell: PASS 0 counts the groups the cell meets;
// PASS 1 writes one (group id, query cell) key per group at koff[k] and the
// cell's query record.  The record's prefix signature covers the query's
// cells before k (prefix_sig semantics: an undecodable cell saturates it;
// `compact` = every earlier cell on this cell's face within +-7 cells).
template <int PASS>
__global__ __launch_bounds__(kBlock) void k_qcells(IndexView a, QueryView qv, int64_t nqc, const uint32_t *cq,
                                                   const uint32_t *dec, int64_t *kcnt, const int64_t *koff,
                                                   uint32_t *gkey, uint32_t *gval, QRec *crec, int32_t *cown,
                                                   const uint8_t *qlong)
{
    const int64_t k = tid64();
    if (!PASS) {
        if (k >= nqc) return;
        const uint32_t q = cq[k];
        uint32_t slot = 0;
        kcnt[k] = __popcll(cell_groups(a, qv.cells[k], qv.tlo[q], qv.thi[q], slot));
        return;
    }
    // PASS 1: every lane of a wave stays to the end (the wave's 64 records
    // leave through LDS as 4 fully coalesced 1 KiB stores); a lane whose
    // cell meets no group writes a record nobody reads
    if (k - (threadIdx.x & 63) >= nqc) return;  // whole wave past the end
    QRec r;
    r.tlo = r.thi = 0;
    r.alo = r.ahi = 0.f;
    r.qv = 0;
    r.bq0 = 0;
    r.sig[0] = r.sig[1] = r.sig[2] = r.sig[3] = 0;
    if (k < nqc) {
        const uint32_t q = cq[k];
        const long long tlo = qv.tlo[q], thi = qv.thi[q];
        const uint64_t cell = qv.cells[k];
        uint32_t slot = 0;
        unsigned long long m = cell_groups(a, cell, tlo, thi, slot);
        int64_t w = koff[k];
        if (m) {
            const unsigned long long m0 = a.s_mask[slot];
            const uint32_t base = a.s_base[slot];
            while (m) {
                const int b = __builtin_ctzll(m);
                m &= m - 1;
                gkey[w] = base + (uint32_t)__popcll(m0 & ((1ull << b) - 1ull));
                gval[w] = (uint32_t)k;
                w++;
            }
            // query record: near-only prefix signature of the query's cells
            // before k (prefix_sig semantics), compact flag, long flag (qlong)
            const int64_t c0 = qv.offs[q];
            const uint32_t dk = dec[k];
            const int f = (int)(dk >> 26), i = (int)((dk >> 13) & 8191u), jj = (int)(dk & 8191u);
            const bool v = dk != kNoDecode;
            Sig256 sig;
            sig.w[0] = sig.w[1] = sig.w[2] = sig.w[3] = 0;
            bool compact = v;
            // the prefix's decodes are loaded 8 at a time (independent loads
            // in flight together), then folded in order
            constexpr int kU = 8;
#if DSS_EXP_QC == 1  // timing experiment only (wrong signatures)
            for (int64_t j0 = k; j0 < k; j0 += kU) {
#else
            for (int64_t j0 = c0; j0 < k; j0 += kU) {
#endif
                uint32_t dd[kU];
#pragma unroll
                for (int u = 0; u < kU; u++) dd[u] = j0 + u < k ? dec[j0 + u] : 0u;
#pragma unroll
                for (int u = 0; u < kU; u++) {
                    if (j0 + u >= k) break;
                    const uint32_t d = dd[u];
                    const int pf = (int)(d >> 26), ci = (int)((d >> 13) & 8191u), cj = (int)(d & 8191u);
                    const int di = ci - i, dj = cj - jj;
                    if (v && d != kNoDecode && pf == f && di >= -7 && di <= 7 && dj >= -7 && dj <= 7) sig_set(sig, ci, cj);
                    else compact = false;
                }
            }
            r.tlo = tlo;
            r.thi = thi;
            r.alo = qv.alo[q];
            r.ahi = qv.ahi[q];
            r.qv = q | (k == c0 ? kRank0 : 0u) | (compact ? kCompact : 0u) | (qlong[q] ? kLong : 0u);
            r.bq0 = bucket_of(tlo < thi ? tlo : thi, a.bk);
            r.sig[0] = sig.w[0];
            r.sig[1] = sig.w[1];
            r.sig[2] = sig.w[2];
            r.sig[3] = sig.w[3];
            if (cown) cown[k] = qv.owner[q];
        }
    }
    __shared__ int4 stage[kBlock / 64][64 * 4];
    const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
    const int4 *rr = reinterpret_cast<const int4 *>(&r);
#pragma unroll
    for (int u = 0; u < 4; u++) stage[wv][4 * lane + u] = rr[u];
    __builtin_amdgcn_wave_barrier();  // one wave writes and reads its own slice, in order
    const int64_t kw = k - lane;
    int4 *dst = reinterpret_cast<int4 *>(crec + kw);
#pragma unroll
    for (int u = 0; u < 4; u++) {
        const int c = 64 * u + lane;
        if (kw + (c >> 2) < nqc) dst[c] = stage[wv][c];
    }
}

// Record range [gbeg[g], gend[g]) of every group in the sorted keys (groups
// no query met keep 0, 0).
__global__ void k_gbounds(int64_t nkeys, const uint32_t *skey, uint32_t *gbeg, uint32_t *gend)
{
    const int64_t i = tid64();
    if (i >= nkeys) return;
    const uint32_t g = skey[i];
    if (i == 0 || skey[i - 1] != g) gbeg[g] = (uint32_t)i;
    if (i == nkeys - 1 || skey[i + 1] != g) gend[g] = (uint32_t)(i + 1);
}

// Postings per lane in a join unit: a unit covers up to 64 * kSlots postings
// of one group, so a typical group (SURVEY config 1: ~75 postings) is one unit
// and each broadcast record is tested against all of it.
#ifndef DSS_JOIN_SLOTS
#define DSS_JOIN_SLOTS 2
#endif
constexpr int kSlots = DSS_JOIN_SLOTS;

// Join unit: (group, tile of <= 64 * kSlots postings, chunk of <= kQChunk
// records), described in 32 bytes so the join reads it with one scalar load.
struct alignas(16) UnitDesc {
    uint32_t p0;     // first posting of the tile
    uint32_t pe;     // end of the group's postings
    uint32_t k0, k1; // the unit's record range in the sorted keys
    uint64_t key;    // group key: slot << 6 | bucket
    uint32_t nslot;  // postings per lane (1..kSlots)
    uint32_t pad;
};
static_assert(sizeof(UnitDesc) == 32, "UnitDesc layout");

// (2) join units, one thread per group of the index; PASS 0 counts, PASS 1
// writes the descriptors at uoff[g].  The unit count stays on the device
// (uoff[ng]); the persistent join reads it.
template <int PASS>
__global__ void k_units(int64_t ng, const uint32_t *bk_start, const uint32_t *gbeg, const uint32_t *gend,
                        const uint64_t *g_key, int64_t *cnt, const int64_t *uoff, UnitDesc *units)
{
    const int64_t g = tid64();
    if (g >= ng) return;
    const int64_t nrec = (int64_t)gend[g] - gbeg[g];
    const int64_t np = (int64_t)bk_start[g + 1] - bk_start[g];
    const int64_t k = min((int64_t)kSlots, max((int64_t)1, (np + 63) / 64));
    const int64_t tp = (np + 64 * k - 1) / (64 * k), tq = (nrec + kQChunk - 1) / kQChunk;
    if (!PASS) {
        cnt[g] = tp * tq;
        return;
    }
    int64_t w = uoff[g];
    for (int64_t i = 0; i < tp; i++)
        for (int64_t j = 0; j < tq; j++, w++) {
            UnitDesc d;
            d.p0 = bk_start[g] + (uint32_t)(i * 64 * k);
            d.pe = bk_start[g + 1];
            d.k0 = gbeg[g] + (uint32_t)(j * kQChunk);
            d.k1 = (uint32_t)min((int64_t)gend[g], (int64_t)d.k0 + kQChunk);
            d.key = g_key[g];
            d.nslot = (uint32_t)k;
            d.pad = 0;
            units[w] = d;
        }
}

// Diagnostics (timing mode): groups met, sum over groups of records x tiles
// (wave iterations before the time pre-filter) and of records x postings
// (useful lane tests).
__global__ void k_work_stats(int64_t ng, const uint32_t *bk_start, const uint32_t *gbeg, const uint32_t *gend,
                             unsigned long long *stat)
{
    int64_t g = tid64();
    unsigned long long it = 0, lt = 0, met = 0;
    if (g < ng) {
        const unsigned long long np = bk_start[g + 1] - bk_start[g];
        const unsigned long long nq = (unsigned long long)(gend[g] - gbeg[g]);
        const unsigned long long k = np > 64 ? kSlots : 1;
        it = nq * ((np + 64 * k - 1) / (64 * k));
        lt = nq * np;
        met = nq ? 1 : 0;
    }
    for (int o = 32; o > 0; o >>= 1) {
        it += __shfl_xor(it, o);
        lt += __shfl_xor(lt, o);
        met += __shfl_xor(met, o);
    }
    if ((threadIdx.x & 63) == 0 && (it || lt || met)) {
        atomicAdd(&stat[0], it);
        atomicAdd(&stat[1], lt);
        atomicAdd(&stat[2], met);
    }
}

// Set bits of m below this lane (v_mbcnt_lo/hi: 2 VALU, no 64-bit and + popcounts).
__device__ __forceinline__ uint32_t mbcnt64(unsigned long long m)
{
    return __builtin_amdgcn_mbcnt_hi((uint32_t)(m >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)m, 0u));
}

// LLVM compare predicates for __builtin_amdgcn_{s,u}icmp / fcmpf (wave masks)
constexpr int kCmpOGE = 3, kCmpOLE = 5, kCmpEQ = 32, kCmpNE = 33, kCmpSGE = 39, kCmpSLE = 41;

struct JoinArgs {
    IndexView ix;
    QueryView qv;
    const int64_t *nunits;  // device: written by the unit scan
    const uint64_t *g_key;  // group -> slot << 6 | bucket
    const uint32_t *gbeg, *gend;
    int64_t cap;
    unsigned long long *counter;  // [0] output pairs, [1] of which tagged (q | kTag)
};

// One posting held by a lane.
struct Slot {
    bool valid, first, compact, lng;
    uint32_t ent;
    int be0;
    float2 alt;
    longlong2 t;
    int32_t own;
    ulonglong2 s01, s23;
};

__device__ __forceinline__ void load_slot(const IndexView &ix, uint32_t p, uint32_t pe, bool owner, Slot &s)
{
    s.valid = p < pe;
    s.first = s.compact = s.lng = false;
    s.ent = 0;
    s.be0 = 0;
    s.alt = make_float2(INFINITY, -INFINITY);    // matches nothing
    s.t = make_longlong2(LLONG_MAX, LLONG_MIN);  // matches nothing
    s.own = 0;
    s.s01 = s.s23 = make_ulonglong2(0, 0);
    if (!s.valid) return;
    const uint32_t v = ix.b_e[p];
    if (is_dead(ix, v & ~kFirstBit)) {  // tombstoned by the write path: matches nothing
        s.valid = false;
        return;
    }
    const uint8_t m = ix.b_meta[p];
    s.ent = v & ~kFirstBit;
    s.first = (v & kFirstBit) != 0;
    s.be0 = m & 0x3f;
    s.compact = (m & 0x80) != 0;
    s.alt = ix.b_alt[p];
    s.t = ix.b_t[p];
    if (owner) s.own = ix.b_owner[p];
    if (!s.first) {
        s.s01 = ix.b_sig[2 * (size_t)p];
        s.s23 = ix.b_sig[2 * (size_t)p + 1];
    }
}

// A lane's posting as loaded (software pipeline: loads issued one unit
// ahead, decoded when the unit starts).
struct RawSlot {
    uint32_t p;  // posting index
    uint32_t v;
    uint32_t m;
    float2 alt;
    longlong2 t;
    int32_t own;
#if DSS_JOIN_SIG_AHEAD
    ulonglong2 s01, s23;
#endif
    bool valid;
};

__device__ __forceinline__ void load_raw(const IndexView &ix, uint32_t p, uint32_t pe, bool owner, RawSlot &r)
{
    r.valid = p < pe;
    r.p = p;
    if (!r.valid) return;
    r.v = ix.b_e[p];
    r.m = ix.b_meta[p];
    r.alt = ix.b_alt[p];
    r.t = ix.b_t[p];
    if (owner) r.own = ix.b_owner[p];
#if DSS_JOIN_SIG_AHEAD
    r.s01 = ix.b_sig[2 * (size_t)p];  // loaded for first postings too: no wait on b_e here
    r.s23 = ix.b_sig[2 * (size_t)p + 1];
#endif
}

__device__ __forceinline__ void decode_raw(const IndexView &ix, const RawSlot &r, bool owner, Slot &s)
{
    s.valid = r.valid && !is_dead(ix, r.v & ~kFirstBit);  // tombstoned (write path): matches nothing
    s.first = s.compact = s.lng = false;
    s.ent = 0;
    s.be0 = 0;
    s.alt = make_float2(INFINITY, -INFINITY);    // matches nothing
    s.t = make_longlong2(LLONG_MAX, LLONG_MIN);  // matches nothing
    s.own = 0;
    s.s01 = s.s23 = make_ulonglong2(0, 0);
    if (!s.valid) return;
    s.ent = r.v & ~kFirstBit;
    s.first = (r.v & kFirstBit) != 0;
    s.be0 = (int)(r.m & 0x3f);
    s.compact = (r.m & 0x80) != 0;
    s.lng = (r.m & 0x40) != 0;
    s.alt = r.alt;
    s.t = r.t;
    if (owner) s.own = r.own;
    if (!s.first) {
#if DSS_JOIN_SIG_AHEAD
        s.s01 = r.s01;
        s.s23 = r.s23;
#else  // issued here, used by the record loop: overlaps the record gathers
        s.s01 = ix.b_sig[2 * (size_t)r.p];
        s.s23 = ix.b_sig[2 * (size_t)r.p + 1];
#endif
    }
}

// (3) one wavefront per unit: up to 64 * kSlots postings in registers, the
// unit's query records staged through LDS 64 at a time and broadcast.
template <bool OWNER, bool LONG>
__global__ __launch_bounds__(64 * kWaves) DSS_JOIN_OCC void k_join(JoinArgs a, const QRec *__restrict__ recs,
                                                      const uint32_t *__restrict__ sval,
                                                      const int32_t *__restrict__ rown,
                                                      const UnitDesc *__restrict__ units,
                                                      uint32_t *__restrict__ out_q, uint32_t *__restrict__ out_e,
                                                      uint32_t *__restrict__ work)
{
    // record heads (time window, altitudes, query, bucket) stay in the
    // loading lane's VGPRs and are broadcast with v_readlane; only the
    // prefix signatures (needed for a minority of records) go through LDS
    __shared__ int4 s_sig[kWaves][2][64];
    __shared__ uint2 sp[kWaves][kStage];  // staged (query, entity) pairs: one ds_write_b64 each
    const int lane = threadIdx.x & 63;
    const int w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    int staged = 0;
    int staged_tag = 0;  // staged entries carrying kTag (long x long, separated after the join)
    auto flush = [&]() {
        __builtin_amdgcn_wave_barrier();
#if DSS_JOIN_EXPERIMENT == 1  // timing experiment: drop the pairs
        staged = 0;
#endif
        unsigned long long base = 0;
        if (lane == 0 && staged) {
            base = atomicAdd(&a.counter[0], (unsigned long long)staged);
            if (staged_tag) atomicAdd(&a.counter[1], (unsigned long long)staged_tag);
#if DSS_JOIN_DIAG
            atomicAdd(&work[1], 1u);  // diagnostics: flushes
#endif
        }
        base = __shfl(base, 0);
        for (int k = lane; k < staged; k += 64) {
            const unsigned long long o = base + (unsigned long long)k;
            if ((int64_t)o < a.cap) {
                const uint2 v = sp[w][k];
                out_q[o] = v.x;
                out_e[o] = v.y;
            }
        }
        staged = 0;
        staged_tag = 0;
        __builtin_amdgcn_wave_barrier();
    };
    const IndexView &ix = a.ix;
    const int4 *rec4 = reinterpret_cast<const int4 *>(recs);
    // persistent waves: units come from one queue, kGrab per atomic; the
    // staging buffer carries over between units.  Software pipeline: the next
    // unit's descriptor, posting loads and first record indices are issued
    // before this unit's record gathers, so the two round trips overlap.
    const int64_t nunits = *a.nunits;
    uint32_t ucur = 0, uend = 0;
    auto next_unit = [&]() -> int64_t {
        if (ucur >= uend) {
            uint32_t ub = 0;
            if (lane == 0) ub = atomicAdd(&work[0], (uint32_t)kGrab);
            ub = __builtin_amdgcn_readfirstlane(__shfl(ub, 0));
            if ((int64_t)ub >= nunits) return -1;
            ucur = ub;
            uend = (uint32_t)min((int64_t)ub + kGrab, nunits);
        }
        return (int64_t)ucur++;
    };
    RawSlot raw[kSlots];
    UnitDesc d{};
    uint32_t ci_pre = 0;
    auto prefetch = [&](int64_t un) {
        d = units[un];
        const uint32_t p0 = d.p0 + (uint32_t)lane;
#pragma unroll
        for (int k = 0; k < kSlots; k++) load_raw(ix, k < (int)d.nslot ? p0 + 64u * k : d.pe, d.pe, OWNER, raw[k]);
        ci_pre = d.k0 + (uint32_t)lane < d.k1 ? sval[d.k0 + lane] : 0u;
    };
    int64_t u = next_unit();
#if DSS_JOIN_PREFETCH
    if (u >= 0) prefetch(u);
#endif
    while (u >= 0) {
#if !DSS_JOIN_PREFETCH
        prefetch(u);
#endif
        const UnitDesc cu = d;
        Slot sl[kSlots];
#pragma unroll
        for (int k = 0; k < kSlots; k++) decode_raw(ix, raw[k], OWNER, sl[k]);
        uint32_t ci_first = ci_pre;
        const int64_t un = next_unit();
#if DSS_JOIN_PREFETCH
        if (un >= 0) prefetch(un);
#endif
        {
            const uint64_t key = cu.key;
            const int b = (int)(key & 63);
            const int nslot = (int)cu.nslot;
            // time and altitude bounds of the unit: records whose window or
            // altitude band misses all postings are skipped
            long long tmin = LLONG_MAX, tmax = LLONG_MIN;
            float amin = INFINITY, amax = -INFINITY;
#pragma unroll
            for (int k = 0; k < kSlots; k++) {
                tmin = min(tmin, sl[k].t.x);
                tmax = max(tmax, sl[k].t.y);
                amin = fminf(amin, sl[k].alt.x);
                amax = fmaxf(amax, sl[k].alt.y);
            }
            for (int o = 32; o > 0; o >>= 1) {
                tmin = min(tmin, __shfl_xor(tmin, o));
                tmax = max(tmax, __shfl_xor(tmax, o));
                amin = fminf(amin, __shfl_xor(amin, o));
                amax = fmaxf(amax, __shfl_xor(amax, o));
            }
            const uint64_t cell = cell_of_slot(ix, (uint32_t)(key >> 6));
            const int64_t k0 = cu.k0, k1 = cu.k1;
            uint32_t ci_cur = ci_first;
            for (int64_t base = k0; base < k1; base += 64) {
                const int64_t kk = base + lane;
                // the next batch's record indices are in flight during this batch
                const uint32_t ci_nx = kk + 64 < k1 ? sval[kk + 64] : 0u;
                bool rel = false;
                int4 r0 = make_int4(0, 0, 0, 0), r1 = make_int4(0, 0, 0, 0);
                int32_t rown_l = -1;
                __builtin_amdgcn_wave_barrier();
                if (kk < k1) {
                    const uint32_t ci = ci_cur;
                    r0 = rec4[4 * ci];
                    r1 = rec4[4 * ci + 1];
                    s_sig[w][0][lane] = rec4[4 * ci + 2];
                    s_sig[w][1][lane] = rec4[4 * ci + 3];
                    if (OWNER) rown_l = rown[ci];
                    const long long tlo = ((long long)r0.y << 32) | (uint32_t)r0.x;
                    const long long thi = ((long long)r0.w << 32) | (uint32_t)r0.z;
                    const float alo = __int_as_float(r1.x), ahi = __int_as_float(r1.y);
                    rel = !(tmax < tlo || tmin > thi) && !(amax < alo || amin > ahi);  // else no posting can match
                }
                __builtin_amdgcn_wave_barrier();
                const unsigned long long todo0 = __ballot(rel);
                // The record loop, specialised on the unit's slot count.  All
                // decisions are 64-bit wave masks (SALU); VALU work per record
                // is the four interval compares per slot, plus the signature
                // overlap for slots holding a candidate that needs it.
                auto records = [&](auto nsc) {
                    constexpr int NS = decltype(nsc)::value;
                    unsigned long long mf[NS], mb[NS];
#pragma unroll
                    for (int k = 0; k < NS; k++) {
                        mf[k] = __ballot(sl[k].first);
                        mb[k] = __ballot(sl[k].be0 == b);
                    }
                    unsigned long long todo = todo0;
                    while (todo) {
                        const int j = __builtin_ctzll(todo);
                        todo &= todo - 1;
                        const long long tlo = ((long long)__builtin_amdgcn_readlane(r0.y, j) << 32) |
                                              (uint32_t)__builtin_amdgcn_readlane(r0.x, j);
                        const long long thi = ((long long)__builtin_amdgcn_readlane(r0.w, j) << 32) |
                                              (uint32_t)__builtin_amdgcn_readlane(r0.z, j);
                        const float alo = __int_as_float(__builtin_amdgcn_readlane(r1.x, j));
                        const float ahi = __int_as_float(__builtin_amdgcn_readlane(r1.y, j));
                        const uint32_t qv = (uint32_t)__builtin_amdgcn_readlane(r1.z, j);
                        const int bq0 = __builtin_amdgcn_readlane(r1.w, j);
                        const int32_t own = OWNER ? __builtin_amdgcn_readlane(rown_l, j) : -1;
                        const uint32_t q = qv & ~kQFlags;
                        // keep a pair only in its first common bucket: b == max(bq0, be0),
                        // i.e. bq0 == b (every lane) or be0 == b (mask mb)
                        const bool all_b = (b == kLongBucket) | (bq0 == b);
                        unsigned long long pm[NS];
#pragma unroll
                        for (int k = 0; k < NS; k++) {
                            const Slot &sk = sl[k];
                            // COALESCE'd predicates of operations.go:394-402 (NULL -> sentinels),
                            // each compare straight to a wave mask (no bool -> VGPR -> ballot trip)
                            unsigned long long m = __builtin_amdgcn_sicmpl(sk.t.y, tlo, kCmpSGE) &
                                                   __builtin_amdgcn_sicmpl(sk.t.x, thi, kCmpSLE) &
                                                   __builtin_amdgcn_fcmpf(sk.alt.y, alo, kCmpOGE) &
                                                   __builtin_amdgcn_fcmpf(sk.alt.x, ahi, kCmpOLE);
                            if (OWNER && own >= 0) m &= __builtin_amdgcn_sicmp(sk.own, own, kCmpEQ);
                            pm[k] = all_b ? m : (m & mb[k]);
                        }
                        // At the smallest shared cell only (SQL DISTINCT, Q13): a lane whose
                        // query and entity share a cell < c (near prefix bits overlap, an
                        // exact test) is dropped; with no overlap the lane is kept, which is
                        // exact when either prefix is compact (prefix_sig).
                        if (!(qv & kRank0)) {
                            unsigned long long need[NS], any = 0;
#pragma unroll
                            for (int k = 0; k < NS; k++) {
                                need[k] = pm[k] & ~mf[k];
                                any |= need[k];
                            }
                            if (any) {
                                const int4 c2 = s_sig[w][0][j], c3 = s_sig[w][1][j];
                                const bool qcompact = (qv & kCompact) != 0;
#pragma unroll
                                for (int k = 0; k < NS; k++) {
                                    if (!need[k]) continue;
                                    const Slot &sk = sl[k];
                                    uint32_t acc = (uint32_t)sk.s01.x & (uint32_t)c2.x;
                                    acc |= (uint32_t)(sk.s01.x >> 32) & (uint32_t)c2.y;
                                    acc |= (uint32_t)sk.s01.y & (uint32_t)c2.z;
                                    acc |= (uint32_t)(sk.s01.y >> 32) & (uint32_t)c2.w;
                                    acc |= (uint32_t)sk.s23.x & (uint32_t)c3.x;
                                    acc |= (uint32_t)(sk.s23.x >> 32) & (uint32_t)c3.y;
                                    acc |= (uint32_t)sk.s23.y & (uint32_t)c3.z;
                                    acc |= (uint32_t)(sk.s23.y >> 32) & (uint32_t)c3.w;
                                    const unsigned long long ov = __builtin_amdgcn_uicmp(acc, 0u, kCmpNE);
                                    pm[k] &= ~(need[k] & ov);
                                    // neither prefix compact means both footprints are long:
                                    // those lanes are tagged below, so this merge is a
                                    // safety net only
                                    unsigned long long ex = qcompact ? 0ull : (need[k] & ~ov);
                                    if (ex) ex &= ~__ballot(sk.compact) & ~__ballot(LONG && DSS_JOIN_LONG && sk.lng);
                                    if (ex) {
#if DSS_JOIN_DIAG
                                        if (lane == 0) {  // diagnostics: merges (events, lanes)
                                            atomicAdd(&work[2], 1u);
                                            atomicAdd(&work[3], (uint32_t)__popcll(ex));
                                        }
#endif
                                        bool drop = false;
                                        if ((ex >> lane) & 1ull) {
                                            const uint64_t *qc = a.qv.cells + a.qv.offs[q];
                                            const int64_t nqc = a.qv.offs[q + 1] - a.qv.offs[q];
                                            drop = !no_smaller_shared<2>(ix, sk.ent, cell, qc, nqc);  // rare: few registers
                                        }
                                        pm[k] &= ~__ballot(drop);
                                    }
                                }
                            }
                        }
                        // long query x long entity: every surviving occurrence is emitted
                        // tagged (the smallest shared cell always survives: nothing
                        // smaller is shared) and the tagged set is deduplicated by one
                        // sort after the join; such a pair is never emitted untagged
                        unsigned long long tg[NS];
#pragma unroll
                        for (int k = 0; k < NS; k++) tg[k] = 0ull;
                        if (LONG && DSS_JOIN_LONG && (qv & kLong)) {  // masks built here: rare, keeps SGPRs free in the loop
#pragma unroll
                            for (int k = 0; k < NS; k++) {
                                tg[k] = pm[k] & __ballot(sl[k].lng);
                                pm[k] &= ~tg[k];
                            }
                        }
                        int tot = 0, ttot = 0;
#pragma unroll
                        for (int k = 0; k < NS; k++) {
                            tot += __popcll(pm[k]);
                            ttot += __popcll(tg[k]);
                        }
                        if (tot + ttot == 0) continue;
                        if (staged + tot + ttot > kStage) flush();
#pragma unroll
                        for (int k = 0; k < NS; k++) {
                            if ((pm[k] >> lane) & 1ull) {
                                const int rk = staged + (int)mbcnt64(pm[k]);
                                sp[w][rk] = make_uint2(q, sl[k].ent);
                            }
                            staged += __popcll(pm[k]);
                        }
                        if (ttot) {  // scalar branch: long x long records only
#pragma unroll
                            for (int k = 0; k < NS; k++) {
                                if ((tg[k] >> lane) & 1ull) {
                                    const int rk = staged + (int)mbcnt64(tg[k]);
                                    sp[w][rk] = make_uint2(q | kTag, sl[k].ent);
                                }
                                staged += __popcll(tg[k]);
                            }
                            staged_tag += ttot;
                        }
                    }
                };
#if DSS_JOIN_EXPERIMENT == 2  // timing experiment: units and records loaded, no tests
                if (todo0 == 0x1234567ull) staged += 1;
#else
#if DSS_JOIN_SPECIALISE
                if (nslot == 1) records(std::integral_constant<int, 1>{});
                else records(std::integral_constant<int, kSlots>{});
#else
                records(std::integral_constant<int, kSlots>{});
#endif
#endif
                ci_cur = ci_nx;
            }
        }
        u = un;
    }
    flush();
}

// Tagged (long x long) pairs after the join.  k_tag_split: the join output
// -> untagged pairs compacted into (q2, e2) and tagged ones as keys
// (q << 32 | e), by one scan of the tag flags; k_tag_unique then appends the
// first of each run of the sorted keys after the untagged pairs.
__global__ void k_tag_mark(int64_t n, const uint32_t *q, int64_t *flag)
{
    const int64_t i = tid64();
    if (i < n) flag[i] = (q[i] & kTag) ? 1 : 0;
}
__global__ void k_tag_split(int64_t n, const uint32_t *q, const uint32_t *e, const int64_t *tpos, uint32_t *q2,
                            uint32_t *e2, unsigned long long *tkey)
{
    const int64_t i = tid64();
    if (i >= n) return;
    const uint32_t qq = q[i];
    if (qq & kTag) tkey[tpos[i]] = ((unsigned long long)(qq & ~kTag) << 32) | e[i];
    else {
        q2[i - tpos[i]] = qq;
        e2[i - tpos[i]] = e[i];
    }
}
__global__ void k_tag_flags(int64_t n, const unsigned long long *key, int64_t *flag)
{
    const int64_t i = tid64();
    if (i < n) flag[i] = (i == 0 || key[i] != key[i - 1]) ? 1 : 0;
}
__global__ void k_tag_scatter(int64_t n, const unsigned long long *key, const int64_t *flag, const int64_t *pos,
                              int64_t at, uint32_t *out_q, uint32_t *out_e)
{
    const int64_t i = tid64();
    if (i >= n || !flag[i]) return;
    out_q[at + pos[i]] = (uint32_t)(key[i] >> 32);
    out_e[at + pos[i]] = (uint32_t)key[i];
}

// Roofline accounting over the plain postings, predicate off: M = postings
// scanned query-cell by query-cell, D = pairs surviving the smallest-shared-
// cell rule (= distinct candidate entities per query, summed).
__global__ __launch_bounds__(kBlock) void k_stats(IndexView a, QueryView qv, unsigned long long *stat)
{
    const int lane = threadIdx.x & 63;
    const int64_t q = (int64_t)blockIdx.x * (kBlock / 64) + (threadIdx.x >> 6);
    unsigned long long my_m = 0, my_d = 0;
    if (q < qv.nq) {
        const int64_t c0 = qv.offs[q], c1 = qv.offs[q + 1];
        for (int64_t ci = c0; ci < c1; ci++) {
            const uint64_t c = qv.cells[ci];
            uint32_t slot, s = 0, e = 0;
            if (find_slot(a, c, slot)) plain_range(a, slot, s, e);
            for (uint32_t base = s; base < e; base += 64) {
                const uint32_t p = base + lane;
                bool pass = false;
                if (p < e) {
                    const uint32_t pe = a.p_e[p];
                    pass = ci == c0 || (pe & kFirstBit) ||
                           no_smaller_shared<8>(a, pe & ~kFirstBit, c, qv.cells + c0, ci - c0);
                }
                my_m += (unsigned long long)(e - base < 64 ? e - base : 64);
                my_d += (unsigned long long)__popcll(__ballot(pass));
            }
        }
    }
    if (lane == 0 && (my_m || my_d)) {
        atomicAdd(&stat[0], my_m);
        atomicAdd(&stat[1], my_d);
    }
}

template <typename K, typename V>
void sort_pairs(const K *ki, K *ko, const V *vi, V *vo, int64_t n, int bits, DevBuf<unsigned char> &tmp, hipStream_t s)
{
    radix_sort_pairs(ki, ko, vi, vo, n, bits, tmp, s);  // radix.hip
}

int bits_for(int64_t n)
{
    int b = 1;
    while (b < 63 && ((int64_t)1 << b) <= n) b++;
    return b;
}

int64_t fetch_i64(const int64_t *p, hipStream_t s)
{
    int64_t v = 0;
    DSS_HIP(hipMemcpyAsync(&v, p, sizeof(v), hipMemcpyDeviceToHost, s));
    DSS_HIP(hipStreamSynchronize(s));
    return v;
}

}  // namespace

// ================================================================== build
void SearchEngine::build(dssg_index *idx, int64_t n, const int64_t *cell_offs, const uint64_t *cells,
                         const float *alt_lo, const float *alt_hi, const int64_t *t0, const int64_t *t1,
                         const int32_t *owner, uint64_t cell_lo, uint64_t cell_hi, hipStream_t s)
{
    idx->cell_lo = cell_lo;
    idx->cell_hi = cell_hi;
    idx->n_e = n;
    idx->has_owner = owner != nullptr;
    const int64_t P = fetch_i64(cell_offs + n, s);
    if (P >= (int64_t)0x7fffffff) throw Error(DSSG_ERR_INVALID, "index: more than 2^31 postings per device");
    if (n >= (int64_t)0x7fffffff) throw Error(DSSG_ERR_INVALID, "index: more than 2^31 entities per device");
    const int64_t Pa = P + 1;
    uint64_t *ka = k0_.ensure(Pa), *kb = k1_.ensure(Pa);
    uint32_t *va = v0_.ensure(Pa), *vb = v1_.ensure(Pa);
    if (P) DSS_HIP(hipMemcpyAsync(ka, cells, sizeof(uint64_t) * P, hipMemcpyDeviceToDevice, s));
    if (n) hipLaunchKernelGGL(k_expand, dim3(grid_for(n, kBlock)), dim3(kBlock), 0, s, n, cell_offs, va);
    // (1) plain postings: sort by cell (stable: entity order kept), unique,
    // regular/irregular partition
    sort_pairs(ka, kb, va, vb, P, 64, tmp_, s);
    int64_t *keep = c0_.ensure(3 * Pa), *reg = keep + Pa, *irr = reg + Pa;
    int64_t *kpos = c1_.ensure(3 * (Pa + 1)), *rpos = kpos + (Pa + 1), *ipos = rpos + (Pa + 1);
    if (P)
        hipLaunchKernelGGL(k_keep_flags, dim3(grid_for(P, kBlock)), dim3(kBlock), 0, s, P, kb, vb, cell_lo, cell_hi, keep, reg,
                           irr);
    exclusive_scan_i64(keep, kpos, P, tmp_, s);
    exclusive_scan_i64(reg, rpos, P, tmp_, s);
    exclusive_scan_i64(irr, ipos, P, tmp_, s);
    int64_t counts[3] = {0, 0, 0};
    DSS_HIP(hipMemcpyAsync(&counts[0], kpos + P, sizeof(int64_t), hipMemcpyDeviceToHost, s));
    DSS_HIP(hipMemcpyAsync(&counts[1], rpos + P, sizeof(int64_t), hipMemcpyDeviceToHost, s));
    DSS_HIP(hipMemcpyAsync(&counts[2], ipos + P, sizeof(int64_t), hipMemcpyDeviceToHost, s));
    DSS_HIP(hipStreamSynchronize(s));
    // Pu: unique (cell, entity) postings (entity cell lists, always whole);
    // Pin: those in this index's cell range (the postings it serves)
    const int64_t Pu = counts[0], n_reg = counts[1], n_irr_p = counts[2];
    const int64_t Pin = n_reg + n_irr_p;
    idx->n_p = Pin;
    idx->n_reg = n_reg;
    uint64_t *p_cell = idx->p_cell.ensure(Pin + 1);
    uint32_t *p_e = idx->p_e.ensure(Pin + 1);
    uint32_t *p_mult = idx->p_mult.ensure(Pin + 1);
    if (P)
        hipLaunchKernelGGL(k_scatter_part, dim3(grid_for(P, kBlock)), dim3(kBlock), 0, s, P, kb, vb, reg, rpos, irr, ipos,
                           n_reg, p_cell, p_e, p_mult);
    // (2) entity -> sorted unique cell lists: unique postings in cell order,
    // then a stable sort by entity
    if (P)
        hipLaunchKernelGGL(k_scatter_unique, dim3(grid_for(P, kBlock)), dim3(kBlock), 0, s, P, kb, vb, keep, kpos, ka, va);
    uint64_t *e_cells = idx->e_cells.ensure(Pu + 1);
    sort_pairs(va, vb, ka, e_cells, Pu, 32, tmp_, s);
    DevBuf<unsigned long long> ecnt;
    unsigned long long *ec = ecnt.ensure(n + 2);
    DSS_HIP(hipMemsetAsync(ec, 0, sizeof(unsigned long long) * (n + 2), s));
    if (Pu) hipLaunchKernelGGL(k_count_by_entity, dim3(grid_for(Pu, kBlock)), dim3(kBlock), 0, s, Pu, vb, ec);
    int64_t *ec64 = c0_.ensure(3 * Pa > n + 1 ? 3 * Pa : n + 1);
    if (n) hipLaunchKernelGGL(k_u64_to_i64, dim3(grid_for(n, kBlock)), dim3(kBlock), 0, s, n, ec, ec64);
    int64_t *e_offs = idx->e_offs.ensure(n + 1);
    exclusive_scan_i64(ec64, e_offs, n, tmp_, s);
    unsigned long long *ncell = ec + n + 1;  // scratch counter (zeroed above)
    if (Pin)
        hipLaunchKernelGGL(k_first_flags, dim3(grid_for(Pin, kBlock)), dim3(kBlock), 0, s, Pin, p_cell, p_e, e_offs, e_cells,
                           ncell);
    {
        unsigned long long h = 0;
        DSS_HIP(hipMemcpyAsync(&h, ncell, sizeof(h), hipMemcpyDeviceToHost, s));
        DSS_HIP(hipStreamSynchronize(s));
        idx->n_cells = (int64_t)h;
    }
    // (3) dense lookup over regular postings
    idx->n_dense = 0;
    idx->kmin = 0;
    if (n_reg > 0) {
        uint64_t first = 0, last = 0;
        DSS_HIP(hipMemcpyAsync(&first, p_cell, sizeof(uint64_t), hipMemcpyDeviceToHost, s));
        DSS_HIP(hipMemcpyAsync(&last, p_cell + n_reg - 1, sizeof(uint64_t), hipMemcpyDeviceToHost, s));
        DSS_HIP(hipStreamSynchronize(s));
        idx->kmin = first >> 35;
        idx->n_dense = (int64_t)((last >> 35) - idx->kmin + 1);
        DevBuf<unsigned long long> h;
        unsigned long long *hc = h.ensure(idx->n_dense + 1);
        DSS_HIP(hipMemsetAsync(hc, 0, sizeof(unsigned long long) * (idx->n_dense + 1), s));
        hipLaunchKernelGGL(k_dense_hist, dim3(grid_for(n_reg, kBlock)), dim3(kBlock), 0, s, n_reg, p_cell, idx->kmin, hc);
        DevBuf<int64_t> h64, hs;
        int64_t *a64 = h64.ensure(idx->n_dense + 1), *sc = hs.ensure(idx->n_dense + 2);
        hipLaunchKernelGGL(k_u64_to_i64, dim3(grid_for(idx->n_dense, kBlock)), dim3(kBlock), 0, s, idx->n_dense, hc, a64);
        exclusive_scan_i64(a64, sc, idx->n_dense, tmp_, s);
        uint32_t *dense = idx->dense.ensure(idx->n_dense + 1);
        hipLaunchKernelGGL(k_i64_to_u32, dim3(grid_for(idx->n_dense + 1, kBlock)), dim3(kBlock), 0, s, idx->n_dense + 1, sc,
                           dense);
        DSS_HIP(hipStreamSynchronize(s));
    } else {
        idx->dense.ensure(2);
        DSS_HIP(hipMemsetAsync(idx->dense.p, 0, 2 * sizeof(uint32_t), s));
    }
    // (4) irregular side table
    idx->n_irr = 0;
    if (n_irr_p > 0) {
        DevBuf<int64_t> fl, fp;
        int64_t *f = fl.ensure(n_irr_p + 1), *fpo = fp.ensure(n_irr_p + 2);
        hipLaunchKernelGGL(k_irr_runs, dim3(grid_for(n_irr_p, kBlock)), dim3(kBlock), 0, s, n_irr_p, p_cell + n_reg, f);
        exclusive_scan_i64(f, fpo, n_irr_p, tmp_, s);
        const int64_t nu = fetch_i64(fpo + n_irr_p, s);
        idx->n_irr = nu;
        uint64_t *ic = idx->irr_cells.ensure(nu + 1);
        uint32_t *irr_start = idx->irr_start.ensure(nu + 1);
        hipLaunchKernelGGL(k_irr_scatter, dim3(grid_for(n_irr_p, kBlock)), dim3(kBlock), 0, s, n_irr_p, p_cell + n_reg, f, fpo,
                           n_reg, ic, irr_start);
        uint32_t endv = (uint32_t)Pin;
        DSS_HIP(hipMemcpyAsync(irr_start + nu, &endv, sizeof(uint32_t), hipMemcpyHostToDevice, s));
        DSS_HIP(hipStreamSynchronize(s));
    } else {
        idx->irr_cells.ensure(1);
        idx->irr_start.ensure(1);
    }
    const int64_t n_slots = idx->n_dense + idx->n_irr;
    // (5) time buckets over the span of the rows that can match.  Width: a
    // power of two >= span / kMaxBuckets and ~ the mean row duration (rounded
    // in log2): narrower buckets copy each posting into more buckets (more
    // bytes per join), wider ones put more non-overlapping pairs in a group
    // (more tests); measured on configs[1]: 36 min 2.47 ms, 72 min 2.08 ms,
    // 143 min 2.55 ms per join launch, mean intent duration 62 min.
    {
        DevBuf<unsigned long long> mmb;
        unsigned long long *mm = mmb.ensure(4), hmm[4] = {~0ull, 0ull, 0ull, 0ull};
        double *dsum = (double *)(mm + 3);
        DSS_HIP(hipMemcpyAsync(mm, hmm, sizeof(hmm), hipMemcpyHostToDevice, s));
        if (n) {
            unsigned g = grid_for(n, kBlock);
            hipLaunchKernelGGL(k_time_range, dim3(g < 1024 ? g : 1024), dim3(kBlock), 0, s, n, t0, t1, mm, dsum);
        }
        DSS_HIP(hipMemcpyAsync(hmm, mm, sizeof(hmm), hipMemcpyDeviceToHost, s));
        DSS_HIP(hipStreamSynchronize(s));
        double dur_sum = 0;
        std::memcpy(&dur_sum, &hmm[3], sizeof(double));
        const double mean_dur = hmm[2] ? dur_sum / (double)hmm[2] : 0.0;
        idx->tbase = 0;
        idx->shift = 0;
        idx->nb = 1;
        if (hmm[1] != 0) {  // some row can match
            const long long tmax = (long long)(hmm[1] ^ 0x8000000000000000ull);
            const long long tmin = hmm[0] == ~0ull ? tmax : (long long)(hmm[0] ^ 0x8000000000000000ull);
            const unsigned long long span = tmax > tmin ? (unsigned long long)tmax - (unsigned long long)tmin : 0;
            int sh = 0;
            while ((span >> sh) >= (unsigned long long)kMaxBuckets) sh++;
            if (mean_dur >= 2.0) sh = std::max(sh, std::min(62, (int)std::lround(std::log2(mean_dur))));
            idx->tbase = tmin;
            idx->shift = sh;
            idx->nb = (int)(span >> sh) + 1;
        }
    }
    const Buckets bk{idx->tbase, idx->shift, idx->nb};
    // (6) bucketed postings
    const IndexView pv = view_of(idx);
    DevBuf<uint32_t> ps_buf;
    uint32_t *pslot = ps_buf.ensure(Pin + 1);
    if (Pin) hipLaunchKernelGGL(k_plain_slot, dim3(grid_for(Pin, kBlock)), dim3(kBlock), 0, s, Pin, p_cell, pv, pslot);
    int64_t *bcnt = c0_.ensure(Pin + 1), *boff = c1_.ensure(Pin + 2);
    if (Pin)
        hipLaunchKernelGGL(k_bucket_copies<0>, dim3(grid_for(Pin, kBlock)), dim3(kBlock), 0, s, Pin, p_e, pslot, t0, t1, bk,
                           bcnt, nullptr, nullptr, nullptr);
    exclusive_scan_i64(bcnt, boff, Pin, tmp_, s);
    const int64_t NB = fetch_i64(boff + Pin, s);
    if (NB >= (int64_t)0x7fffffff) throw Error(DSSG_ERR_INVALID, "index: more than 2^31 bucketed postings per device");
    idx->n_b = NB;
    uint64_t *bk0 = k0_.ensure(NB + 1), *bk1 = k1_.ensure(NB + 1);
    uint32_t *bv0 = v0_.ensure(NB + 1), *bv1 = v1_.ensure(NB + 1);
    if (Pin)
        hipLaunchKernelGGL(k_bucket_copies<1>, dim3(grid_for(Pin, kBlock)), dim3(kBlock), 0, s, Pin, p_e, pslot, t0, t1, bk,
                           nullptr, boff, bk0, bv0);
    sort_pairs(bk0, bk1, bv0, bv1, NB, bits_for(n_slots) + 6, tmp_, s);
    uint32_t *b_e = idx->b_e.ensure(NB + 1);
    float2 *b_alt = idx->b_alt.ensure(NB + 1);
    longlong2 *b_t = idx->b_t.ensure(NB + 1);
    uint8_t *b_meta = idx->b_meta.ensure(NB + 1);
    ulonglong2 *b_sig = idx->b_sig.ensure(2 * (NB + 1));
    int32_t *b_owner = idx->b_owner.ensure(owner ? NB + 1 : 1);
    if (NB)
        hipLaunchKernelGGL(k_bucket_gather, dim3(grid_for(NB, kBlock)), dim3(kBlock), 0, s, NB, bv1, p_cell, p_e, e_offs,
                           e_cells, alt_lo, alt_hi, t0, t1, owner, bk, b_e, b_alt, b_t, b_meta, b_sig, b_owner);
    unsigned long long *nlong_d = (unsigned long long *)c1_.ensure(2);
    DSS_HIP(hipMemsetAsync(nlong_d, 0, sizeof(unsigned long long), s));
    if (NB) hipLaunchKernelGGL(k_count_long, dim3(grid_for(NB, kBlock)), dim3(kBlock), 0, s, NB, b_meta, nlong_d);
    unsigned long long nlong_h = 0;
    DSS_HIP(hipMemcpyAsync(&nlong_h, nlong_d, sizeof(nlong_h), hipMemcpyDeviceToHost, s));
    DSS_HIP(hipStreamSynchronize(s));
    idx->n_long_b = (int64_t)nlong_h;
    // (7) groups = runs of equal (slot, bucket)
    unsigned long long *s_mask = idx->s_mask.ensure(n_slots + 1);
    DSS_HIP(hipMemsetAsync(s_mask, 0, sizeof(unsigned long long) * (n_slots + 1), s));
    int64_t ng = 0;
    if (NB) {
        uint64_t *gkey = bk0;  // reuse
        int64_t *gcnt = c0_.ensure(NB + 1), *ngd = c1_.ensure(2);
        size_t bytes = 0;
        DSS_HIP(hipcub::DeviceRunLengthEncode::Encode(nullptr, bytes, bk1, gkey, gcnt, ngd, (int)NB, s));
        tmp_.ensure(bytes + 16);
        DSS_HIP(hipcub::DeviceRunLengthEncode::Encode(tmp_.p, bytes, bk1, gkey, gcnt, ngd, (int)NB, s));
        ng = fetch_i64(ngd, s);
        DevBuf<int64_t> gs;
        int64_t *gst = gs.ensure(ng + 2);
        exclusive_scan_i64(gcnt, gst, ng, tmp_, s);
        uint32_t *bk_start = idx->bk_start.ensure(ng + 1);
        hipLaunchKernelGGL(k_i64_to_u32, dim3(grid_for(ng + 1, kBlock)), dim3(kBlock), 0, s, ng + 1, gst, bk_start);
        hipLaunchKernelGGL(k_group_mask, dim3(grid_for(ng, kBlock)), dim3(kBlock), 0, s, ng, gkey, s_mask);
        uint64_t *g_key = idx->g_key.ensure(ng + 1);
        DSS_HIP(hipMemcpyAsync(g_key, gkey, sizeof(uint64_t) * ng, hipMemcpyDeviceToDevice, s));
        // join-unit bound inputs: posting tiles per group (k_units)
        std::vector<uint32_t> hb((size_t)ng + 1);
        DSS_HIP(hipMemcpyAsync(hb.data(), bk_start, sizeof(uint32_t) * (ng + 1), hipMemcpyDeviceToHost, s));
        DSS_HIP(hipStreamSynchronize(s));
        idx->tiles_total = 0;
        idx->tiles_max = 0;
        for (int64_t g = 0; g < ng; g++) {
            const int64_t np = (int64_t)hb[g + 1] - hb[g];
            const int64_t k = std::min((int64_t)kSlots, std::max((int64_t)1, (np + 63) / 64));
            const int64_t tp = (np + 64 * k - 1) / (64 * k);
            idx->tiles_total += tp;
            idx->tiles_max = std::max(idx->tiles_max, tp);
        }
    } else {
        idx->bk_start.ensure(1);
        DSS_HIP(hipMemsetAsync(idx->bk_start.p, 0, sizeof(uint32_t), s));
        idx->g_key.ensure(1);
        idx->tiles_total = idx->tiles_max = 0;
    }
    idx->n_groups = ng;
    {
        DevBuf<int64_t> pc, po;
        int64_t *pcnt = pc.ensure(n_slots + 1), *poff = po.ensure(n_slots + 2);
        if (n_slots)
            hipLaunchKernelGGL(k_slot_pop, dim3(grid_for(n_slots, kBlock)), dim3(kBlock), 0, s, n_slots, s_mask, pcnt);
        exclusive_scan_i64(pcnt, poff, n_slots, tmp_, s);
        uint32_t *s_base = idx->s_base.ensure(n_slots + 1);
        hipLaunchKernelGGL(k_i64_to_u32, dim3(grid_for(n_slots + 1, kBlock)), dim3(kBlock), 0, s, n_slots + 1, poff, s_base);
        DSS_HIP(hipStreamSynchronize(s));
    }
    // (8) entity-level attributes: ends_at, owner, owner -> entities, counters
    int64_t *et1 = idx->e_t1.ensure(n + 1);
    if (n) DSS_HIP(hipMemcpyAsync(et1, t1, sizeof(int64_t) * n, hipMemcpyDeviceToDevice, s));
    int64_t *notify = idx->e_notify.ensure(n + 1);
    DSS_HIP(hipMemsetAsync(notify, 0, sizeof(int64_t) * (n + 1), s));
    if (owner) {
        int32_t *eo = idx->e_owner.ensure(n + 1);
        if (n) DSS_HIP(hipMemcpyAsync(eo, owner, sizeof(int32_t) * n, hipMemcpyDeviceToDevice, s));
        uint32_t *k0 = v0_.ensure(n + 1), *v0 = v1_.ensure(n + 1);
        uint32_t *ok = idx->o_key.ensure(n + 1), *oe = idx->o_ent.ensure(n + 1);
        if (n) hipLaunchKernelGGL(k_owner_keys, dim3(grid_for(n, kBlock)), dim3(kBlock), 0, s, n, owner, k0, v0);
        sort_pairs(k0, ok, v0, oe, n, 32, tmp_, s);
    }
    DSS_HIP(hipStreamSynchronize(s));
}

// ================================================================== search
void SearchEngine::stats(const dssg_index *idx, int64_t nq, const int64_t *q_offs, const uint64_t *q_cells, hipStream_t s,
                         int64_t *matched, int64_t *distinct)
{
    unsigned long long *cnt = counter_.ensure(4);
    DSS_HIP(hipMemsetAsync(cnt, 0, 4 * sizeof(unsigned long long), s));
    QueryView qv{nq, q_offs, q_cells, nullptr, nullptr, nullptr, nullptr, nullptr};
    if (nq > 0) hipLaunchKernelGGL(k_stats, dim3(grid_for(nq, kBlock / 64)), dim3(kBlock), 0, s, view_of(idx), qv, cnt);
    unsigned long long h[4];
    DSS_HIP(hipMemcpyAsync(h, cnt, sizeof(h), hipMemcpyDeviceToHost, s));
    DSS_HIP(hipStreamSynchronize(s));
    *matched = (int64_t)h[0];
    *distinct = (int64_t)h[1];
}

void SearchEngine::search(const dssg_index *idx, int64_t nq, const int64_t *q_offs, const uint64_t *q_cells,
                          const float *q_alt_lo, const float *q_alt_hi, const int64_t *q_tlo, const int64_t *q_thi,
                          const int32_t *q_owner, hipStream_t s, dssg_pairs *out)
{
    if (q_owner && !idx->has_owner) throw Error(DSSG_ERR_INVALID, "search by owner on an index built without owners");
    if (nq >= (int64_t)kLong) throw Error(DSSG_ERR_INVALID, "search: more than 2^29 queries per batch");
    if (timing_ && !ev0_) {
        DSS_HIP(hipEventCreate(&ev0_));
        DSS_HIP(hipEventCreate(&ev1_));
    }
    const IndexView ix = view_of(idx);
    const QueryView qv{nq, q_offs, q_cells, q_alt_lo, q_alt_hi, q_tlo, q_thi, q_owner};
    auto empty = [&]() {
        out->q = oq_.ensure(1);
        out->e = oe_.ensure(1);
        out->n = 0;
        units_ = keys_ = 0;
        join_ms_ = 0;
    };
    if (nq <= 0 || idx->n_b == 0) return empty();
    const int64_t ng = idx->n_groups;
    // (1) per query cell: group keys + records; the one host sync before the
    // join sizes the key buffers (the radix sort takes a host count)
    int64_t nqc = 0;
    DSS_HIP(hipMemcpyAsync(&nqc, q_offs + nq, sizeof(int64_t), hipMemcpyDeviceToHost, s));
    DSS_HIP(hipStreamSynchronize(s));
    if (nqc >= (int64_t)0xffffffffll) throw Error(DSSG_ERR_CAPACITY, "search: more than 2^32 query cells per batch");
    if (nqc == 0) return empty();
    uint32_t *cq = cq_.ensure(nqc + 1);
    uint32_t *dec = dec_.ensure(nqc + 1);
    int64_t *kcnt = c0_.ensure(nqc + 1), *koff = c1_.ensure(nqc + 2);
    uint8_t *qlong = qlong_.ensure(nq + 1);
    unsigned long long *nlongq_d = counter_.ensure(8) + 5;
    DSS_HIP(hipMemsetAsync(nlongq_d, 0, sizeof(unsigned long long), s));
    hipLaunchKernelGGL(k_cell_query, dim3(grid_for(nq, kBlock)), dim3(kBlock), 0, s, nq, q_offs, q_cells, cq, dec, qlong,
                       nlongq_d);
    hipLaunchKernelGGL(k_qcells<0>, dim3(grid_for(nqc, kBlock)), dim3(kBlock), 0, s, ix, qv, nqc, cq, dec, kcnt, nullptr,
                       nullptr, nullptr, nullptr, nullptr, nullptr);
    exclusive_scan_i64(kcnt, koff, nqc, tmp_, s);
    int64_t nkeys = 0;
    unsigned long long nlongq = 0;
    DSS_HIP(hipMemcpyAsync(&nkeys, koff + nqc, sizeof(nkeys), hipMemcpyDeviceToHost, s));
    DSS_HIP(hipMemcpyAsync(&nlongq, nlongq_d, sizeof(nlongq), hipMemcpyDeviceToHost, s));
    DSS_HIP(hipStreamSynchronize(s));
    keys_ = nkeys;
    long_queries_ = (int64_t)nlongq;
    long_postings_ = idx->n_long_b;
    const bool any_long = nlongq > 0 && idx->n_long_b > 0;  // else no long x long pair exists
    if (nkeys == 0) return empty();
    if (nkeys >= (int64_t)0x7fffffff) throw Error(DSSG_ERR_CAPACITY, "search: more than 2^31 (cell, bucket) keys per batch");
    QRec *recs = (QRec *)rec_.ensure(sizeof(QRec) * (nqc + 1));
    int32_t *rown = q_owner ? (int32_t *)own_.ensure(nqc + 1) : nullptr;
    uint32_t *key = v0_.ensure(nkeys + 1), *skey = v2_.ensure(nkeys + 1);
    uint32_t *val = v1_.ensure(nkeys + 1), *sval = v3_.ensure(nkeys + 1);
    hipLaunchKernelGGL(k_qcells<1>, dim3(grid_for(nqc, kBlock)), dim3(kBlock), 0, s, ix, qv, nqc, cq, dec, nullptr, koff,
                       key, val, recs, rown, (const uint8_t *)qlong);
    // (2) group by group id (radix sort over bits_for(ng) bits), then each
    // group's record range
    sort_pairs(key, skey, val, sval, nkeys, bits_for(ng), tmp_, s);
    uint32_t *gbeg = gb_.ensure(ng + 1), *gend = ge_.ensure(ng + 1);
    DSS_HIP(hipMemsetAsync(gbeg, 0, sizeof(uint32_t) * (ng + 1), s));
    DSS_HIP(hipMemsetAsync(gend, 0, sizeof(uint32_t) * (ng + 1), s));
    hipLaunchKernelGGL(k_gbounds, dim3(grid_for(nkeys, kBlock)), dim3(kBlock), 0, s, nkeys, skey, gbeg, gend);
    // (3) join units over all groups; the total stays on the device.  Bound:
    // each group contributes tiles x ceil(records / kQChunk) units.
    int64_t *ucnt = uc_.ensure(ng + 1), *uoff = uo_.ensure(ng + 2);
    hipLaunchKernelGGL(k_units<0>, dim3(grid_for(ng, kBlock)), dim3(kBlock), 0, s, ng, idx->bk_start.p, gbeg, gend,
                       idx->g_key.p, ucnt, nullptr, nullptr);
    exclusive_scan_i64(ucnt, uoff, ng, tmp_, s);
    const int64_t ubound = idx->tiles_total + (nkeys / kQChunk + 1) * idx->tiles_max;
    if (ubound >= (int64_t)0xffffffffll - kGrab) throw Error(DSSG_ERR_CAPACITY, "search: too many join units");
    UnitDesc *units = (UnitDesc *)units_buf_.ensure(sizeof(UnitDesc) * (ubound + 1));
    hipLaunchKernelGGL(k_units<1>, dim3(grid_for(ng, kBlock)), dim3(kBlock), 0, s, ng, idx->bk_start.p, gbeg, gend,
                       idx->g_key.p, nullptr, uoff, units);
    if (timing_) {
        unsigned long long *st = counter_.ensure(8) + 2;
        DSS_HIP(hipMemsetAsync(st, 0, 3 * sizeof(unsigned long long), s));
        hipLaunchKernelGGL(k_work_stats, dim3(grid_for(ng, kBlock)), dim3(kBlock), 0, s, ng, idx->bk_start.p, gbeg, gend,
                           st);
        unsigned long long h[3];
        int64_t nu = 0;
        DSS_HIP(hipMemcpyAsync(h, st, sizeof(h), hipMemcpyDeviceToHost, s));
        DSS_HIP(hipMemcpyAsync(&nu, uoff + ng, sizeof(nu), hipMemcpyDeviceToHost, s));
        DSS_HIP(hipStreamSynchronize(s));
        iters_ = (int64_t)h[0];
        tests_ = (int64_t)h[1];
        runs_ = (int64_t)h[2];
        units_ = nu;
    }
    // (4) join; grow the output and rerun if the guess was too small
    JoinArgs ja{};
    ja.ix = ix;
    ja.qv = qv;
    ja.nunits = uoff + ng;
    ja.g_key = idx->g_key.p;
    ja.gbeg = gbeg;
    ja.gend = gend;
    if (out_cap_ == 0) out_cap_ = (size_t)nq * 16 + 1024;
    // persistent grid: a few workgroups per CU (LDS-limited), units pulled from a queue
    if (n_cu_ == 0) {
        int dev = 0, ncu = 0;
        DSS_HIP(hipGetDevice(&dev));
        DSS_HIP(hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, dev));
        n_cu_ = ncu > 0 ? ncu : 256;
    }
    const unsigned nblocks = (unsigned)n_cu_ * kJoinBlocksPerCU;
    uint32_t *work = work_.ensure(4);  // [0] unit queue head, [1..3] diagnostics
    unsigned long long *counter = counter_.ensure(2);
    ja.counter = counter;
    for (int attempt = 0; attempt < 3; attempt++) {
        uint32_t *oq = oq_.ensure(out_cap_), *oe = oe_.ensure(out_cap_);
        DSS_HIP(hipMemsetAsync(counter, 0, 2 * sizeof(unsigned long long), s));
        DSS_HIP(hipMemsetAsync(work, 0, 4 * sizeof(uint32_t), s));
        ja.cap = (int64_t)out_cap_;
        if (timing_) DSS_HIP(hipEventRecord(ev0_, s));
        if (nblocks) {
            auto kern = q_owner ? (any_long ? k_join<true, true> : k_join<true, false>)
                                : (any_long ? k_join<false, true> : k_join<false, false>);
            hipLaunchKernelGGL(kern, dim3(nblocks), dim3(64 * kWaves), 0, s, ja, (const QRec *)recs,
                               (const uint32_t *)sval, (const int32_t *)(q_owner ? rown : nullptr),
                               (const UnitDesc *)units, oq, oe, work);
        }
        if (timing_) DSS_HIP(hipEventRecord(ev1_, s));
        unsigned long long tot[2] = {0, 0};
        DSS_HIP(hipMemcpyAsync(tot, counter, sizeof(tot), hipMemcpyDeviceToHost, s));
        DSS_HIP(hipStreamSynchronize(s));
        if (timing_) {
            float ms = 0;
            DSS_HIP(hipEventElapsedTime(&ms, ev0_, ev1_));
            join_ms_ = ms;
            uint32_t hw[4];
            DSS_HIP(hipMemcpy(hw, work, sizeof(hw), hipMemcpyDeviceToHost));
            flushes_ = hw[1];
            merges_ = hw[2];
            merge_lanes_ = hw[3];
        }
        const unsigned long long total = tot[0], ntag = tot[1];
        tagged_ = (int64_t)ntag;
        if (total > out_cap_) {
            out_cap_ = (size_t)(total + total / 8 + 1024);
            continue;
        }
        int64_t nout = (int64_t)total;
        if (ntag > 0) {  // long x long pairs: split off, sort, unique, append
            const int64_t n = (int64_t)total, nt = (int64_t)ntag;
            uint32_t *q2 = oq2_.ensure(out_cap_), *e2 = oe2_.ensure(out_cap_);
            unsigned long long *k1 = tkey_.ensure(nt + 1), *k2 = tkey2_.ensure(nt + 1);
            int64_t *flag = c0_.ensure(n + 1), *pos = c1_.ensure(n + 2);
            hipLaunchKernelGGL(k_tag_mark, dim3(grid_for(n, kBlock)), dim3(kBlock), 0, s, n, oq, flag);
            exclusive_scan_i64(flag, pos, n, tmp_, s);
            hipLaunchKernelGGL(k_tag_split, dim3(grid_for(n, kBlock)), dim3(kBlock), 0, s, n, oq, oe, pos, q2, e2, k1);
            radix_sort_keys(k1, k2, nt, 64, tmp_, s);
            hipLaunchKernelGGL(k_tag_flags, dim3(grid_for(nt, kBlock)), dim3(kBlock), 0, s, nt, k2, flag);
            exclusive_scan_i64(flag, pos, nt, tmp_, s);
            nout = n - nt;
            hipLaunchKernelGGL(k_tag_scatter, dim3(grid_for(nt, kBlock)), dim3(kBlock), 0, s, nt, k2, flag, pos, nout, q2,
                               e2);
            nout += fetch_i64(pos + nt, s);
            out->q = q2;
            out->e = e2;
            out->n = nout;
            return;
        }
        out->q = oq;
        out->e = oe;
        out->n = nout;
        return;
    }
    throw Error(DSSG_ERR_DEVICE, "search: output size did not converge");
}

}  // namespace dss
