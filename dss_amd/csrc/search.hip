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
// Index layout in HBM (built once, resident): postings sorted by
// (cell, entity), structure-of-arrays with the filter attributes inlined
// (entity u32 | alt float2 | time longlong2 = 28 B), so a cell's posting list
// streams with 16-byte coalesced loads.  Level-13 cells are found with one
// dense lookup (slot = cell >> 35, a 29-bit face+Hilbert prefix); any other
// id (the reference tests use invalid face-7 ids as opaque keys, Q12) goes
// through a small sorted side table.
//
// Join: one wavefront per query walks its cells in ascending order; lanes
// stream the cell's postings, apply the fused altitude/time/owner predicate,
// and keep a pair only at the smallest cell the query and the entity share
// (the SQL DISTINCT, Q13, without a dedupe pass; it also lets cell-range
// shards emit disjoint pair sets).  Survivors are staged per wave in LDS and
// flushed with one atomic per batch.
#include <hip/hip_runtime.h>

#include <hipcub/hipcub.hpp>

#include "search.hpp"

namespace dss {
namespace {

constexpr unsigned kBlock = 256;
constexpr uint32_t kFirstBit = 0x80000000u;
constexpr uint64_t kLsb13 = 1ull << 34;

__device__ __forceinline__ int64_t tid64() { return (int64_t)blockIdx.x * blockDim.x + threadIdx.x; }
__host__ __device__ __forceinline__ bool is_regular(uint64_t c)
{
    return (c & ((kLsb13 << 1) - 1)) == kLsb13 && (c >> 61) < 6;  // level 13, valid face
}

__global__ void k_expand(int64_t n, const int64_t *offs, uint32_t *val)
{
    int64_t e = tid64();
    if (e >= n) return;
    for (int64_t k = offs[e]; k < offs[e + 1]; k++) val[k] = (uint32_t)e;
}

__global__ void k_keep_flags(int64_t P, const uint64_t *key, const uint32_t *val, int64_t *keep, int64_t *reg,
                             int64_t *irr)
{
    int64_t i = tid64();
    if (i >= P) return;
    bool k = i == 0 || key[i] != key[i - 1] || val[i] != val[i - 1];
    bool r = is_regular(key[i]);
    keep[i] = k;
    reg[i] = k && r;
    irr[i] = k && !r;
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
                               uint64_t *p_cell, uint32_t *p_e)
{
    int64_t i = tid64();
    if (i >= P) return;
    if (reg[i]) {
        p_cell[rpos[i]] = key[i];
        p_e[rpos[i]] = val[i];
    } else if (irr[i]) {
        p_cell[n_reg + ipos[i]] = key[i];
        p_e[n_reg + ipos[i]] = val[i];
    }
}

__global__ void k_time_keys(int64_t n, const uint32_t *p_e, const int64_t *t0, uint64_t *key, uint32_t *perm)
{
    int64_t i = tid64();
    if (i >= n) return;
    key[i] = (uint64_t)t0[p_e[i]] ^ 0x8000000000000000ull;  // signed order as unsigned
    perm[i] = (uint32_t)i;
}
__global__ void k_gather_cell(int64_t n, const uint64_t *cell, const uint32_t *perm, uint64_t *out)
{
    int64_t i = tid64();
    if (i < n) out[i] = cell[perm[i]];
}
__global__ void k_apply_perm(int64_t n, const uint32_t *perm, const uint64_t *cell_in, const uint32_t *e_in,
                             uint64_t *cell_out, uint32_t *e_out)
{
    int64_t i = tid64();
    if (i >= n) return;
    cell_out[i] = cell_in[perm[i]];
    e_out[i] = e_in[perm[i]];
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

__global__ void k_attrs(int64_t P, const uint64_t *p_cell, uint32_t *p_e, const int64_t *e_offs, const uint64_t *e_cells,
                        const float *alo, const float *ahi, const int64_t *t0, const int64_t *t1, const int32_t *owner,
                        float2 *p_alt, longlong2 *p_t, int32_t *p_owner)
{
    int64_t i = tid64();
    if (i >= P) return;
    uint32_t e = p_e[i];
    bool first = e_cells[e_offs[e]] == p_cell[i];
    p_e[i] = e | (first ? kFirstBit : 0u);
    p_alt[i] = make_float2(alo[e], ahi[e]);
    p_t[i] = make_longlong2(t0[e], t1[e]);
    if (owner) p_owner[i] = owner[e];
}

__global__ void k_dense_hist(int64_t n_reg, const uint64_t *p_cell, uint64_t kmin, unsigned long long *cnt)
{
    int64_t i = tid64();
    if (i < n_reg) atomicAdd(&cnt[(p_cell[i] >> 35) - kmin], 1ull);
}

__global__ void k_i64_to_u32(int64_t n, const int64_t *a, uint32_t *b)
{
    int64_t k = tid64();
    if (k < n) b[k] = (uint32_t)a[k];
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

struct JoinArgs {
    // queries
    int64_t nq;
    const int64_t *q_offs;
    const uint64_t *q_cells;
    const float *q_alo, *q_ahi;
    const int64_t *q_tlo, *q_thi;
    const int32_t *q_owner;
    // index
    const uint32_t *p_e;
    const float2 *p_alt;
    const longlong2 *p_t;
    const int32_t *p_owner;
    const int64_t *e_offs;
    const uint64_t *e_cells;
    uint64_t kmin;
    int64_t n_dense;
    const uint32_t *dense;
    int64_t n_irr;
    const uint64_t *irr_cells;
    const uint32_t *irr_start;
    // output
    uint32_t *out_q, *out_e;
    unsigned long long *counter;
    int64_t cap;
    // stats mode (roofline accounting): predicate off, count postings
    // scanned (M) and canonical survivors (= distinct candidates D)
    int stats;
    unsigned long long *stat_m, *stat_d;
};

__device__ __forceinline__ void lookup(const JoinArgs &a, uint64_t c, uint32_t &s, uint32_t &e)
{
    s = e = 0;
    if (is_regular(c)) {
        uint64_t k = c >> 35;
        if (k >= a.kmin && (int64_t)(k - a.kmin) < a.n_dense) {
            s = a.dense[k - a.kmin];
            e = a.dense[k - a.kmin + 1];
        }
        return;
    }
    int64_t lo = 0, hi = a.n_irr;
    while (lo < hi) {
        int64_t mid = (lo + hi) >> 1;
        if (a.irr_cells[mid] < c) lo = mid + 1;
        else hi = mid;
    }
    if (lo < a.n_irr && a.irr_cells[lo] == c) {
        s = a.irr_start[lo];
        e = a.irr_start[lo + 1];
    }
}

// True iff no cell < c is shared by the query (cells qc[0..nqc), all < c)
// and the entity.
__device__ bool smallest_shared(const JoinArgs &a, uint32_t ent, uint64_t c, const uint64_t *qc, int64_t nqc)
{
    const uint64_t *ec = a.e_cells + a.e_offs[ent];
    int64_t ne = a.e_offs[ent + 1] - a.e_offs[ent];
    int64_t i = 0, j = 0;
    while (i < nqc && j < ne) {
        uint64_t x = qc[i], y = ec[j];
        if (y >= c) break;
        if (x == y) return false;
        if (x < y) i++;
        else j++;
    }
    return true;
}

constexpr int kStage = 256;  // pairs staged per wave in LDS

__global__ __launch_bounds__(kBlock) void k_join(JoinArgs a)
{
    __shared__ uint32_t sq[kBlock / 64][kStage];
    __shared__ uint32_t se[kBlock / 64][kStage];
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    int64_t q = (int64_t)blockIdx.x * (kBlock / 64) + w;
    int staged = 0;
    unsigned long long my_m = 0, my_d = 0;
    auto flush = [&]() {
        unsigned long long base = 0;
        if (lane == 0 && staged) base = atomicAdd(a.counter, (unsigned long long)staged);
        base = __shfl(base, 0);
        for (int k = lane; k < staged; k += 64) {
            unsigned long long o = base + (unsigned long long)k;
            if ((int64_t)o < a.cap) {
                a.out_q[o] = sq[w][k];
                a.out_e[o] = se[w][k];
            }
        }
        staged = 0;
    };
    if (q < a.nq) {
        const int64_t tlo = a.q_tlo[q], thi = a.q_thi[q];
        const float alo = a.q_alo[q], ahi = a.q_ahi[q];
        const int32_t own = a.q_owner ? a.q_owner[q] : -1;
        const int64_t c0 = a.q_offs[q], c1 = a.q_offs[q + 1];
        const uint64_t *qc = a.q_cells + c0;
        for (int64_t ci = c0; ci < c1; ci++) {
            uint64_t c = a.q_cells[ci];
            uint32_t s, e;
            lookup(a, c, s, e);
            for (uint32_t base = s; base < e; base += 64) {
                uint32_t p = base + lane;
                bool pass = false;
                uint32_t ent = 0;
                if (p < e) {
                    uint32_t pe = a.p_e[p];
                    float2 alt = a.p_alt[p];
                    longlong2 t = a.p_t[p];
                    ent = pe & ~kFirstBit;
                    // COALESCE'd predicates of operations.go:394-402 after
                    // the NULL->sentinel mapping (dssgpu.h)
                    pass = a.stats || (t.y >= tlo && t.x <= thi && alt.y >= alo && alt.x <= ahi);
                    if (pass && own >= 0 && !a.stats) pass = a.p_owner[p] == own;
                    if (pass && ci != c0 && !(pe & kFirstBit)) pass = smallest_shared(a, ent, c, qc, ci - c0);
                }
                unsigned long long m = __ballot(pass);
                int nsurv = __popcll(m);
                if (a.stats) {
                    my_m += (unsigned long long)(e - base < 64 ? e - base : 64);
                    my_d += (unsigned long long)nsurv;
                    continue;
                }
                if (nsurv == 0) continue;
                if (staged + nsurv > kStage) flush();
                if (pass) {
                    int r = __popcll(m & ((1ull << lane) - 1ull));
                    sq[w][staged + r] = (uint32_t)q;
                    se[w][staged + r] = ent;
                }
                staged += nsurv;
            }
        }
    }
    if (a.stats) {
        if (lane == 0 && (my_m || my_d)) {
            atomicAdd(a.stat_m, my_m);
            atomicAdd(a.stat_d, my_d);
        }
        return;
    }
    flush();
}


// ---------------------------------------------------------------- tiled join
// The batch's (query, cell) pairs are grouped by index slot (radix sort), and
// each workgroup joins one tile: kTileP postings of one cell (one per lane,
// loaded once) against up to kTileQ of that cell's queries staged in LDS.
__device__ __forceinline__ int s2pos_to_ij(int o, int pos) { return (int)((0x874B78B4u >> (8 * o + 2 * pos)) & 3u); }
__device__ __forceinline__ int s2pos_to_orientation(int pos) { return (int)((0xC1u >> (2 * pos)) & 3u); }
constexpr int kTileP = 256;
constexpr int kTileQ = 256;
constexpr uint32_t kRank0 = 0x80000000u;

// slot of cell c in the index (dense slot, or n_dense + irregular index);
// returns false if the index holds no posting for c.
__device__ __forceinline__ bool cell_slot(const JoinArgs &a, uint64_t c, uint32_t &slot)
{
    if (is_regular(c)) {
        uint64_t k = c >> 35;
        if (k < a.kmin || (int64_t)(k - a.kmin) >= a.n_dense) return false;
        uint32_t sl = (uint32_t)(k - a.kmin);
        if (a.dense[sl + 1] == a.dense[sl]) return false;
        slot = sl;
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
__device__ __forceinline__ void slot_range(const JoinArgs &a, uint32_t slot, uint32_t &s, uint32_t &e, uint64_t &cell)
{
    if ((int64_t)slot < a.n_dense) {
        s = a.dense[slot];
        e = a.dense[slot + 1];
        cell = ((a.kmin + slot) << 35) | kLsb13;
    } else {
        uint32_t k = slot - (uint32_t)a.n_dense;
        s = a.irr_start[k];
        e = a.irr_start[k + 1];
        cell = a.irr_cells[k];
    }
}

template <int PASS>
__global__ void k_qc(JoinArgs a, int64_t *cnt, const int64_t *off, uint32_t *key, uint32_t *val)
{
    int64_t q = tid64();
    if (q >= a.nq) return;
    int64_t c0 = a.q_offs[q], c1 = a.q_offs[q + 1];
    int64_t n = 0, w = PASS ? off[q] : 0;
    for (int64_t k = c0; k < c1; k++) {
        uint32_t slot;
        if (!cell_slot(a, a.q_cells[k], slot)) continue;
        if (PASS) {
            key[w] = slot;
            val[w] = (uint32_t)q | (k == c0 ? kRank0 : 0u);
            w++;
        }
        n++;
    }
    if (!PASS) cnt[q] = n;
}

template <int PASS>
__global__ void k_tiles(int64_t nruns, JoinArgs a, const uint32_t *ukey, const int64_t *rstart, int64_t *cnt,
                        const int64_t *toff, uint32_t *t_run, uint32_t *t_p, uint32_t *t_q)
{
    int64_t r = tid64();
    if (r >= nruns) return;
    uint32_t s, e;
    uint64_t cell;
    slot_range(a, ukey[r], s, e, cell);
    int64_t np = (int64_t)(e - s), nq = rstart[r + 1] - rstart[r];
    int64_t tp = (np + kTileP - 1) / kTileP, tq = (nq + kTileQ - 1) / kTileQ;
    if (!PASS) {
        cnt[r] = tp * tq;
        return;
    }
    int64_t w = toff[r];
    for (int64_t i = 0; i < tp; i++)
        for (int64_t j = 0; j < tq; j++, w++) {
            t_run[w] = (uint32_t)r;
            t_p[w] = (uint32_t)i;
            t_q[w] = (uint32_t)j;
        }
}

struct QAttr {
    int64_t tlo, thi;
    float alo, ahi;
    uint32_t qv;  // query id | kRank0 if the cell is the query's first cell
    int32_t own;  // owner filter, or -1; bit 30 of `compact` below
};

// True iff q and entity `ent` share no cell smaller than c (both lists sorted).
__device__ bool smallest_shared_q(const JoinArgs &a, uint32_t ent, uint64_t c, uint32_t q)
{
    const uint64_t *ec = a.e_cells + a.e_offs[ent];
    int64_t ne = a.e_offs[ent + 1] - a.e_offs[ent];
    const uint64_t *qc = a.q_cells + a.q_offs[q];
    int64_t nq = a.q_offs[q + 1] - a.q_offs[q];
    int64_t i = 0, j = 0;
    while (i < nq && j < ne) {
        uint64_t x = qc[i], y = ec[j];
        if (x >= c || y >= c) break;
        if (x == y) return false;
        if (x < y) i++;
        else j++;
    }
    return true;
}

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

// Prefix signature of a sorted cell list: one bit per (i mod 16, j mod 16)
// (256 bits) for every cell < c; `compact` iff all of them lie within +-7
// cells of c on c's face, so that equal bits imply equal cells.
struct Sig256 {
    uint64_t w[4];
};
__device__ __forceinline__ void prefix_sig(const uint64_t *cells, int64_t n, uint64_t c, int fc, int ic, int jc,
                                           bool cvalid, Sig256 &sig, bool &compact)
{
    sig.w[0] = sig.w[1] = sig.w[2] = sig.w[3] = 0;
    compact = cvalid;
    for (int64_t k = 0; k < n; k++) {
        uint64_t x = cells[k];
        if (x >= c) break;
        int f, i, j;
        if (decode13(x, f, i, j)) {
            int b = ((i & 15) << 4) | (j & 15);
            uint64_t bit = 1ull << (b & 63);
            int wi = b >> 6;
            sig.w[0] |= wi == 0 ? bit : 0;
            sig.w[1] |= wi == 1 ? bit : 0;
            sig.w[2] |= wi == 2 ? bit : 0;
            sig.w[3] |= wi == 3 ? bit : 0;
            int di = i - ic, dj = j - jc;
            if (f != fc || di < -7 || di > 7 || dj < -7 || dj > 7) compact = false;
        } else {
            sig.w[0] = sig.w[1] = sig.w[2] = sig.w[3] = ~0ull;  // unknown position: force the exact check
            compact = false;
        }
    }
}
__device__ __forceinline__ bool sig_overlap(const Sig256 &a, const uint64_t *b)
{
    return ((a.w[0] & b[0]) | (a.w[1] & b[1]) | (a.w[2] & b[2]) | (a.w[3] & b[3])) != 0;
}

__global__ __launch_bounds__(kTileP) void k_join_tile(JoinArgs a, const uint32_t *ukey, const int64_t *rstart,
                                                      const uint32_t *sval, const uint32_t *t_run, const uint32_t *t_p,
                                                      const uint32_t *t_q)
{
    __shared__ QAttr sq_attr[kTileQ];
    __shared__ uint64_t sq_sig[kTileQ][4];
    __shared__ uint8_t sq_compact[kTileQ];
    __shared__ uint32_t sq[kTileP / 64][kStage];
    __shared__ uint32_t se[kTileP / 64][kStage];
    const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
    const uint32_t r = t_run[blockIdx.x];
    uint32_t ps, pe;
    uint64_t cell;
    slot_range(a, ukey[r], ps, pe, cell);
    const int64_t q0 = rstart[r] + (int64_t)t_q[blockIdx.x] * kTileQ;
    const int64_t q1 = min(rstart[r + 1], q0 + kTileQ);
    const int nqt = (int)(q1 - q0);
    int fc = 0, ic = 0, jc = 0;
    const bool cvalid = decode13(cell, fc, ic, jc);
    if (tid < nqt) {
        uint32_t v = sval[q0 + tid];
        uint32_t q = v & ~kRank0;
        QAttr qa;
        qa.tlo = a.q_tlo[q];
        qa.thi = a.q_thi[q];
        qa.alo = a.q_alo[q];
        qa.ahi = a.q_ahi[q];
        qa.qv = v;
        qa.own = a.q_owner ? a.q_owner[q] : -1;
        bool cp;
        Sig256 qs;
        prefix_sig(a.q_cells + a.q_offs[q], a.q_offs[q + 1] - a.q_offs[q], cell, fc, ic, jc, cvalid, qs, cp);
        sq_attr[tid] = qa;
        sq_sig[tid][0] = qs.w[0];
        sq_sig[tid][1] = qs.w[1];
        sq_sig[tid][2] = qs.w[2];
        sq_sig[tid][3] = qs.w[3];
        sq_compact[tid] = cp ? 1 : 0;
    }
    const uint32_t p = ps + t_p[blockIdx.x] * kTileP + tid;
    const bool valid = p < pe;
    uint32_t pev = 0;
    float2 alt = make_float2(0.f, 0.f);
    longlong2 t = make_longlong2(0, 0);
    int32_t pown = 0;
    if (valid) {
        pev = a.p_e[p];
        alt = a.p_alt[p];
        t = a.p_t[p];
        if (a.q_owner) pown = a.p_owner[p];
    }
    const uint32_t ent = pev & ~kFirstBit;
    const bool efirst = (pev & kFirstBit) != 0;
    // time bounds of this posting tile (postings are ordered by start time
    // within a cell): queries whose window misses them are skipped whole
    __shared__ long long s_tmin[kTileP / 64], s_tmax[kTileP / 64];
    {
        long long mn = valid ? t.x : LLONG_MAX, mx = valid ? t.y : LLONG_MIN;
        for (int o = 32; o > 0; o >>= 1) {
            mn = min(mn, __shfl_xor(mn, o));
            mx = max(mx, __shfl_xor(mx, o));
        }
        if (lane == 0) {
            s_tmin[w] = mn;
            s_tmax[w] = mx;
        }
    }
    Sig256 esig;
    esig.w[0] = esig.w[1] = esig.w[2] = esig.w[3] = 0;
    bool ecompact = true;
    if (valid && !efirst)
        prefix_sig(a.e_cells + a.e_offs[ent], a.e_offs[ent + 1] - a.e_offs[ent], cell, fc, ic, jc, cvalid, esig, ecompact);
    __syncthreads();
    long long tmin = s_tmin[0], tmax = s_tmax[0];
#pragma unroll
    for (int k = 1; k < kTileP / 64; k++) {
        tmin = min(tmin, s_tmin[k]);
        tmax = max(tmax, s_tmax[k]);
    }
    int staged = 0;
    auto flush = [&]() {
        __builtin_amdgcn_wave_barrier();
        unsigned long long base = 0;
        if (lane == 0 && staged) base = atomicAdd(a.counter, (unsigned long long)staged);
        base = __shfl(base, 0);
        for (int k = lane; k < staged; k += 64) {
            unsigned long long o = base + (unsigned long long)k;
            if ((int64_t)o < a.cap) {
                a.out_q[o] = sq[w][k];
                a.out_e[o] = se[w][k];
            }
        }
        staged = 0;
        __builtin_amdgcn_wave_barrier();
    };
    for (int k = 0; k < nqt; k++) {
        const QAttr qa = sq_attr[k];
        if (qa.thi < tmin || qa.tlo > tmax) continue;  // no posting of the tile can match
        // COALESCE'd predicates of operations.go:394-402 (NULL -> sentinels)
        bool pass = valid && t.y >= qa.tlo && t.x <= qa.thi && alt.y >= qa.alo && alt.x <= qa.ahi;
        if (qa.own >= 0) pass = pass && pown == qa.own;
        // keep the pair only at the smallest shared cell (SQL DISTINCT, Q13)
        if (pass && !efirst && !(qa.qv & kRank0) && sig_overlap(esig, sq_sig[k])) {
            if (ecompact && sq_compact[k]) pass = false;  // a shared smaller cell exists
            else pass = smallest_shared_q(a, ent, cell, qa.qv & ~kRank0);
        }
        unsigned long long m = __ballot(pass);
        if (m == 0) continue;
        int nsurv = __popcll(m);
        if (staged + nsurv > kStage) flush();
        if (pass) {
            int rk = __popcll(m & ((1ull << lane) - 1ull));
            sq[w][staged + rk] = qa.qv & ~kRank0;
            se[w][staged + rk] = ent;
        }
        staged += nsurv;
    }
    flush();
}

}  // namespace

// ---------------------------------------------------------------- build
void SearchEngine::build(dssg_index *idx, int64_t n, const int64_t *cell_offs, const uint64_t *cells,
                         const float *alt_lo, const float *alt_hi, const int64_t *t0, const int64_t *t1,
                         const int32_t *owner, hipStream_t s)
{
    idx->n_e = n;
    idx->has_owner = owner != nullptr;
    int64_t P = 0;
    DSS_HIP(hipMemcpyAsync(&P, cell_offs + n, sizeof(int64_t), hipMemcpyDeviceToHost, s));
    DSS_HIP(hipStreamSynchronize(s));
    if (P >= (int64_t)0x7fffffff) throw Error(DSSG_ERR_INVALID, "index: more than 2^31 postings per device");
    if (n >= (int64_t)0x7fffffff) throw Error(DSSG_ERR_INVALID, "index: more than 2^31 entities per device");
    const int64_t Pa = P + 1;
    uint64_t *ka = k0_.ensure(Pa), *kb = k1_.ensure(Pa);
    uint32_t *va = v0_.ensure(Pa), *vb = v1_.ensure(Pa);
    DSS_HIP(hipMemcpyAsync(ka, cells, sizeof(uint64_t) * P, hipMemcpyDeviceToDevice, s));
    if (n) hipLaunchKernelGGL(k_expand, dim3(grid_for(n, kBlock)), dim3(kBlock), 0, s, n, cell_offs, va);
    // sort postings by cell (stable: entity order preserved within a cell)
    size_t bytes = 0;
    if (P) {
        DSS_HIP(hipcub::DeviceRadixSort::SortPairs(nullptr, bytes, ka, kb, va, vb, (int)P, 0, 64, s));
        tmp_.ensure(bytes + 16);
        DSS_HIP(hipcub::DeviceRadixSort::SortPairs(tmp_.p, bytes, ka, kb, va, vb, (int)P, 0, 64, s));
    }
    // unique (cell, entity) + regular/irregular partition
    int64_t *keep = c0_.ensure(3 * Pa), *reg = keep + Pa, *irr = reg + Pa;
    int64_t *kpos = c1_.ensure(3 * (Pa + 1)), *rpos = kpos + (Pa + 1), *ipos = rpos + (Pa + 1);
    if (P) hipLaunchKernelGGL(k_keep_flags, dim3(grid_for(P, kBlock)), dim3(kBlock), 0, s, P, kb, vb, keep, reg, irr);
    exclusive_scan_i64(keep, kpos, P, tmp_, s);
    exclusive_scan_i64(reg, rpos, P, tmp_, s);
    exclusive_scan_i64(irr, ipos, P, tmp_, s);
    int64_t counts[3] = {0, 0, 0};
    DSS_HIP(hipMemcpyAsync(&counts[0], kpos + P, sizeof(int64_t), hipMemcpyDeviceToHost, s));
    DSS_HIP(hipMemcpyAsync(&counts[1], rpos + P, sizeof(int64_t), hipMemcpyDeviceToHost, s));
    DSS_HIP(hipMemcpyAsync(&counts[2], ipos + P, sizeof(int64_t), hipMemcpyDeviceToHost, s));
    DSS_HIP(hipStreamSynchronize(s));
    const int64_t Pu = counts[0], n_reg = counts[1], n_irr_p = counts[2];
    idx->n_p = Pu;
    idx->n_reg = n_reg;
    uint64_t *p_cell = idx->p_cell.ensure(Pu + 1);
    uint32_t *p_e = idx->p_e.ensure(Pu + 1);
    if (P)
        hipLaunchKernelGGL(k_scatter_part, dim3(grid_for(P, kBlock)), dim3(kBlock), 0, s, P, kb, vb, reg, rpos, irr, ipos,
                           n_reg, p_cell, p_e);
    // within each cell, order postings by start time (segments sorted apart
    // so regular postings stay in front): sort by t0, then stable by cell
    {
        DevBuf<uint64_t> tk, tk2, cb;
        DevBuf<uint32_t> pm, pm2;
        DevBuf<uint64_t> pc2;
        DevBuf<uint32_t> pe2;
        uint64_t *tkey = tk.ensure(Pu + 1), *tkey2 = tk2.ensure(Pu + 1), *cbuf = cb.ensure(Pu + 1), *pcn = pc2.ensure(Pu + 1);
        uint32_t *perm = pm.ensure(Pu + 1), *perm2 = pm2.ensure(Pu + 1), *pen = pe2.ensure(Pu + 1);
        int64_t segs[2][2] = {{0, n_reg}, {n_reg, Pu}};
        for (auto &sg : segs) {
            int64_t o = sg[0], m = sg[1] - sg[0];
            if (m <= 1) {
                if (m == 1) {
                    DSS_HIP(hipMemcpyAsync(pcn + o, p_cell + o, sizeof(uint64_t), hipMemcpyDeviceToDevice, s));
                    DSS_HIP(hipMemcpyAsync(pen + o, p_e + o, sizeof(uint32_t), hipMemcpyDeviceToDevice, s));
                }
                continue;
            }
            hipLaunchKernelGGL(k_time_keys, dim3(grid_for(m, kBlock)), dim3(kBlock), 0, s, m, p_e + o, t0, tkey, perm);
            size_t b2 = 0;
            DSS_HIP(hipcub::DeviceRadixSort::SortPairs(nullptr, b2, tkey, tkey2, perm, perm2, (int)m, 0, 64, s));
            tmp_.ensure(b2 + 16);
            DSS_HIP(hipcub::DeviceRadixSort::SortPairs(tmp_.p, b2, tkey, tkey2, perm, perm2, (int)m, 0, 64, s));
            hipLaunchKernelGGL(k_gather_cell, dim3(grid_for(m, kBlock)), dim3(kBlock), 0, s, m, p_cell + o, perm2, cbuf);
            b2 = 0;
            DSS_HIP(hipcub::DeviceRadixSort::SortPairs(nullptr, b2, cbuf, tkey, perm2, perm, (int)m, 0, 64, s));
            tmp_.ensure(b2 + 16);
            DSS_HIP(hipcub::DeviceRadixSort::SortPairs(tmp_.p, b2, cbuf, tkey, perm2, perm, (int)m, 0, 64, s));
            hipLaunchKernelGGL(k_apply_perm, dim3(grid_for(m, kBlock)), dim3(kBlock), 0, s, m, perm, p_cell + o, p_e + o,
                               pcn + o, pen + o);
        }
        DSS_HIP(hipMemcpyAsync(p_cell, pcn, sizeof(uint64_t) * Pu, hipMemcpyDeviceToDevice, s));
        DSS_HIP(hipMemcpyAsync(p_e, pen, sizeof(uint32_t) * Pu, hipMemcpyDeviceToDevice, s));
        DSS_HIP(hipStreamSynchronize(s));
    }
    // entity -> sorted unique cell lists: unique postings in cell order, then
    // a stable sort by entity.
    if (P)
        hipLaunchKernelGGL(k_scatter_unique, dim3(grid_for(P, kBlock)), dim3(kBlock), 0, s, P, kb, vb, keep, kpos, ka, va);
    uint64_t *e_cells = idx->e_cells.ensure(Pu + 1);
    uint32_t *vsorted = vb;
    if (Pu) {
        bytes = 0;
        DSS_HIP(hipcub::DeviceRadixSort::SortPairs(nullptr, bytes, va, vb, ka, e_cells, (int)Pu, 0, 32, s));
        tmp_.ensure(bytes + 16);
        DSS_HIP(hipcub::DeviceRadixSort::SortPairs(tmp_.p, bytes, va, vb, ka, e_cells, (int)Pu, 0, 32, s));
    }
    DevBuf<unsigned long long> ecnt;
    unsigned long long *ec = ecnt.ensure(n + 1);
    DSS_HIP(hipMemsetAsync(ec, 0, sizeof(unsigned long long) * (n + 1), s));
    if (Pu) hipLaunchKernelGGL(k_count_by_entity, dim3(grid_for(Pu, kBlock)), dim3(kBlock), 0, s, Pu, vsorted, ec);
    int64_t *ec64 = c0_.ensure(3 * Pa > n + 1 ? 3 * Pa : n + 1);
    if (n) hipLaunchKernelGGL(k_u64_to_i64, dim3(grid_for(n, kBlock)), dim3(kBlock), 0, s, n, ec, ec64);
    int64_t *e_offs = idx->e_offs.ensure(n + 1);
    exclusive_scan_i64(ec64, e_offs, n, tmp_, s);
    // inline attributes + first-cell flag
    float2 *p_alt = idx->p_alt.ensure(Pu + 1);
    longlong2 *p_t = idx->p_t.ensure(Pu + 1);
    int32_t *p_owner = idx->p_owner.ensure(Pu + 1);
    if (Pu)
        hipLaunchKernelGGL(k_attrs, dim3(grid_for(Pu, kBlock)), dim3(kBlock), 0, s, Pu, p_cell, p_e, e_offs, e_cells,
                           alt_lo, alt_hi, t0, t1, owner, p_alt, p_t, p_owner);
    // dense lookup over regular postings
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
    // irregular side table
    idx->n_irr = 0;
    uint32_t *irr_start = nullptr;
    if (n_irr_p > 0) {
        DevBuf<int64_t> fl, fp;
        int64_t *f = fl.ensure(n_irr_p + 1), *fpo = fp.ensure(n_irr_p + 2);
        hipLaunchKernelGGL(k_irr_runs, dim3(grid_for(n_irr_p, kBlock)), dim3(kBlock), 0, s, n_irr_p, p_cell + n_reg, f);
        exclusive_scan_i64(f, fpo, n_irr_p, tmp_, s);
        int64_t nu = 0;
        DSS_HIP(hipMemcpyAsync(&nu, fpo + n_irr_p, sizeof(int64_t), hipMemcpyDeviceToHost, s));
        DSS_HIP(hipStreamSynchronize(s));
        idx->n_irr = nu;
        uint64_t *ic = idx->irr_cells.ensure(nu + 1);
        irr_start = idx->irr_start.ensure(nu + 1);
        hipLaunchKernelGGL(k_irr_scatter, dim3(grid_for(n_irr_p, kBlock)), dim3(kBlock), 0, s, n_irr_p, p_cell + n_reg, f, fpo,
                           n_reg, ic, irr_start);
        uint32_t endv = (uint32_t)Pu;
        DSS_HIP(hipMemcpyAsync(irr_start + nu, &endv, sizeof(uint32_t), hipMemcpyHostToDevice, s));
    } else {
        idx->irr_cells.ensure(1);
        idx->irr_start.ensure(1);
    }
    DSS_HIP(hipStreamSynchronize(s));
}

// ---------------------------------------------------------------- search
static JoinArgs make_args(const dssg_index *idx, int64_t nq, const int64_t *q_offs, const uint64_t *q_cells,
                          const float *q_alt_lo, const float *q_alt_hi, const int64_t *q_tlo, const int64_t *q_thi,
                          const int32_t *q_owner)
{
    JoinArgs a{};
    a.nq = nq; a.q_offs = q_offs; a.q_cells = q_cells; a.q_alo = q_alt_lo; a.q_ahi = q_alt_hi;
    a.q_tlo = q_tlo; a.q_thi = q_thi; a.q_owner = q_owner;
    a.p_e = idx->p_e.p; a.p_alt = idx->p_alt.p; a.p_t = idx->p_t.p; a.p_owner = idx->p_owner.p;
    a.e_offs = idx->e_offs.p; a.e_cells = idx->e_cells.p;
    a.kmin = idx->kmin; a.n_dense = idx->n_dense; a.dense = idx->dense.p;
    a.n_irr = idx->n_irr; a.irr_cells = idx->irr_cells.p; a.irr_start = idx->irr_start.p;
    return a;
}

void SearchEngine::stats(const dssg_index *idx, int64_t nq, const int64_t *q_offs, const uint64_t *q_cells, hipStream_t s,
                         int64_t *matched, int64_t *distinct)
{
    unsigned long long *cnt = counter_.ensure(4);
    DSS_HIP(hipMemsetAsync(cnt, 0, 4 * sizeof(unsigned long long), s));
    JoinArgs a = make_args(idx, nq, q_offs, q_cells, nullptr, nullptr, nullptr, nullptr, nullptr);
    // the predicate reads are skipped in stats mode; give the kernel valid
    // (unused) query attribute pointers anyway
    DevBuf<float> fz;
    DevBuf<int64_t> iz;
    float *f = fz.ensure(nq + 1);
    int64_t *t = iz.ensure(nq + 1);
    DSS_HIP(hipMemsetAsync(f, 0, sizeof(float) * (nq + 1), s));
    DSS_HIP(hipMemsetAsync(t, 0, sizeof(int64_t) * (nq + 1), s));
    a.q_alo = f; a.q_ahi = f; a.q_tlo = t; a.q_thi = t;
    a.stats = 1;
    a.stat_m = cnt + 1;
    a.stat_d = cnt + 2;
    a.counter = cnt;
    if (nq > 0) hipLaunchKernelGGL(k_join, dim3(grid_for(nq, kBlock / 64)), dim3(kBlock), 0, s, a);
    unsigned long long h[4];
    DSS_HIP(hipMemcpyAsync(h, cnt, sizeof(h), hipMemcpyDeviceToHost, s));
    DSS_HIP(hipStreamSynchronize(s));
    *matched = (int64_t)h[1];
    *distinct = (int64_t)h[2];
}

void SearchEngine::search(const dssg_index *idx, int64_t nq, const int64_t *q_offs, const uint64_t *q_cells,
                          const float *q_alt_lo, const float *q_alt_hi, const int64_t *q_tlo, const int64_t *q_thi,
                          const int32_t *q_owner, hipStream_t s, dssg_pairs *out)
{
    if (q_owner && !idx->has_owner) throw Error(DSSG_ERR_INVALID, "search by owner on an index built without owners");
    unsigned long long *counter = counter_.ensure(1);
    JoinArgs a = make_args(idx, nq, q_offs, q_cells, q_alt_lo, q_alt_hi, q_tlo, q_thi, q_owner);
    if (timing_) {
        if (!ev0_) { DSS_HIP(hipEventCreate(&ev0_)); DSS_HIP(hipEventCreate(&ev1_)); }
    }
    // (1) (slot, query) pairs for every query cell that has postings
    int64_t *qcnt = c0_.ensure(nq + 1), *qoff = c1_.ensure(nq + 2);
    if (nq > 0) hipLaunchKernelGGL(k_qc<0>, dim3(grid_for(nq, kBlock)), dim3(kBlock), 0, s, a, qcnt, nullptr, nullptr, nullptr);
    exclusive_scan_i64(qcnt, qoff, nq, tmp_, s);
    int64_t npairs = 0;
    DSS_HIP(hipMemcpyAsync(&npairs, qoff + nq, sizeof(int64_t), hipMemcpyDeviceToHost, s));
    DSS_HIP(hipStreamSynchronize(s));
    if (npairs == 0) {
        out->q = oq_.ensure(1);
        out->e = oe_.ensure(1);
        out->n = 0;
        return;
    }
    uint32_t *key = v0_.ensure(npairs + 1), *val = v1_.ensure(npairs + 1);
    uint32_t *skey = sk_.ensure(npairs + 1), *sval = sv_.ensure(npairs + 1);
    hipLaunchKernelGGL(k_qc<1>, dim3(grid_for(nq, kBlock)), dim3(kBlock), 0, s, a, nullptr, qoff, key, val);
    // (2) group by slot (stable: query order kept within a slot)
    int64_t nslots = idx->n_dense + idx->n_irr;
    int bits = 1;
    while (bits < 32 && ((int64_t)1 << bits) <= nslots) bits++;
    size_t bytes = 0;
    DSS_HIP(hipcub::DeviceRadixSort::SortPairs(nullptr, bytes, key, skey, val, sval, (int)npairs, 0, bits, s));
    tmp_.ensure(bytes + 16);
    DSS_HIP(hipcub::DeviceRadixSort::SortPairs(tmp_.p, bytes, key, skey, val, sval, (int)npairs, 0, bits, s));
    // (3) runs of equal slots
    uint32_t *ukey = uk_.ensure(npairs + 1);
    int64_t *rcnt = rc_.ensure(npairs + 1), *rstart = rs_.ensure(npairs + 2);
    int64_t *nruns_d = nr_.ensure(2);
    bytes = 0;
    DSS_HIP(hipcub::DeviceRunLengthEncode::Encode(nullptr, bytes, skey, ukey, rcnt, nruns_d, (int)npairs, s));
    tmp_.ensure(bytes + 16);
    DSS_HIP(hipcub::DeviceRunLengthEncode::Encode(tmp_.p, bytes, skey, ukey, rcnt, nruns_d, (int)npairs, s));
    int64_t nruns = 0;
    DSS_HIP(hipMemcpyAsync(&nruns, nruns_d, sizeof(int64_t), hipMemcpyDeviceToHost, s));
    DSS_HIP(hipStreamSynchronize(s));
    exclusive_scan_i64(rcnt, rstart, nruns, tmp_, s);
    // (4) tiles
    int64_t *tcnt = tc_.ensure(nruns + 1), *toff = to_.ensure(nruns + 2);
    hipLaunchKernelGGL(k_tiles<0>, dim3(grid_for(nruns, kBlock)), dim3(kBlock), 0, s, nruns, a, ukey, rstart, tcnt, nullptr,
                       nullptr, nullptr, nullptr);
    exclusive_scan_i64(tcnt, toff, nruns, tmp_, s);
    int64_t ntiles = 0;
    DSS_HIP(hipMemcpyAsync(&ntiles, toff + nruns, sizeof(int64_t), hipMemcpyDeviceToHost, s));
    DSS_HIP(hipStreamSynchronize(s));
    uint32_t *t_run = tr_.ensure(ntiles + 1), *t_p = tp_.ensure(ntiles + 1), *t_q = tq_.ensure(ntiles + 1);
    hipLaunchKernelGGL(k_tiles<1>, dim3(grid_for(nruns, kBlock)), dim3(kBlock), 0, s, nruns, a, ukey, rstart, nullptr, toff,
                       t_run, t_p, t_q);
    // (5) join tiles; grow the output and rerun if the guess was too small
    if (out_cap_ == 0) out_cap_ = (size_t)(nq > 0 ? nq : 1) * 16 + 1024;
    for (int attempt = 0; attempt < 3; attempt++) {
        uint32_t *oq = oq_.ensure(out_cap_), *oe = oe_.ensure(out_cap_);
        DSS_HIP(hipMemsetAsync(counter, 0, sizeof(unsigned long long), s));
        a.out_q = oq;
        a.out_e = oe;
        a.counter = counter;
        a.cap = (int64_t)out_cap_;
        if (timing_) DSS_HIP(hipEventRecord(ev0_, s));
        hipLaunchKernelGGL(k_join_tile, dim3((unsigned)ntiles), dim3(kTileP), 0, s, a, ukey, rstart, sval, t_run, t_p, t_q);
        if (timing_) DSS_HIP(hipEventRecord(ev1_, s));
        unsigned long long total = 0;
        DSS_HIP(hipMemcpyAsync(&total, counter, sizeof(total), hipMemcpyDeviceToHost, s));
        DSS_HIP(hipStreamSynchronize(s));
        if (timing_) {
            float ms = 0;
            DSS_HIP(hipEventElapsedTime(&ms, ev0_, ev1_));
            join_ms_ = ms;
        }
        if (total <= out_cap_) {
            out->q = oq;
            out->e = oe;
            out->n = (int64_t)total;
            return;
        }
        out_cap_ = (size_t)(total + total / 8 + 1024);
    }
    throw Error(DSSG_ERR_DEVICE, "search: output size did not converge");
}

}  // namespace dss
