// Cell-range shard routing on gfx950.
//
// The reference partitions its postings table scd_cells_operations by
// cell_id range inside CockroachDB (pkg/scd/store/cockroach/store.go:140-147)
// and lets the SQL layer fan a query out to the ranges its cells hit.  Here
// the fan-out is explicit, one process per GPU:
//
//   home rank:  covered query batch --k_route<0>/k_route<1>--> one send
//               buffer of part-major segments, each [rows | cells] (one
//               32-byte row per (query, shard that owns >= 1 of its cells),
//               then those queries' whole cell lists, padded to 32 bytes):
//               one all-to-all carries both;
//   exchange:   all-to-all (RCCL over xGMI; dss_amd/shard.py);
//   shard:      k_unpack_rows + k_gather_cells -> a plain query batch for
//               dssg_search_device against the shard's cell-range index;
//   shard:      k_route_pairs<0>/<1> -> the pair set by the query's home
//               rank: the shard's own queries' pairs straight into its
//               output arrays, the others part-major, packed
//               (home-local query << 32 | entity);
//   exchange:   all-to-all back; each home rank holds its queries' pairs.
//
// A shard receives a query's WHOLE cell list, and the shard index keeps every
// entity's whole cell list, so the smallest-shared-cell rule of the join
// emits each (query, entity) pair on exactly one shard: no cross-shard dedupe.
//
// Slots inside a destination segment come from one 64-bit atomic per wave and
// destination, packing (rows << 40 | cells): a segment's cell lists are laid
// out in the order of its rows, which is all the receiver needs to rebuild
// the CSR offsets.  Row order within a segment is unspecified (result sets
// are unordered, quirk Q13).
#include <hip/hip_runtime.h>

#include <algorithm>

#include "route.hpp"

namespace dss {
namespace {

constexpr unsigned kBlock = 256;
constexpr int kCellBits = 40;
constexpr unsigned long long kCellMask = (1ull << kCellBits) - 1ull;

__device__ __forceinline__ int64_t tid64() { return (int64_t)blockIdx.x * blockDim.x + threadIdx.x; }

// First part r with c <= hi[r] (hi ascending, hi[np-1] = UINT64_MAX).
__device__ __forceinline__ int part_of(uint64_t c, const uint64_t *hi, int np)
{
    int lo = 0, h = np - 1;
    while (lo < h) {
        const int m = (lo + h) >> 1;
        if (c <= hi[m]) h = m;
        else lo = m + 1;
    }
    return lo;
}

__device__ __forceinline__ unsigned long long wave_or(unsigned long long v)
{
    for (int o = 32; o > 0; o >>= 1) v |= __shfl_xor(v, o);
    return v;
}

// Inclusive wave scan of v (64 lanes).
__device__ __forceinline__ unsigned long long wave_scan(unsigned long long v, int lane)
{
    for (int o = 1; o < 64; o <<= 1) {
        const unsigned long long t = __shfl_up(v, o);
        if (lane >= o) v += t;
    }
    return v;
}

// PASS 0: destination mask of every query (parts holding >= 1 of its cells)
// and per-part totals (rows, cells).  PASS 1: rows and cell lists written
// into the part-major buffers at row_base[d] / cell_base[d] + cursor.
template <int PASS>
__global__ __launch_bounds__(kBlock) void k_route(int64_t nq, const int64_t *offs, const uint64_t *cells, const float *alo,
                                                  const float *ahi, const int64_t *tlo, const int64_t *thi, int np,
                                                  const uint64_t *part_hi, unsigned long long *mask,
                                                  unsigned long long *tot_rows, unsigned long long *tot_cells,
                                                  const int64_t *row_base, const int64_t *cell_base,
                                                  unsigned long long *cursor, QRow *rows, uint64_t *out_cells)
{
    const int64_t q = tid64();
    const int lane = threadIdx.x & 63;
    const bool live = q < nq;
    unsigned long long m = 0;
    int64_t c0 = 0, nc = 0;
    if (live) {
        c0 = offs[q];
        nc = offs[q + 1] - c0;
        if (PASS == 0) {
            for (int64_t k = 0; k < nc; k++) m |= 1ull << part_of(cells[c0 + k], part_hi, np);
            mask[q] = m;
        } else {
            m = mask[q];
        }
    }
    unsigned long long wm = wave_or(m);
    const unsigned long long below = (1ull << lane) - 1ull;
    while (wm) {  // wave-uniform loop over the destinations this wave meets
        const int d = __builtin_ctzll(wm);
        wm &= wm - 1;
        const bool has = (m >> d) & 1ull;
        const unsigned long long bal = __ballot(has);
        const unsigned long long v = has ? (unsigned long long)nc : 0ull;
        const unsigned long long inc = wave_scan(v, lane);
        const unsigned long long wcells = __shfl(inc, 63);
        const unsigned long long wrows = (unsigned long long)__popcll(bal);
        if (PASS == 0) {
            if (lane == 0) {
                atomicAdd(&tot_rows[d], wrows);
                atomicAdd(&tot_cells[d], wcells);
            }
            continue;
        }
        unsigned long long base = 0;
        if (lane == 0) base = atomicAdd(&cursor[d], (wrows << kCellBits) | wcells);
        base = __shfl(base, 0);
        if (!has) continue;
        const int64_t r = row_base[d] + (int64_t)(base >> kCellBits) + __popcll(bal & below);
        const int64_t cp = cell_base[d] + (int64_t)(base & kCellMask) + (int64_t)(inc - v);
        QRow row;
        row.tlo = tlo[q];
        row.thi = thi[q];
        row.alo = alo[q];
        row.ahi = ahi[q];
        row.qid = (uint32_t)q;
        row.ncells = (uint32_t)nc;
        rows[r] = row;
        for (int64_t k = 0; k < nc; k++) out_cells[cp + k] = cells[c0 + k];
    }
}

// Received segments (source-part-major) -> a plain query batch: SoA
// attributes, per-row cell counts (scanned into offsets by the host driver),
// home part and home-local query id.  t: per source, its first batch row (a),
// its segment's byte offset (b) and its first batch cell (c).
struct PartTable {
    int64_t a[DSSG_MAX_PARTS + 1], b[DSSG_MAX_PARTS + 1], c[DSSG_MAX_PARTS + 1];
};
__device__ __forceinline__ int src_of(const int64_t *base, int np, int64_t i)  // last s with base[s] <= i
{
    int lo = 0, hi = np;
    while (hi - lo > 1) {
        const int m = (lo + hi) >> 1;
        if (base[m] <= i) lo = m;
        else hi = m;
    }
    return lo;
}
__global__ void k_unpack_rows(int64_t n, const unsigned char *recv, int np, PartTable t, int64_t *ncells, float *alo,
                              float *ahi, int64_t *tlo, int64_t *thi, uint32_t *home, uint32_t *qid)
{
    const int64_t i = tid64();
    if (i >= n) return;
    const int src = src_of(t.a, np, i);
    const QRow r = reinterpret_cast<const QRow *>(recv + t.b[src])[i - t.a[src]];
    ncells[i] = r.ncells;
    alo[i] = r.alo;
    ahi[i] = r.ahi;
    tlo[i] = r.tlo;
    thi[i] = r.thi;
    home[i] = (uint32_t)src;
    qid[i] = r.qid;
}
// Each source's cell lists (after its rows) into one contiguous array, in
// source order -- the batch's CSR order.  t.b here: the byte offset of the
// source's cells.
__global__ void k_gather_cells(int64_t nc, const unsigned char *recv, int np, PartTable t, uint64_t *out)
{
    for (int64_t k = tid64(); k < nc; k += (int64_t)gridDim.x * blockDim.x) {
        const int src = src_of(t.c, np, k);
        out[k] = reinterpret_cast<const uint64_t *>(recv + t.b[src])[k - t.c[src]];
    }
}

// Pairs (batch row, entity) -> part-major by the row's home part, packed
// (home-local query << 32 | entity).  PASS 0 counts, PASS 1 fills.  A block
// takes a tile of kPairTile pairs: per-destination counts (and each pair's
// rank among its destination's) come from LDS atomics, and the block adds to
// / reserves from each destination's global counter once -- one global
// atomic per (block, destination), not per (wave, destination): with 10^8
// pairs per step the same-address atomics would otherwise serialise.
constexpr int kPairItems = 16, kPairTile = kBlock * kPairItems;
template <int PASS>
__global__ __launch_bounds__(kBlock) void k_route_pairs(int64_t n, const uint32_t *__restrict__ pq,
                                                        const uint32_t *__restrict__ pe, const uint32_t *__restrict__ home,
                                                        const uint32_t *__restrict__ qid, int np,
                                                        unsigned long long *tot, const int64_t *base_d,
                                                        unsigned long long *cursor, uint64_t *out, int self_part,
                                                        uint32_t *__restrict__ self_q, uint32_t *__restrict__ self_e)
{
    __shared__ uint32_t s_cnt[DSSG_MAX_PARTS];
    __shared__ unsigned long long s_base[DSSG_MAX_PARTS];
    for (int d = threadIdx.x; d < np; d += kBlock) s_cnt[d] = 0;
    __syncthreads();
    const int64_t t0 = (int64_t)blockIdx.x * kPairTile;
    int dst[kPairItems];
    uint32_t rank[kPairItems];
#pragma unroll
    for (int j = 0; j < kPairItems; j++) {
        const int64_t i = t0 + (int64_t)j * kBlock + threadIdx.x;
        dst[j] = -1;
        if (i < n) {
            dst[j] = (int)home[pq[i]];
            rank[j] = atomicAdd(&s_cnt[dst[j]], 1u);
        }
    }
    __syncthreads();
    if (PASS == 0) {
        for (int d = threadIdx.x; d < np; d += kBlock)
            if (s_cnt[d]) atomicAdd(&tot[d], (unsigned long long)s_cnt[d]);
        return;
    }
    for (int d = threadIdx.x; d < np; d += kBlock)
        s_base[d] = s_cnt[d] ? atomicAdd(&cursor[d], (unsigned long long)s_cnt[d]) : 0ull;
    __syncthreads();
#pragma unroll
    for (int j = 0; j < kPairItems; j++) {
        if (dst[j] < 0) continue;
        const int64_t i = t0 + (int64_t)j * kBlock + threadIdx.x;
        const int64_t w = (int64_t)(s_base[dst[j]] + rank[j]);
        if (dst[j] == self_part) {  // this rank's own queries: final (q, e) at once, no exchange
            self_q[w] = qid[pq[i]];
            self_e[w] = pe[i];
        } else {
            out[base_d[dst[j]] + w] = ((uint64_t)qid[pq[i]] << 32) | pe[i];
        }
    }
}

}  // namespace

int64_t route_segment_bytes(int64_t rows, int64_t cells)
{
    return rows * (int64_t)sizeof(QRow) + ((cells * 8 + 31) / 32) * 32;
}

void RouteEngine::plan(int64_t nq, const int64_t *offs, const uint64_t *cells, int np, const uint64_t *part_hi,
                       hipStream_t s, int64_t *row_counts, int64_t *cell_counts, int64_t *seg_bytes)
{
    if (np < 1 || np > kMaxParts) throw Error(DSSG_ERR_INVALID, "route: nparts must be in [1, 64]");
    if (nq >= (1ll << 24)) throw Error(DSSG_ERR_INVALID, "route: more than 2^24 queries per batch");
    unsigned long long *mask = mask_.ensure(nq + 1);
    unsigned long long *acc = acc_.ensure(3 * kMaxParts);  // totals rows | totals cells | cursors
    DSS_HIP(hipMemsetAsync(acc, 0, 3 * kMaxParts * sizeof(unsigned long long), s));
    if (nq > 0)
        hipLaunchKernelGGL(k_route<0>, dim3(grid_for(nq, kBlock)), dim3(kBlock), 0, s, nq, offs, cells, nullptr, nullptr,
                           nullptr, nullptr, np, part_hi, mask, acc, acc + kMaxParts, nullptr, nullptr, nullptr, nullptr,
                           nullptr);
    unsigned long long *h = host_words();
    DSS_HIP(hipMemcpyAsync(h, acc, sizeof(unsigned long long) * 2 * kMaxParts, hipMemcpyDeviceToHost, s));
    DSS_HIP(hipStreamSynchronize(s));
    // fused layout: part d's segment = its rows, then its cell lists, padded
    // to 32 bytes; the fill kernel's bases are the segment's row and cell
    // positions in QRow / uint64 units of the one send buffer
    int64_t *hb = reinterpret_cast<int64_t *>(host_words() + 2 * kMaxParts);
    wait_h2d(h2d_plan_);
    int64_t off = 0, Cn = 0;
    for (int d = 0; d < np; d++) {
        row_counts[d] = (int64_t)h[d];
        cell_counts[d] = (int64_t)h[kMaxParts + d];
        seg_bytes[d] = route_segment_bytes(row_counts[d], cell_counts[d]);
        hb[d] = off / (int64_t)sizeof(QRow);
        hb[kMaxParts + d] = (off + row_counts[d] * (int64_t)sizeof(QRow)) / 8;
        off += seg_bytes[d];
        Cn += cell_counts[d];
    }
    if (Cn >= (int64_t)kCellMask) throw Error(DSSG_ERR_INVALID, "route: more than 2^40 routed cells");
    int64_t *bases = base_.ensure(2 * kMaxParts);
    DSS_HIP(hipMemcpyAsync(bases, hb, sizeof(int64_t) * 2 * kMaxParts, hipMemcpyHostToDevice, s));
    mark_h2d(h2d_plan_, s);
    plan_nq_ = nq;
    plan_np_ = np;
    plan_offs_ = offs;
    plan_cells_ = cells;
    plan_part_hi_ = part_hi;
}

void RouteEngine::fill(int64_t nq, const int64_t *offs, const uint64_t *cells, const float *alo, const float *ahi,
                       const int64_t *tlo, const int64_t *thi, hipStream_t s, void *send)
{
    if (plan_np_ == 0 || nq != plan_nq_ || offs != plan_offs_ || cells != plan_cells_)
        throw Error(DSSG_ERR_INVALID, "route fill: no matching dssg_route_plan_device on this context");
    unsigned long long *acc = acc_.p;
    if (nq > 0)
        hipLaunchKernelGGL(k_route<1>, dim3(grid_for(nq, kBlock)), dim3(kBlock), 0, s, nq, offs, cells, alo, ahi, tlo, thi,
                           plan_np_, plan_part_hi_, mask_.p, nullptr, nullptr, base_.p, base_.p + kMaxParts,
                           acc + 2 * kMaxParts, (QRow *)send, (uint64_t *)send);
    plan_np_ = 0;  // one fill per plan (the cursors are spent)
}

void RouteEngine::unpack(const void *recv, int np, const int64_t *src_rows, const int64_t *src_cells, hipStream_t s,
                         dssg_batch *out)
{
    if (np < 1 || np > kMaxParts) throw Error(DSSG_ERR_INVALID, "unpack: nparts must be in [1, 64]");
    PartTable rt{}, ct{};
    int64_t nrows = 0, ncells = 0, off = 0;
    for (int d = 0; d < np; d++) {
        if (src_rows[d] < 0 || src_cells[d] < 0) throw Error(DSSG_ERR_INVALID, "unpack: negative counts");
        rt.a[d] = nrows;
        rt.b[d] = off;
        ct.c[d] = ncells;
        ct.b[d] = off + src_rows[d] * (int64_t)sizeof(QRow);
        nrows += src_rows[d];
        ncells += src_cells[d];
        off += route_segment_bytes(src_rows[d], src_cells[d]);
    }
    if ((nrows > 0 || ncells > 0) && !recv) throw Error(DSSG_ERR_INVALID, "unpack: NULL receive buffer");
    int64_t *nc = ncell_.ensure(nrows + 1);
    float *alo = alo_.ensure(nrows + 1), *ahi = ahi_.ensure(nrows + 1);
    int64_t *tlo = tlo_.ensure(nrows + 1), *thi = thi_.ensure(nrows + 1);
    uint32_t *home = home_.ensure(nrows + 1), *qid = qid_.ensure(nrows + 1);
    int64_t *offs = offs_.ensure(nrows + 2);
    uint64_t *cells = cells_.ensure(ncells + 1);
    const unsigned char *r = (const unsigned char *)recv;
    if (nrows > 0)
        hipLaunchKernelGGL(k_unpack_rows, dim3(grid_for(nrows, kBlock)), dim3(kBlock), 0, s, nrows, r, np, rt, nc, alo,
                           ahi, tlo, thi, home, qid);
    if (ncells > 0)
        hipLaunchKernelGGL(k_gather_cells, dim3((unsigned)std::min<int64_t>(grid_for(ncells, kBlock), 8192)),
                           dim3(kBlock), 0, s, ncells, r, np, ct, cells);
    exclusive_scan_i64(nc, offs, nrows, tmp_, s);
    out->n = nrows;
    out->offs = offs;
    out->cells = cells;
    out->alt_lo = alo;
    out->alt_hi = ahi;
    out->tlo = tlo;
    out->thi = thi;
    out->home = home;
    out->qid = qid;
}

void RouteEngine::pairs_plan(const dssg_batch *b, const dssg_pairs *p, int np, int self_part, hipStream_t s,
                             int64_t *counts)
{
    if (np < 1 || np > kMaxParts) throw Error(DSSG_ERR_INVALID, "route_pairs: nparts must be in [1, 64]");
    if (self_part < -1 || self_part >= np) throw Error(DSSG_ERR_INVALID, "route_pairs: self part out of range");
    unsigned long long *acc = pacc_.ensure(2 * kMaxParts);
    DSS_HIP(hipMemsetAsync(acc, 0, 2 * kMaxParts * sizeof(unsigned long long), s));
    const int64_t n = p->n;
    if (n > 0)
        hipLaunchKernelGGL(k_route_pairs<0>, dim3(grid_for(n, kPairTile)), dim3(kBlock), 0, s, n, p->q, p->e, b->home,
                           b->qid, np, acc, nullptr, nullptr, nullptr, -1, nullptr, nullptr);
    unsigned long long *h = host_words() + 4 * kMaxParts;
    DSS_HIP(hipMemcpyAsync(h, acc, sizeof(unsigned long long) * kMaxParts, hipMemcpyDeviceToHost, s));
    DSS_HIP(hipStreamSynchronize(s));
    // send-buffer bases: part-major, the self part (written to its own
    // output arrays instead) taking no space
    int64_t *pb = reinterpret_cast<int64_t *>(host_words() + 5 * kMaxParts), tot = 0;
    wait_h2d(h2d_pairs_);
    for (int d = 0; d < np; d++) {
        pb[d] = tot;
        counts[d] = (int64_t)h[d];
        if (d != self_part) tot += counts[d];
    }
    int64_t *d_pb = pbase_.ensure(kMaxParts);
    DSS_HIP(hipMemcpyAsync(d_pb, pb, sizeof(int64_t) * np, hipMemcpyHostToDevice, s));
    mark_h2d(h2d_pairs_, s);
    pplan_n_ = n;
    pplan_np_ = np;
    pplan_self_ = self_part;
    pplan_self_n_ = self_part >= 0 ? counts[self_part] : 0;
    pplan_q_ = p->q;
}

void RouteEngine::pairs_fill(const dssg_batch *b, const dssg_pairs *p, hipStream_t s, uint64_t *out, uint32_t *self_q,
                             uint32_t *self_e)
{
    if (pplan_np_ == 0 || p->n != pplan_n_ || p->q != pplan_q_)
        throw Error(DSSG_ERR_INVALID, "route_pairs fill: no matching dssg_route_pairs_plan_device on this context");
    if (pplan_self_n_ > 0 && (!self_q || !self_e)) throw Error(DSSG_ERR_INVALID, "route_pairs fill: NULL self output");
    if (p->n > pplan_self_n_ && !out) throw Error(DSSG_ERR_INVALID, "route_pairs fill: NULL send buffer");
    if (p->n > 0)
        hipLaunchKernelGGL(k_route_pairs<1>, dim3(grid_for(p->n, kPairTile)), dim3(kBlock), 0, s, p->n, p->q, p->e,
                           b->home, b->qid, pplan_np_, nullptr, pbase_.p, pacc_.p + kMaxParts, out, pplan_self_,
                           self_q, self_e);
    pplan_np_ = 0;
}

// Pinned host words for the count round trips (no pageable staging copy):
// [0, 2P) plan counts, [2P, 4P) plan bases, [4P, 5P) pair counts, [5P, 6P)
// pair bases -- separate regions, so no host write races a pending copy.
unsigned long long *RouteEngine::host_words()
{
    if (!h_counts_) DSS_HIP(hipHostMalloc((void **)&h_counts_, sizeof(unsigned long long) * 6 * kMaxParts,
                                          hipHostMallocDefault));
    return h_counts_;
}

void RouteEngine::wait_h2d(hipEvent_t &ev)
{
    if (ev) DSS_HIP(hipEventSynchronize(ev));
}

void RouteEngine::mark_h2d(hipEvent_t &ev, hipStream_t s)
{
    if (!ev) DSS_HIP(hipEventCreateWithFlags(&ev, hipEventDisableTiming));
    DSS_HIP(hipEventRecord(ev, s));
}

RouteEngine::~RouteEngine()
{
    if (h2d_plan_) {
        (void)hipEventSynchronize(h2d_plan_);
        (void)hipEventDestroy(h2d_plan_);
    }
    if (h2d_pairs_) {
        (void)hipEventSynchronize(h2d_pairs_);
        (void)hipEventDestroy(h2d_pairs_);
    }
    if (h_counts_) (void)hipHostFree(h_counts_);
}

namespace {
__global__ void k_split_pairs(int64_t n, const uint64_t *__restrict__ in, uint32_t *__restrict__ q,
                              uint32_t *__restrict__ e)
{
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
        const uint64_t k = in[i];
        q[i] = (uint32_t)(k >> 32);
        e[i] = (uint32_t)k;
    }
}
}  // namespace

void RouteEngine::split_pairs(int64_t n, const uint64_t *in, uint32_t *q, uint32_t *e, hipStream_t s)
{
    if (n <= 0) return;
    const unsigned g = (unsigned)std::min<int64_t>((n + 255) / 256, 8192);
    hipLaunchKernelGGL(k_split_pairs, dim3(g), dim3(256), 0, s, n, in, q, e);
    DSS_HIP(hipGetLastError());
}

}  // namespace dss
