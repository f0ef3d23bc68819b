// Order-preserving stream compaction, hand-written for gfx950 (wave64).
//
// compact_if(n, pred, emit): emit(i, rank) for every i in [0, n) with
// pred(i), rank = number of earlier i with pred -- without materialising a
// flag array (the predicate is evaluated twice, once per pass); split_if
// also places the failing elements (rank i - passing before i):
//   k_cmp_count  one 1024-element tile per block: count -> cnt[tile]
//   exclusive_scan_i64 over the tile counts (scan.hip)
//   k_cmp_emit   the tile again: per 256-element row a ballot per wave, the
//                row/wave prefix from LDS, rank = tile base + prefix + mbcnt.
// HBM: whatever pred/emit touch, plus 16 B per tile.  Replaces hipCUB's
// DevicePartition / RunLengthEncode and the int64 flag + scan arrays of the
// index build (8 B of flags per element per predicate).
//
// Pred: __device__ bool operator()(int64_t i) const
// Emit: __device__ void operator()(int64_t i, int64_t rank) const
#pragma once
#include <hip/hip_runtime.h>

#include <type_traits>

#include "common.hpp"

namespace dss {
namespace cmpct {

constexpr int kBlock = 256, kWaves = kBlock / 64, kRows = 4, kTile = kBlock * kRows;  // (1024-element tiles: a 1M-element split fills the chip; 4096 left it at one block per CU)

__device__ __forceinline__ uint32_t lanes_below(unsigned long long m)
{
    return __builtin_amdgcn_mbcnt_hi((uint32_t)(m >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)m, 0u));
}

template <class Pred>
__global__ __launch_bounds__(kBlock) void k_cmp_count(int64_t n, Pred pred, int64_t *__restrict__ cnt)
{
    __shared__ uint32_t ws[kWaves];
    const int64_t base = (int64_t)blockIdx.x * kTile;
    uint32_t c = 0;
#pragma unroll 4
    for (int r = 0; r < kRows; r++) {
        const int64_t i = base + (int64_t)r * kBlock + threadIdx.x;
        const bool p = i < n && pred(i);
        c += (uint32_t)__popcll(__ballot(p));
    }
    if ((threadIdx.x & 63) == 0) ws[threadIdx.x >> 6] = c;
    __syncthreads();
    if (threadIdx.x == 0) {
        uint32_t t = 0;
#pragma unroll
        for (int w = 0; w < kWaves; w++) t += ws[w];
        cnt[blockIdx.x] = (int64_t)t;
    }
}

struct NoEmit {
    __device__ void operator()(int64_t, int64_t) const {}
};

// EmitF: also place the elements failing pred (rank among those = i - the
// passing ones before i); NoEmit: compaction only.
template <class Pred, class Emit, class EmitF>
__global__ __launch_bounds__(kBlock) void k_cmp_emit(int64_t n, Pred pred, Emit emit, EmitF emit_f,
                                                     const int64_t *__restrict__ off)
{
    constexpr bool kSplit = !std::is_same<EmitF, NoEmit>::value;
    __shared__ uint32_t rc[kRows * kWaves];  // (row, wave) counts, then their exclusive prefix
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    const int64_t base = (int64_t)blockIdx.x * kTile;
    unsigned long long bal[kRows];
    uint32_t pm = 0;  // bit r: this lane's element of row r passes
#pragma unroll
    for (int r = 0; r < kRows; r++) {
        const int64_t i = base + (int64_t)r * kBlock + threadIdx.x;
        const bool p = i < n && pred(i);
        bal[r] = __ballot(p);
        pm |= p ? (1u << r) : 0u;
        if (lane == 0) rc[r * kWaves + w] = (uint32_t)__popcll(bal[r]);
    }
    __syncthreads();
    static_assert(kRows * kWaves <= 64, "one wave scans the (row, wave) counts");
    if (threadIdx.x < 64) {  // exclusive scan of the (row, wave) counts, row-major = element order
        const uint32_t v = threadIdx.x < kRows * kWaves ? rc[threadIdx.x] : 0u;
        uint32_t x = v;
#pragma unroll
        for (int o = 1; o < 64; o <<= 1) {
            const uint32_t y = __shfl_up(x, o, 64);
            if (lane >= o) x += y;
        }
        if (threadIdx.x < kRows * kWaves) rc[threadIdx.x] = x - v;
    }
    __syncthreads();
    const int64_t tb = off[blockIdx.x];
#pragma unroll
    for (int r = 0; r < kRows; r++) {
        const int64_t i = base + (int64_t)r * kBlock + threadIdx.x;
        const int64_t rank = tb + (int64_t)rc[r * kWaves + w] + (int64_t)lanes_below(bal[r]);
        if ((pm >> r) & 1u)
            emit(i, rank);
        else if (kSplit && i < n)
            emit_f(i, i - rank);
    }
}

// Number of tiles and the scratch bytes compact_if needs for n elements.
inline int64_t tiles_for(int64_t n) { return (n + kTile - 1) / kTile; }

}  // namespace cmpct

// Where split_if(n, ..., tmp, ...) leaves the passing count on the device
// (the last word of its tile scan in `tmp`), for an emit_f that places the
// failing elements after the passing ones; valid from the emit pass on.
inline const int64_t *split_total_slot(int64_t n, DevBuf<unsigned char> &tmp)
{
    const int64_t nt = cmpct::tiles_for(n);
    return (const int64_t *)tmp.ensure(sizeof(int64_t) * (2 * nt + 2)) + 2 * nt;
}

// Order-preserving split: emit(i, rank) for the elements passing pred,
// emit_f(i, rank) for the others (each rank within its side); the passing
// count lands in *d_total (device, int64; skipped when null) and, when
// `h_total` is non-null, on the host (one stream sync).  EmitF =
// cmpct::NoEmit: plain compaction.
template <class Pred, class Emit, class EmitF>
void split_if(int64_t n, Pred pred, Emit emit, EmitF emit_f, DevBuf<unsigned char> &tmp,
              DevBuf<unsigned char> &scan_tmp, hipStream_t s, int64_t *d_total, int64_t *h_total)
{
    const int64_t nt = cmpct::tiles_for(n);
    if (n <= 0) {
        if (d_total) DSS_HIP(hipMemsetAsync(d_total, 0, sizeof(int64_t), s));
        if (h_total) *h_total = 0;
        return;
    }
    // scratch: tile counts (nt) + their exclusive scan (nt + 1) in `tmp`; the
    // scan's own scratch in `scan_tmp`
    int64_t *cnt = (int64_t *)tmp.ensure(sizeof(int64_t) * (2 * nt + 2));
    int64_t *off = cnt + nt;
    hipLaunchKernelGGL(cmpct::k_cmp_count<Pred>, dim3((unsigned)nt), dim3(cmpct::kBlock), 0, s, n, pred, cnt);
    exclusive_scan_i64(cnt, off, nt, scan_tmp, s);
    hipLaunchKernelGGL((cmpct::k_cmp_emit<Pred, Emit, EmitF>), dim3((unsigned)nt), dim3(cmpct::kBlock), 0, s, n, pred,
                       emit, emit_f, (const int64_t *)off);
    if (d_total) DSS_HIP(hipMemcpyAsync(d_total, off + nt, sizeof(int64_t), hipMemcpyDeviceToDevice, s));
    DSS_HIP(hipGetLastError());
    if (h_total) {
        DSS_HIP(hipMemcpyAsync(h_total, off + nt, sizeof(int64_t), hipMemcpyDeviceToHost, s));
        DSS_HIP(hipStreamSynchronize(s));
    }
}

// Order-preserving compaction (split_if without the failing side).
template <class Pred, class Emit>
void compact_if(int64_t n, Pred pred, Emit emit, DevBuf<unsigned char> &tmp, DevBuf<unsigned char> &scan_tmp,
                hipStream_t s, int64_t *d_total, int64_t *h_total)
{
    split_if(n, pred, emit, cmpct::NoEmit{}, tmp, scan_tmp, s, d_total, h_total);
}

}  // namespace dss
