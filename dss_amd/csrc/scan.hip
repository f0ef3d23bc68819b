// Device-wide scans used by the covering and search pipelines for
// order-preserving compaction (the int64 exclusive scan below, the
// polygon/circle partition over compact.cuh), plus the device copy.
#include <cstdlib>
#include <string>

#include "common.hpp"
#include "compact.cuh"

namespace dss {

namespace {

__device__ __forceinline__ int64_t tid64_s() { return (int64_t)blockIdx.x * blockDim.x + threadIdx.x; }

// Exclusive int64 prefix sum, reduce-then-scan over 2048-element tiles
// (256 lanes x 8 consecutive elements):
//   k_scan_reduce  tile sums -> part[t]            (skipped for one tile)
//   k_scan_parts   one block: exclusive scan of the tile sums, in place
//   k_scan_down    tile t again: lane sums, block scan, + part[t] -> out
// No look-back spin and no library state: 3 launches (1 for n <= 2048; 2 up
// to 2M elements, k_scan_down_fold summing the tile sums itself), HBM 8n
// read twice + 8n written.
constexpr int kSBlock = 256, kSWaves = kSBlock / 64, kSItems = 8, kSTile = kSBlock * kSItems;

__device__ __forceinline__ long long block_incl_scan_i64(long long x, long long *ws, long long &total)
{
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
#pragma unroll
    for (int off = 1; off < 64; off <<= 1) {
        const long long y = __shfl_up(x, off, 64);
        if (lane >= off) x += y;
    }
    if (lane == 63) ws[w] = x;
    __syncthreads();
    long long pre = 0, tot = 0;
#pragma unroll
    for (int i = 0; i < kSWaves; i++) {
        const long long t = ws[i];
        pre += i < w ? t : 0;
        tot += t;
    }
    __syncthreads();
    total = tot;
    return x + pre;
}

__device__ __forceinline__ long long lane_items(const int64_t *in, int64_t n, int64_t i0, long long v[kSItems])
{
    long long t = 0;
    const bool a16 = ((uintptr_t)in & 15) == 0;  // callers pass offsets into shared buffers
    if (a16 && i0 + kSItems <= n) {
        const longlong2 *p = reinterpret_cast<const longlong2 *>(in + i0);  // i0 is a multiple of 8
#pragma unroll
        for (int u = 0; u < kSItems / 2; u++) {
            const longlong2 q = p[u];
            v[2 * u] = q.x;
            v[2 * u + 1] = q.y;
        }
    } else {
#pragma unroll
        for (int u = 0; u < kSItems; u++) v[u] = i0 + u < n ? in[i0 + u] : 0;
    }
#pragma unroll
    for (int u = 0; u < kSItems; u++) t += v[u];
    return t;
}

__global__ __launch_bounds__(kSBlock) void k_scan_reduce(const int64_t *__restrict__ in, int64_t n,
                                                         long long *__restrict__ part)
{
    __shared__ long long ws[kSWaves];
    long long v[kSItems];
    const long long t = lane_items(in, n, (int64_t)blockIdx.x * kSTile + (int64_t)threadIdx.x * kSItems, v);
    long long total;
    block_incl_scan_i64(t, ws, total);
    if (threadIdx.x == 0) part[blockIdx.x] = total;
}

__global__ __launch_bounds__(kSBlock) void k_scan_parts(long long *__restrict__ part, int64_t nt)
{
    __shared__ long long ws[kSWaves];
    long long carry = 0;
    for (int64_t b0 = 0; b0 < nt; b0 += kSBlock) {
        const int64_t i = b0 + threadIdx.x;
        const long long v = i < nt ? part[i] : 0;
        long long total;
        const long long incl = block_incl_scan_i64(v, ws, total);
        if (i < nt) part[i] = carry + incl - v;
        carry += total;
    }
}

__global__ __launch_bounds__(kSBlock) void k_scan_down(const int64_t *__restrict__ in, int64_t n,
                                                       const long long *__restrict__ part, int64_t *__restrict__ out,
                                                       int64_t *mail)
{
    __shared__ long long ws[kSWaves];
    const int64_t i0 = (int64_t)blockIdx.x * kSTile + (int64_t)threadIdx.x * kSItems;
    long long v[kSItems];
    const long long t = lane_items(in, n, i0, v);
    long long total;
    long long run = block_incl_scan_i64(t, ws, total) - t + (part ? part[blockIdx.x] : 0);
    if (blockIdx.x == 0 && threadIdx.x == 0) out[0] = 0;
#pragma unroll
    for (int u = 0; u < kSItems; u++) {
        run += v[u];
        if (i0 + u < n) out[i0 + u + 1] = run;  // out[k + 1] = in[0] + ... + in[k]
        if (mail && i0 + u + 1 == n) *mail = run;
    }
}

// k_scan_down for up to kSFoldTiles tiles without k_scan_parts: each block
// sums the tile sums before it itself (<= 1024 L2-resident words), one
// launch fewer per scan -- a 1M-element scan is 489 tiles.
constexpr int64_t kSFoldTiles = 1024;
__global__ __launch_bounds__(kSBlock) void k_scan_down_fold(const int64_t *__restrict__ in, int64_t n,
                                                            const long long *__restrict__ part,
                                                            int64_t *__restrict__ out, int64_t *mail)
{
    __shared__ long long ws[kSWaves];
    long long pre = 0, total;
    for (int64_t t = threadIdx.x; t < (int64_t)blockIdx.x; t += kSBlock) pre += part[t];
    block_incl_scan_i64(pre, ws, total);
    pre = total;  // the tiles before this one
    const int64_t i0 = (int64_t)blockIdx.x * kSTile + (int64_t)threadIdx.x * kSItems;
    long long v[kSItems];
    const long long t = lane_items(in, n, i0, v);
    long long run = block_incl_scan_i64(t, ws, total) - t + pre;
    if (blockIdx.x == 0 && threadIdx.x == 0) out[0] = 0;
#pragma unroll
    for (int u = 0; u < kSItems; u++) {
        run += v[u];
        if (i0 + u < n) out[i0 + u + 1] = run;
        if (mail && i0 + u + 1 == n) *mail = run;
    }
}

__global__ void k_mail_counters(const unsigned int *a, const unsigned int *b, const unsigned int *c, int64_t *mail)
{
    if (threadIdx.x == 0) {
        mail[0] = a ? (int64_t)*a : 0;
        mail[1] = b ? (int64_t)*b : 0;
        mail[2] = c ? (int64_t)*c : 0;
    }
}

}  // namespace

void exclusive_scan_i64(const int64_t *in, int64_t *out, int64_t n, DevBuf<unsigned char> &tmp, hipStream_t s,
                        int64_t *mail)
{
    if (n <= 0) {
        DSS_HIP(hipMemsetAsync(out, 0, sizeof(int64_t), s));
        if (mail) DSS_HIP(hipMemsetAsync(mail, 0, sizeof(int64_t), s));
        return;
    }
    const int64_t nt = (n + kSTile - 1) / kSTile;
    long long *part = nullptr;
    if (nt > 1) {
        part = (long long *)tmp.ensure(sizeof(long long) * nt);
        hipLaunchKernelGGL(k_scan_reduce, dim3((unsigned)nt), dim3(kSBlock), 0, s, in, n, part);
        if (nt <= kSFoldTiles) {
            hipLaunchKernelGGL(k_scan_down_fold, dim3((unsigned)nt), dim3(kSBlock), 0, s, in, n, (const long long *)part,
                               out, mail);
            DSS_HIP(hipGetLastError());
            return;
        }
        hipLaunchKernelGGL(k_scan_parts, dim3(1), dim3(kSBlock), 0, s, part, nt);
    }
    hipLaunchKernelGGL(k_scan_down, dim3((unsigned)nt), dim3(kSBlock), 0, s, in, n, (const long long *)part, out, mail);
    DSS_HIP(hipGetLastError());
}

void mail_counters(const unsigned int *a, const unsigned int *b, const unsigned int *c, int64_t *mail, hipStream_t s)
{
    hipLaunchKernelGGL(k_mail_counters, dim3(1), dim3(64), 0, s, a, b, c, mail);
    DSS_HIP(hipGetLastError());
}

namespace {
struct IsCircle {
    const int32_t *kind;
    bool want;
    __device__ bool operator()(int64_t i) const { return (kind[i] == DSSG_KIND_CIRCLE) == want; }
};
struct PlaceAt {
    uint32_t *perm;
    const int64_t *base;  // device: the first part's size (nullptr: 0)
    __device__ void operator()(int64_t i, int64_t r) const { perm[(base ? *base : 0) + r] = (uint32_t)i; }
};

// 16-B vectors, four per thread per round with every load issued before
// the stores (a grid-stride loop of one vector keeps one load in flight per
// lane: 4.7 TB/s read + write on 4 GiB)
__global__ __launch_bounds__(256) void k_copy16(int64_t n16, const uint4 *__restrict__ src, uint4 *__restrict__ dst)
{
    const int64_t stride = (int64_t)gridDim.x * blockDim.x;
    int64_t i = tid64_s();
    for (; i + 3 * stride < n16; i += 4 * stride) {
        const uint4 a = src[i], b = src[i + stride], c = src[i + 2 * stride], d = src[i + 3 * stride];
        dst[i] = a;
        dst[i + stride] = b;
        dst[i + 2 * stride] = c;
        dst[i + 3 * stride] = d;
    }
    for (; i < n16; i += stride) dst[i] = src[i];
}
__global__ void k_copy1(int64_t n, const unsigned char *__restrict__ src, unsigned char *__restrict__ dst)
{
    for (int64_t i = tid64_s(); i < n; i += (int64_t)gridDim.x * blockDim.x) dst[i] = src[i];
}
}  // namespace

void partition_polygons_first(const int32_t *kind, uint32_t *perm, unsigned long long *nsel, int64_t n,
                              DevBuf<unsigned char> &tmp, DevBuf<unsigned char> &tmp2, hipStream_t s)
{
    if (n <= 0) return;
    // non-circles first, then circles after them: one split (count, scan,
    // place both sides) instead of a compaction per side
    (void)nsel;
    split_if(n, IsCircle{kind, false}, PlaceAt{perm, nullptr}, PlaceAt{perm, split_total_slot(n, tmp)}, tmp, tmp2, s,
             nullptr, nullptr);
}

void device_copy(void *dst, const void *src, size_t bytes, hipStream_t s)
{
    if (!bytes) return;
    const bool a16 = (((uintptr_t)dst | (uintptr_t)src) & 15) == 0;
    const int64_t n16 = a16 ? (int64_t)(bytes / 16) : 0, done = n16 * 16;
    const unsigned g = 8192;  // grid-stride: any size, work items < 2^32
    if (n16) hipLaunchKernelGGL(k_copy16, dim3(g), dim3(256), 0, s, n16, (const uint4 *)src, (uint4 *)dst);
    if ((int64_t)bytes > done)
        hipLaunchKernelGGL(k_copy1, dim3(g), dim3(256), 0, s, (int64_t)bytes - done, (const unsigned char *)src + done,
                           (unsigned char *)dst + done);
    DSS_HIP(hipGetLastError());
}

void stage_check(hipStream_t s, const char *stage)
{
    static const bool on = [] {
        const char *e = std::getenv("DSSG_SYNC_CHECK");
        return e && *e && *e != '0';
    }();
    if (!on) return;
    const hipError_t e = hipStreamSynchronize(s);
    if (e != hipSuccess) throw Error(DSSG_ERR_DEVICE, std::string("after ") + stage + ": " + hipGetErrorString(e));
}

}  // namespace dss
