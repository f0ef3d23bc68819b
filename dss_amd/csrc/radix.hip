// LSD radix sort, hand-written for gfx950 (wave64).  Replaces the CockroachDB
// index ordering of `scd_cells_operations` (PK (cell_id, operation_id),
// pkg/scd/store/cockroach/store.go:140-147) in the index build, and groups a
// batch's (cell, bucket) keys before the join.
//
// Per pass over `rb` <= 8 digit bits (passes = ceil(span / 8), digit width
// balanced across passes: 18 bits -> 3 x 6, level-13 cell ids -> 4 x 7-8;
// 9-bit digits measured slower: 0.26 vs 0.20 ms on 11.6M 18-bit keys),
// three launches:
//   k_rs_hist    one 2048-key tile per block (8 keys per thread: the
//                scatter's 24 KiB of LDS staging for (u32, u64) pairs lets
//                more blocks share a CU than 16 keys' 48 KiB; configs[2]'s
//                per-search key-sort scatter 0.059 -> 0.041 ms per pass,
//                187.2M against 183.9M q/s, profiles/r04s_radix_tiles), per-wave
//                LDS digit counts,
//                written digit-major hist[d][tile] (so one row scan gives
//                every tile its global start per digit);
//   k_rs_scan    one block per digit: exclusive scan of its row in place,
//                row total -> dtot[d];
//   k_rs_scatter the same tile again: each wave ranks its 512 keys by
//                ballot match (rb ballots per 64 keys -> the lanes holding the
//                same digit; rank = popcount of those below the lane) against
//                a per-wave LDS digit counter, so the order stays stable
//                (wave, iteration, lane) = input order; the block then places
//                the keys digit-sorted in LDS and writes them out in tile
//                order, so every digit's run leaves as a contiguous burst.
// HBM per pass: 4n key bytes (hist) + (|K| + |V|) n read + (|K| + |V|) n
// written, plus 4 * 2^rb * tiles of counts.
#include <hip/hip_runtime.h>

#include <algorithm>

#include "radix.hpp"

namespace dss {
namespace {

constexpr int kRBlock = 256;
#ifndef DSS_RADIX_BITS
#define DSS_RADIX_BITS 8
#endif
#ifndef DSS_RADIX_ITEMS
#define DSS_RADIX_ITEMS 8
#endif
constexpr int kMaxDigitBits = DSS_RADIX_BITS;    // digit bits per pass (8: 256 digits, one per thread)
constexpr int kMaxDigits = 1 << kMaxDigitBits;
constexpr int kDPT = kMaxDigits / kRBlock;       // digits per thread in the per-digit phases
constexpr int kRWaves = kRBlock / 64;
constexpr int kItems = DSS_RADIX_ITEMS;

template <typename K>
__device__ __forceinline__ uint32_t digit_of(K k, int shift, uint32_t mask)
{
    return (uint32_t)(k >> shift) & mask;
}

__device__ __forceinline__ uint32_t lanes_below(unsigned long long m)
{
    return __builtin_amdgcn_mbcnt_hi((uint32_t)(m >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)m, 0u));
}

// Inclusive block scan of one value per thread; `total` = block sum.  Syncs
// on entry use of ws and before returning, so ws can be reused at once.
__device__ __forceinline__ uint32_t block_incl_scan(uint32_t x, uint32_t *ws, uint32_t &total)
{
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
#pragma unroll
    for (int off = 1; off < 64; off <<= 1) {
        const uint32_t y = __shfl_up(x, off, 64);
        if (lane >= off) x += y;
    }
    if (lane == 63) ws[w] = x;
    __syncthreads();
    uint32_t pre = 0, tot = 0;
#pragma unroll
    for (int i = 0; i < kRWaves; i++) {
        const uint32_t t = ws[i];
        pre += i < w ? t : 0u;
        tot += t;
    }
    __syncthreads();
    total = tot;
    return x + pre;
}

template <typename K, int ITEMS = kItems>
__global__ __launch_bounds__(kRBlock) void k_rs_hist(const K *__restrict__ keys, int64_t n, const int64_t *__restrict__ dn,
                                                     int shift, int rbits, uint32_t *__restrict__ hist, int64_t stride)
{
    if (dn) n = min(n, *dn);
    __shared__ uint32_t h[kRWaves][kMaxDigits];
    const int tid = threadIdx.x, w = tid >> 6;
    const uint32_t nd = 1u << rbits, mask = nd - 1;
    for (int i = tid; i < kRWaves * kMaxDigits; i += kRBlock) (&h[0][0])[i] = 0;
    __syncthreads();
    const int64_t base = (int64_t)blockIdx.x * (kRBlock * ITEMS);
    K k[ITEMS];
#pragma unroll
    for (int j = 0; j < ITEMS; j++) {
        const int64_t i = base + j * kRBlock + tid;
        k[j] = i < n ? keys[i] : K(0);
    }
#ifdef DSS_HIST_MATCH
    // (variant) lanes of one digit found by ballot match, one LDS add per run:
    // clustered keys (hotspot cells) otherwise serialise on the same counter
    const int lane = tid & 63;
#pragma unroll
    for (int j = 0; j < ITEMS; j++) {
        const bool ok = base + j * kRBlock + tid < n;
        const uint32_t d = digit_of(k[j], shift, mask);
        unsigned long long m = __ballot(ok);
        for (int b = 0; b < rbits; b++) {
            const unsigned long long bb = __ballot((d >> b) & 1u);
            m &= ((d >> b) & 1u) ? bb : ~bb;
        }
        if (ok && lanes_below(m) == 0) atomicAdd(&h[w][d], (uint32_t)__popcll(m));
        (void)lane;
    }
#else
#pragma unroll
    for (int j = 0; j < ITEMS; j++)
        if (base + j * kRBlock + tid < n) atomicAdd(&h[w][digit_of(k[j], shift, mask)], 1u);
#endif
    __syncthreads();
    for (int d = tid; d < (int)nd; d += kRBlock) {
        uint32_t c = 0;
#pragma unroll
        for (int i = 0; i < kRWaves; i++) c += h[i][d];
        hist[(int64_t)d * stride + blockIdx.x] = c;
    }
}

__global__ __launch_bounds__(kRBlock) void k_rs_scan(uint32_t *__restrict__ hist, int64_t stride, int64_t ntiles,
                                                     uint32_t *__restrict__ dtot)
{
    __shared__ uint32_t ws[kRWaves];
    uint32_t *row = hist + (int64_t)blockIdx.x * stride;
    uint32_t carry = 0;
    for (int64_t b0 = 0; b0 < ntiles; b0 += kRBlock * 4) {
        const int64_t i0 = b0 + (int64_t)threadIdx.x * 4;
        uint32_t v[4], t = 0;
#pragma unroll
        for (int k = 0; k < 4; k++) {
            v[k] = i0 + k < ntiles ? row[i0 + k] : 0u;
            t += v[k];
        }
        uint32_t total;
        uint32_t run = carry + block_incl_scan(t, ws, total) - t;
#pragma unroll
        for (int k = 0; k < 4; k++) {
            if (i0 + k < ntiles) row[i0 + k] = run;
            run += v[k];
        }
        carry += total;
    }
    if (threadIdx.x == 0) dtot[blockIdx.x] = carry;
}

// PK (packed 8-B words, radix_sort_pairs_packed): bit 0 -- the pass reads
// (key, value) and sorts the word (key & ~lomask) | value; bit 1 -- it writes
// the word back out as (word & ~lomask) | kconst and value word & lomask.
// Middle passes move the words alone (HAS_V false).
template <typename K, typename V, bool HAS_V, int PK = 0, int ITEMS = kItems>
__global__ __launch_bounds__(kRBlock) void k_rs_scatter(const K *__restrict__ ki, const V *__restrict__ vi,
                                                        K *__restrict__ ko, V *__restrict__ vo, int64_t n,
                                                        const int64_t *__restrict__ dn, int shift, int rbits,
                                                        const uint32_t *__restrict__ hist, int64_t stride,
                                                        const uint32_t *__restrict__ dtot, K lomask = 0, K kconst = 0)
{
    static_assert(PK == 0 || !HAS_V, "packed passes stage the words alone");
    if (dn) n = min(n, *dn);
    __shared__ uint32_t wh[kRWaves][kMaxDigits];  // per-wave digit counters, then their exclusive prefix over waves
    __shared__ uint32_t dstart[kMaxDigits];       // tile-local start of each digit
    __shared__ uint32_t gbase[kMaxDigits];        // global position of tile slot 0 of each digit
    __shared__ uint32_t ws[kRWaves];
    constexpr int kT = kRBlock * ITEMS, kWT = 64 * ITEMS;
    __shared__ K sk[kT];
    __shared__ V sv[HAS_V ? kT : 1];
    const int tid = threadIdx.x, w = tid >> 6, lane = tid & 63;
    const uint32_t nd = 1u << rbits, mask = nd - 1;
    for (int i = tid; i < kRWaves * kMaxDigits; i += kRBlock) (&wh[0][0])[i] = 0;
    // global start of digits kDPT*tid .. +kDPT-1 in this tile: all smaller
    // digits + the same digit in earlier tiles
    uint32_t dt[kDPT], dsum = 0;
#pragma unroll
    for (int u = 0; u < kDPT; u++) {
        const uint32_t d = (uint32_t)(kDPT * tid + u);
        dt[u] = d < nd ? dtot[d] : 0u;
        dsum += dt[u];
    }
    uint32_t unused;
    uint32_t gstart[kDPT];
    {
        uint32_t run = block_incl_scan(dsum, ws, unused) - dsum;
#pragma unroll
        for (int u = 0; u < kDPT; u++) {
            const uint32_t d = (uint32_t)(kDPT * tid + u);
            gstart[u] = d < nd ? run + hist[(int64_t)d * stride + blockIdx.x] : 0u;
            run += dt[u];
        }
    }

    const int64_t sub = (int64_t)blockIdx.x * kT + (int64_t)w * kWT;
    K k[ITEMS];
    V v[ITEMS];
    uint32_t loc[ITEMS];
#pragma unroll
    for (int j = 0; j < ITEMS; j++) {
        const int64_t i = sub + j * 64 + lane;
        const bool ok = i < n;
        if constexpr ((PK & 1) != 0) k[j] = ok ? ((ki[i] & ~lomask) | (K)vi[i]) : K(0);
        else k[j] = ok ? ki[i] : K(0);
        if (HAS_V) v[j] = ok ? vi[i] : V(0);
    }
#pragma unroll
    for (int j = 0; j < ITEMS; j++) {
        const bool ok = sub + j * 64 + lane < n;
        const uint32_t d = digit_of(k[j], shift, mask);
        unsigned long long m = __ballot(ok);
        for (int b = 0; b < rbits; b++) {
            const unsigned long long bb = __ballot((d >> b) & 1u);
            m &= ((d >> b) & 1u) ? bb : ~bb;
        }
        // every lane reads its digit's counter before the run's last lane
        // bumps it (one wave, program order)
        const uint32_t before = wh[w][d];
        const uint32_t rank = lanes_below(m);
        const uint32_t cnt = (uint32_t)__popcll(m);
        if (ok && rank + 1 == cnt) wh[w][d] = before + cnt;
        loc[j] = before + rank;
    }
    __syncthreads();
    uint32_t cnt[kDPT], csum = 0;
#pragma unroll
    for (int u = 0; u < kDPT; u++) {
        const int d = kDPT * tid + u;
        uint32_t c = 0;
#pragma unroll
        for (int i = 0; i < kRWaves; i++) {
            const uint32_t t = wh[i][d];
            wh[i][d] = c;
            c += t;
        }
        cnt[u] = c;
        csum += c;
    }
    {
        uint32_t st = block_incl_scan(csum, ws, unused) - csum;
#pragma unroll
        for (int u = 0; u < kDPT; u++) {
            const int d = kDPT * tid + u;
            dstart[d] = st;
            gbase[d] = gstart[u] - st;  // modular: gbase + slot lands in [gstart, gstart + cnt)
            st += cnt[u];
        }
    }
    __syncthreads();
#pragma unroll
    for (int j = 0; j < ITEMS; j++) {
        if (sub + j * 64 + lane < n) {
            const uint32_t d = digit_of(k[j], shift, mask);
            const uint32_t slot = dstart[d] + wh[w][d] + loc[j];
            sk[slot] = k[j];
            if (HAS_V) sv[slot] = v[j];
        }
    }
    __syncthreads();
    const int64_t rem = n - (int64_t)blockIdx.x * kT;
    const int tile_n = rem < kT ? (int)rem : kT;
    for (int i = tid; i < tile_n; i += kRBlock) {
        const K kk = sk[i];
        const uint32_t p = gbase[digit_of(kk, shift, mask)] + (uint32_t)i;
        if constexpr ((PK & 2) != 0) {
            ko[p] = (kk & ~lomask) | kconst;
            vo[p] = (V)(kk & lomask);
        } else {
            ko[p] = kk;
        }
        if (HAS_V) vo[p] = sv[i];
    }
}

// OR over all keys of (key ^ keys[0]): the bits that vary.  Bits constant
// across the batch need no pass (a level-13 cell id varies in bits 35..63
// only, so a 64-bit (cell, entity) sort runs 4 passes instead of 8).
// (vals != nullptr: the OR of the values too, in part[np + block] -- the
// value bits a packed sort must leave room for)
template <typename K>
__global__ __launch_bounds__(kRBlock) void k_rs_varying(const K *__restrict__ keys, int64_t n,
                                                        unsigned long long *__restrict__ part,
                                                        const uint32_t *__restrict__ vals = nullptr)
{
    __shared__ unsigned long long wacc[kRWaves], wv[kRWaves];
    const K k0 = keys[0];
    unsigned long long acc = 0, vacc = 0;
    for (int64_t i = (int64_t)blockIdx.x * kRBlock + threadIdx.x; i < n; i += (int64_t)gridDim.x * kRBlock) {
        acc |= (unsigned long long)(keys[i] ^ k0);
        if (vals) vacc |= vals[i];
    }
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) {
        acc |= __shfl_xor(acc, off, 64);
        vacc |= __shfl_xor(vacc, off, 64);
    }
    if ((threadIdx.x & 63) == 0) {
        wacc[threadIdx.x >> 6] = acc;
        wv[threadIdx.x >> 6] = vacc;
    }
    __syncthreads();
    if (threadIdx.x == 0) {
        unsigned long long r = 0, rv = 0;
#pragma unroll
        for (int i = 0; i < kRWaves; i++) {
            r |= wacc[i];
            rv |= wv[i];
        }
        part[blockIdx.x] = r;  // one partial per block: no same-address atomics
        if (vals) part[gridDim.x + blockIdx.x] = rv;
    }
}

__global__ __launch_bounds__(kRBlock) void k_rs_or_parts(const unsigned long long *__restrict__ part, int np,
                                                         unsigned long long *__restrict__ out)
{
    __shared__ unsigned long long wacc[kRWaves];
    unsigned long long acc = 0;
    for (int i = threadIdx.x; i < np; i += kRBlock) acc |= part[i];
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) acc |= __shfl_xor(acc, off, 64);
    if ((threadIdx.x & 63) == 0) wacc[threadIdx.x >> 6] = acc;
    __syncthreads();
    if (threadIdx.x == 0) {
        unsigned long long r = 0;
#pragma unroll
        for (int i = 0; i < kRWaves; i++) r |= wacc[i];
        *out = r;
    }
}

inline size_t align256(size_t x) { return (x + 255) & ~(size_t)255; }

template <typename K, typename V, bool HAS_V>
void radix_sort(const K *ki, K *ko, const V *vi, V *vo, int64_t n, const int64_t *dn, int bits, DevBuf<unsigned char> &tmp,
                hipStream_t s)
{
    // 8-B keys alone: 4096-key tiles (16 per thread; 32 KiB of LDS staging,
    // twice the digit-run length per tile -- the packed path's measurement)
    constexpr int IT = (!HAS_V && sizeof(K) == 8) ? 2 * kItems : kItems, kT = kRBlock * IT;
    if (n <= 0) return;
    // positions are uint32: the digit offsets of the last tile stay < 2^32
    if (n >= ((int64_t)1 << 32) - kT) throw Error(DSSG_ERR_CAPACITY, "radix sort: more than 2^32 - 4096 keys");
    const int kbits = (int)(8 * sizeof(K));
    if (bits > kbits) bits = kbits;
    if (bits <= 0) {
        device_copy(ko, ki, sizeof(K) * n, s);
        if (HAS_V) device_copy(vo, vi, sizeof(V) * n, s);
        return;
    }
    const int64_t ntiles = (n + kT - 1) / kT, stride = (ntiles + 3) & ~(int64_t)3;
    const size_t hist_b = align256(sizeof(uint32_t) * kMaxDigits * stride), dtot_b = align256(sizeof(uint32_t) * kMaxDigits);
    // wide keys: sort only the span of bits that vary (one read + one host
    // sync, against up to 4 passes saved)
    int lo = 0;
    if (bits > 24 && !dn) {  // (a device-side count: the caller's exact bit width)
        const int g = (int)std::min<int64_t>(ntiles, 1024);
        unsigned long long *vm = (unsigned long long *)tmp.ensure(std::max(hist_b + dtot_b, sizeof(unsigned long long) * (g + 1))),
                           *part = vm + 1;
        hipLaunchKernelGGL(k_rs_varying<K>, dim3((unsigned)g), dim3(kRBlock), 0, s, ki, n, part);
        hipLaunchKernelGGL(k_rs_or_parts, dim3(1), dim3(kRBlock), 0, s, part, g, vm);
        unsigned long long var = 0;
        DSS_HIP(hipMemcpyAsync(&var, vm, sizeof(var), hipMemcpyDeviceToHost, s));
        DSS_HIP(hipStreamSynchronize(s));
        if (bits < 64) var &= (1ull << bits) - 1;
        if (var == 0) bits = 0;  // every key equal on the sorted bits: stable = identity
        else {
            lo = __builtin_ctzll(var);
            bits = 64 - __builtin_clzll(var);
        }
    }
    if (bits <= lo) {
        device_copy(ko, ki, sizeof(K) * n, s);
        if (HAS_V) device_copy(vo, vi, sizeof(V) * n, s);
        return;
    }
    const int span = bits - lo, passes = (span + kMaxDigitBits - 1) / kMaxDigitBits, rb = (span + passes - 1) / passes;
    const size_t ka_b = passes > 1 ? align256(sizeof(K) * n) : 0, va_b = passes > 1 && HAS_V ? align256(sizeof(V) * n) : 0;
    unsigned char *t = tmp.ensure(hist_b + dtot_b + ka_b + va_b);
    uint32_t *hist = (uint32_t *)t, *dtot = (uint32_t *)(t + hist_b);
    K *kalt = (K *)(t + hist_b + dtot_b);
    V *valt = (V *)(t + hist_b + dtot_b + ka_b);
    const K *src = ki;
    const V *srcv = vi;
    for (int p = 0; p < passes; p++) {
        const int shift = lo + p * rb, r = bits - shift < rb ? bits - shift : rb;
        // the last pass lands in ko; earlier ones alternate ko / kalt backwards
        const bool to_out = ((passes - 1 - p) & 1) == 0;
        K *dst = to_out ? ko : kalt;
        V *dstv = to_out ? vo : valt;
        hipLaunchKernelGGL((k_rs_hist<K, IT>), dim3((unsigned)ntiles), dim3(kRBlock), 0, s, src, n, dn, shift, r, hist, stride);
        hipLaunchKernelGGL(k_rs_scan, dim3(1u << r), dim3(kRBlock), 0, s, hist, stride, ntiles, dtot);
        hipLaunchKernelGGL((k_rs_scatter<K, V, HAS_V, 0, IT>), dim3((unsigned)ntiles), dim3(kRBlock), 0, s, src, srcv, dst, dstv,
                           n, dn, shift, r, hist, stride, dtot);
        DSS_HIP(hipGetLastError());
        src = dst;
        srcv = dstv;
    }
}

// (u64 key, u32 value) pairs sorted as packed 8-B words when the keys' low
// bits below their lowest varying bit are constant and wide enough for every
// value (level-13 cell ids: bits 0..34 constant, entity ids < 2^32): the
// first pass packs (key & ~lomask) | value, the middle passes move 8 B per
// element instead of 12, the last unpacks.  Stable on the key bits, so equal
// keys keep their input order -- (cell, entity) postings arriving in entity
// order leave in PK (cell_id, operation_id) order.  Otherwise: radix_sort.
void radix_sort_packed(const uint64_t *ki, uint64_t *ko, const uint32_t *vi, uint32_t *vo, int64_t n, int bits,
                       DevBuf<unsigned char> &tmp, hipStream_t s)
{
    using K = uint64_t;
    // 4096-word tiles (16 per thread): the words alone need 32 KiB of LDS
    // staging, and a digit's run per tile is twice as long as at 2048 (the
    // scatter's writes are the pass's cost where the low digits are random)
#ifndef DSS_PACKED_ITEMS
#define DSS_PACKED_ITEMS 16
#endif
    constexpr int kPI = DSS_PACKED_ITEMS, kPT = kRBlock * kPI;
    if (n <= 0) return;
    if (n >= ((int64_t)1 << 32) - kPT) throw Error(DSSG_ERR_CAPACITY, "radix sort: more than 2^32 - 4096 keys");
    if (bits > 64) bits = 64;
    const int64_t ntiles = (n + kPT - 1) / kPT, stride = (ntiles + 3) & ~(int64_t)3;
    const size_t hist_b = align256(sizeof(uint32_t) * kMaxDigits * stride), dtot_b = align256(sizeof(uint32_t) * kMaxDigits);
    const int g = (int)std::min<int64_t>(ntiles, 1024);
    unsigned long long var = 0, vor = 0, k0 = 0;
    {
        unsigned long long *vm = (unsigned long long *)tmp.ensure(
                               std::max(hist_b + dtot_b, sizeof(unsigned long long) * (2 * g + 3))),
                           *part = vm + 3;
        // the keys' varying bits first; the values are scanned only when the
        // keys' constant low bits are fewer than 32 (level-13 ids: 35)
        hipLaunchKernelGGL(k_rs_varying<K>, dim3((unsigned)g), dim3(kRBlock), 0, s, ki, n, part, nullptr);
        hipLaunchKernelGGL(k_rs_or_parts, dim3(1), dim3(kRBlock), 0, s, part, g, vm);
        DSS_HIP(hipMemcpyAsync(&var, vm, sizeof(var), hipMemcpyDeviceToHost, s));
        DSS_HIP(hipMemcpyAsync(&k0, ki, sizeof(k0), hipMemcpyDeviceToHost, s));
        DSS_HIP(hipStreamSynchronize(s));
        const unsigned long long vsorted = bits < 64 ? var & ((1ull << bits) - 1) : var;
        if (vsorted != 0 && __builtin_ctzll(vsorted) < 32) {
            hipLaunchKernelGGL(k_rs_varying<K>, dim3((unsigned)g), dim3(kRBlock), 0, s, ki, n, part, vi);
            hipLaunchKernelGGL(k_rs_or_parts, dim3(1), dim3(kRBlock), 0, s, part + g, g, vm + 1);
            DSS_HIP(hipMemcpyAsync(&vor, vm + 1, sizeof(vor), hipMemcpyDeviceToHost, s));
            DSS_HIP(hipStreamSynchronize(s));
        } else {
            vor = 0xffffffffull;  // any u32 value fits below bit 32
        }
    }
    if (bits < 64) var &= (1ull << bits) - 1;
    const int lo = var ? __builtin_ctzll(var) : 64, hi = var ? 64 - __builtin_clzll(var) : 0;
    const int vbits = vor ? 64 - __builtin_clzll(vor) : 0;
    if (var == 0 || vbits > lo) {  // nothing to sort, or no room for the values: the plain sort
        radix_sort<K, uint32_t, true>(ki, ko, vi, vo, n, nullptr, bits, tmp, s);
        return;
    }
    const K lomask = lo >= 64 ? ~0ull : ((1ull << lo) - 1), kconst = k0 & lomask;
    const int span = hi - lo, passes = (span + kMaxDigitBits - 1) / kMaxDigitBits, rb = (span + passes - 1) / passes;
    const size_t ka_b = passes > 1 ? align256(sizeof(K) * n) : 0;
    unsigned char *t = tmp.ensure(hist_b + dtot_b + ka_b);
    uint32_t *hist = (uint32_t *)t, *dtot = (uint32_t *)(t + hist_b);
    K *kalt = (K *)(t + hist_b + dtot_b);
    const K *src = ki;
    for (int p = 0; p < passes; p++) {
        const int shift = lo + p * rb, r = hi - shift < rb ? hi - shift : rb;
        const bool to_out = ((passes - 1 - p) & 1) == 0;
        K *dst = to_out ? ko : kalt;
        hipLaunchKernelGGL((k_rs_hist<K, kPI>), dim3((unsigned)ntiles), dim3(kRBlock), 0, s, src, n, nullptr, shift, r,
                           hist, stride);
        hipLaunchKernelGGL(k_rs_scan, dim3(1u << r), dim3(kRBlock), 0, s, hist, stride, ntiles, dtot);
        const bool first = p == 0, last = p == passes - 1;
        if (first && last)
            hipLaunchKernelGGL((k_rs_scatter<K, uint32_t, false, 3, kPI>), dim3((unsigned)ntiles), dim3(kRBlock), 0, s,
                               src, vi, dst, vo, n, nullptr, shift, r, hist, stride, dtot, lomask, kconst);
        else if (first)
            hipLaunchKernelGGL((k_rs_scatter<K, uint32_t, false, 1, kPI>), dim3((unsigned)ntiles), dim3(kRBlock), 0, s,
                               src, vi, dst, vo, n, nullptr, shift, r, hist, stride, dtot, lomask, kconst);
        else if (last)
            hipLaunchKernelGGL((k_rs_scatter<K, uint32_t, false, 2, kPI>), dim3((unsigned)ntiles), dim3(kRBlock), 0, s,
                               src, vi, dst, vo, n, nullptr, shift, r, hist, stride, dtot, lomask, kconst);
        else
            hipLaunchKernelGGL((k_rs_scatter<K, uint32_t, false, 0, kPI>), dim3((unsigned)ntiles), dim3(kRBlock), 0, s,
                               src, vi, dst, vo, n, nullptr, shift, r, hist, stride, dtot, lomask, kconst);
        DSS_HIP(hipGetLastError());
        src = dst;
    }
}

}  // namespace

void radix_sort_pairs_packed(const uint64_t *ki, uint64_t *ko, const uint32_t *vi, uint32_t *vo, int64_t n, int bits,
                             DevBuf<unsigned char> &tmp, hipStream_t s)
{
    radix_sort_packed(ki, ko, vi, vo, n, bits, tmp, s);
}

template <typename K, typename V>
void radix_sort_pairs(const K *ki, K *ko, const V *vi, V *vo, int64_t n, int bits, DevBuf<unsigned char> &tmp,
                      hipStream_t s)
{
    radix_sort<K, V, true>(ki, ko, vi, vo, n, nullptr, bits, tmp, s);
}

template <typename K, typename V>
void radix_sort_pairs_dn(const K *ki, K *ko, const V *vi, V *vo, int64_t n_max, const int64_t *dn, int bits,
                         DevBuf<unsigned char> &tmp, hipStream_t s)
{
    radix_sort<K, V, true>(ki, ko, vi, vo, n_max, dn, bits, tmp, s);
}

template <typename K>
void radix_sort_keys(const K *ki, K *ko, int64_t n, int bits, DevBuf<unsigned char> &tmp, hipStream_t s)
{
    radix_sort<K, uint32_t, false>(ki, ko, nullptr, nullptr, n, nullptr, bits, tmp, s);
}

template void radix_sort_pairs<unsigned long, uint32_t>(const unsigned long *, unsigned long *, const uint32_t *,
                                                        uint32_t *, int64_t, int, DevBuf<unsigned char> &, hipStream_t);
template void radix_sort_pairs<uint32_t, uint32_t>(const uint32_t *, uint32_t *, const uint32_t *, uint32_t *, int64_t,
                                                   int, DevBuf<unsigned char> &, hipStream_t);
template void radix_sort_pairs<uint32_t, unsigned long>(const uint32_t *, uint32_t *, const unsigned long *,
                                                        unsigned long *, int64_t, int, DevBuf<unsigned char> &,
                                                        hipStream_t);
template void radix_sort_pairs<unsigned long long, uint32_t>(const unsigned long long *, unsigned long long *,
                                                             const uint32_t *, uint32_t *, int64_t, int,
                                                             DevBuf<unsigned char> &, hipStream_t);
template void radix_sort_pairs_dn<uint32_t, unsigned long>(const uint32_t *, uint32_t *, const unsigned long *,
                                                           unsigned long *, int64_t, const int64_t *, int,
                                                           DevBuf<unsigned char> &, hipStream_t);
template void radix_sort_pairs_dn<uint32_t, uint32_t>(const uint32_t *, uint32_t *, const uint32_t *, uint32_t *, int64_t,
                                                      const int64_t *, int, DevBuf<unsigned char> &, hipStream_t);
template void radix_sort_keys<unsigned long long>(const unsigned long long *, unsigned long long *, int64_t, int,
                                                  DevBuf<unsigned char> &, hipStream_t);
template void radix_sort_keys<unsigned long>(const unsigned long *, unsigned long *, int64_t, int,
                                             DevBuf<unsigned char> &, hipStream_t);

}  // namespace dss
