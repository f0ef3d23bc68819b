// Batched ingress: models.UnionVolumes4D (pkg/models/geo.go:126-190) for a
// batch of multi-extent volumes.
//
// The reference covers every extent of a request and merges the cells in a
// Go map (precomputedCellGeometry, geo.go:100-122), taking min start, max
// end, min altitude_lower and max altitude_upper over the extents that carry
// them (NULLs skipped), and stops at the first covering error in extent
// order.  Here one cover launch handles every extent of the batch; the union
// is one radix sort of (volume << 29 | cell >> 35) keys -- a level-13 cell id
// has 29 significant bits above its marker bit 34 -- followed by an adjacent
// unique.  The union comes out sorted per volume; the reference's map order
// is unspecified (quirk Q14), and every consumer treats it as a set.
#include <hip/hip_runtime.h>


#include <cmath>

#include "ingress.hpp"
#include "radix.hpp"

namespace dss {
namespace {

constexpr unsigned kBlock = 256;
constexpr uint64_t kLsb13 = 1ull << 34;

__device__ __forceinline__ int64_t tid64() { return (int64_t)blockIdx.x * blockDim.x + threadIdx.x; }

// Extent -> volume.
__global__ void k_extent_vol(int64_t nvol, const int64_t *vol_offs, uint32_t *evol)
{
    const int64_t v = tid64();
    if (v >= nvol) return;
    for (int64_t x = vol_offs[v]; x < vol_offs[v + 1]; x++) evol[x] = (uint32_t)v;
}

// One key per covered cell of an extent that has a footprint.
__global__ void k_union_keys(int64_t nx, const int64_t *offs, const uint64_t *cells, const uint32_t *evol,
                             const uint8_t *has_fp, unsigned long long *key)
{
    const int64_t x = tid64();
    if (x >= nx) return;
    const int64_t c0 = offs[x], c1 = offs[x + 1];
    const unsigned long long hi = (unsigned long long)evol[x] << 29;
    const bool use = has_fp[x] != 0;
    for (int64_t k = c0; k < c1; k++) key[k] = use ? (hi | (cells[k] >> 35)) : ~0ull;
}

__global__ void k_unique_flags(int64_t n, const unsigned long long *key, int64_t *flag)
{
    const int64_t i = tid64();
    if (i >= n) return;
    flag[i] = key[i] != ~0ull && (i == 0 || key[i] != key[i - 1]) ? 1 : 0;
}

__global__ void k_unique_scatter(int64_t n, const unsigned long long *key, const int64_t *flag, const int64_t *pos,
                                 uint64_t *cells, unsigned long long *vcnt)
{
    const int64_t i = tid64();
    if (i >= n || !flag[i]) return;
    cells[pos[i]] = ((key[i] & ((1ull << 29) - 1)) << 35) | kLsb13;
    atomicAdd(&vcnt[key[i] >> 29], 1ull);
}

__global__ void k_u64_to_i64_n(int64_t n, const unsigned long long *a, int64_t *b)
{
    const int64_t k = tid64();
    if (k < n) b[k] = (int64_t)a[k];
}

// Per volume: first covering error in extent order, NULL-skipping min/max.
__global__ void k_volume_attrs(int64_t nvol, const int64_t *vol_offs, const int32_t *xstatus, const double *xarea,
                               const uint8_t *has_fp, const float *alo, const float *ahi, const int64_t *t0,
                               const int64_t *t1, int32_t *status, double *area, float *oalo, float *oahi,
                               int64_t *ot0, int64_t *ot1, uint8_t *ofp)
{
    const int64_t v = tid64();
    if (v >= nvol) return;
    int32_t st = 0;
    double ar = 0;
    float lo = NAN, hi = NAN;
    long long s = INT64_MIN, e = INT64_MAX;
    bool any_s = false, any_e = false, fp = false;
    for (int64_t x = vol_offs[v]; x < vol_offs[v + 1]; x++) {
        if (t1[x] != INT64_MAX) {  // EndTime set
            e = any_e ? max(e, (long long)t1[x]) : (long long)t1[x];
            any_e = true;
        }
        if (t0[x] != INT64_MIN) {  // StartTime set
            s = any_s ? min(s, (long long)t0[x]) : (long long)t0[x];
            any_s = true;
        }
        if (!isnan(alo[x])) lo = isnan(lo) ? alo[x] : fminf(lo, alo[x]);
        if (!isnan(ahi[x])) hi = isnan(hi) ? ahi[x] : fmaxf(hi, ahi[x]);
        if (has_fp[x]) {
            fp = true;
            if (xstatus[x] != 0) {  // CalculateCovering error: UnionVolumes4D returns it
                st = xstatus[x];
                ar = xarea[x];
                break;
            }
        }
    }
    status[v] = st;
    area[v] = ar;
    // NULL out as the search's sentinels (dssgpu.h conventions): a union volume
    // feeds dssg_search* / the index build directly, and the ordered compares
    // there treat -INF/+INF like COALESCE(..., true) where NaN would match nothing
    oalo[v] = isnan(lo) ? -INFINITY : lo;
    oahi[v] = isnan(hi) ? INFINITY : hi;
    ot0[v] = s;
    ot1[v] = e;
    ofp[v] = fp ? 1 : 0;
}

}  // namespace

void IngressEngine::union_volumes(CoverEngine &ce, int64_t nvol, const int64_t *vol_offs, int64_t nx, const int32_t *kind,
                                  const int64_t *voff, const double *lat, const double *lng, const float *radius_m,
                                  const uint8_t *has_fp, const float *alo, const float *ahi, const int64_t *t0,
                                  const int64_t *t1, hipStream_t s, dssg_volumes *out)
{
    if (nvol >= (1ll << 34)) throw Error(DSSG_ERR_INVALID, "union: too many volumes");
    dssg_cells cv;
    ce.run(nx, kind, voff, lat, lng, radius_m, s, &cv);
    const int64_t C = cv.total_cells;
    uint32_t *evol = evol_.ensure(nx + 1);
    if (nvol > 0) hipLaunchKernelGGL(k_extent_vol, dim3(grid_for(nvol, kBlock)), dim3(kBlock), 0, s, nvol, vol_offs, evol);
    unsigned long long *k0 = k0_.ensure(C + 1), *k1 = k1_.ensure(C + 1);
    if (nx > 0)
        hipLaunchKernelGGL(k_union_keys, dim3(grid_for(nx, kBlock)), dim3(kBlock), 0, s, nx, cv.offs, cv.cells, evol,
                           has_fp, k0);
    if (C > 0) {
        // sort on the key bits in use: 29 cell bits + enough for nvol (the
        // ~0 keys of footprint-less extents sort last within that range)
        int bits = 30;
        while (bits < 64 && ((unsigned long long)nvol >> (bits - 29)) != 0) bits++;
        radix_sort_keys(k0, k1, C, bits, tmp_, s);
    }
    int64_t *flag = flag_.ensure(C + 1), *pos = pos_.ensure(C + 2);
    if (C > 0) hipLaunchKernelGGL(k_unique_flags, dim3(grid_for(C, kBlock)), dim3(kBlock), 0, s, C, k1, flag);
    exclusive_scan_i64(flag, pos, C, tmp_, s);
    int64_t U = 0;
    if (C > 0) {
        DSS_HIP(hipMemcpyAsync(&U, pos + C, sizeof(int64_t), hipMemcpyDeviceToHost, s));
        DSS_HIP(hipStreamSynchronize(s));
    }
    uint64_t *cells = cells_.ensure(U + 1);
    unsigned long long *vcnt = vcnt_.ensure(nvol + 1);
    DSS_HIP(hipMemsetAsync(vcnt, 0, sizeof(unsigned long long) * (nvol + 1), s));
    if (C > 0)
        hipLaunchKernelGGL(k_unique_scatter, dim3(grid_for(C, kBlock)), dim3(kBlock), 0, s, C, k1, flag, pos, cells, vcnt);
    int64_t *v64 = v64_.ensure(nvol + 1), *offs = offs_.ensure(nvol + 2);
    if (nvol > 0)
        hipLaunchKernelGGL(k_u64_to_i64_n, dim3(grid_for(nvol, kBlock)), dim3(kBlock), 0, s, nvol, vcnt, v64);
    exclusive_scan_i64(v64, offs, nvol, tmp_, s);
    int32_t *status = status_.ensure(nvol + 1);
    double *area = area_.ensure(nvol + 1);
    float *lo = lo_.ensure(nvol + 1), *hi = hi_.ensure(nvol + 1);
    int64_t *a0 = t0_.ensure(nvol + 1), *a1 = t1_.ensure(nvol + 1);
    uint8_t *fp = fp_.ensure(nvol + 1);
    if (nvol > 0)
        hipLaunchKernelGGL(k_volume_attrs, dim3(grid_for(nvol, kBlock)), dim3(kBlock), 0, s, nvol, vol_offs, cv.status,
                           cv.area_km2, has_fp, alo, ahi, t0, t1, status, area, lo, hi, a0, a1, fp);
    DSS_HIP(hipStreamSynchronize(s));
    out->n = nvol;
    out->offs = offs;
    out->cells = cells;
    out->status = status;
    out->area_km2 = area;
    out->alt_lo = lo;
    out->alt_hi = hi;
    out->t0 = a0;
    out->t1 = a1;
    out->has_footprint = fp;
    out->total_cells = U;
}

}  // namespace dss
