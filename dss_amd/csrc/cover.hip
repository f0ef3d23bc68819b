// Level-13 S2 covering of DSS footprints on gfx950.
//
// Reference semantics: pkg/geo/s2.go:99-122 (Covering: area check, in-place
// reversal, zero-area -> open polyline), pkg/models/geo.go:224-268 (circle
// 20-gon, polygon range checks), golang/geo RegionCoverer{13,13}: the result
// is the sorted set of level-13 cells c with region.IntersectsCell(c).
//
// Two paths (CoverEngine::run): batches of <= 16k footprints (the per-request
// path) take k_cover_wave, one wavefront per footprint; larger batches take
// the general pipeline (all device resident):
//   k_nverts, k_circle_frames, k_verts, k_fan, k_orient, k_fan_area
//              vertex slots, S2 points with Go's Cephes trig, RegularLoop,
//              (u,v) images, Loop.Area's fan terms (one thread per vertex /
//              needed triangle)
//   k_setup    one thread per footprint: origin containment, area sum,
//              reversal, status/mode, touched-face mask, start cells, with
//              triage predicates; k_setup_exact redoes the few footprints the
//              triage cannot decide, one wave each, exactly
//   k_cand_fp / k_cand_exact
//              direct candidates of the single-face small loops (most
//              footprints): the cells of their padded bound, tested exactly
//   k_clip_items  ClipToPaddedFace of every edge of the descent footprints on
//              every touched face, fine (level-13) and coarse (pruning) pads
//   k_start    <= 4 start cells per face around the clipped-edge bound
//   k_expand_* level-synchronous descent over the descent footprints'
//              frontier nodes at once (exact S2 node tests deferred to
//              k_expand_exact); children written in Hilbert (= id) order
//              behind an exclusive scan, so each footprint's output is sorted
//              by construction -- no sort pass
//   k_cand_emit / k_emit   level-13 ids into the CSR per footprint.
// Roofline: FP64 VALU (edge clip / crossing tests); see DESIGN.md.
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>

#include "common.hpp"
#include "compact.cuh"
#include "cover.hpp"
#include "loopdev.cuh"

namespace dss {
using namespace s2;

namespace {

constexpr int kBlock = 256;
constexpr double kCoarsePad = 1e-9;  // pruning padding, >> FACE_CLIP_PLUS_RECT_ERR (2.36e-15)
constexpr double kFinePad = DSS_FACE_CLIP_PLUS_RECT_ERR;

enum : uint8_t { MODE_NONE = 0, MODE_LOOP = 1, MODE_POLYLINE = 2 };
enum : uint8_t { FL_SMALL = 1, FL_PLANAR = 2, FL_FAST = 4 };
// Direct candidate path: single-face small loops whose start block is at
// level >= kFastMinLevel (<= 4 * 4^(13 - L) level-13 candidates).
constexpr int kFastMinLevel = 10;
constexpr int kCandStageV = 2048;  // (u,v) vertices a k_cand_fp block stages in LDS (float2: 16 KiB)
// node meta: level (bits 0-4), orientation (5-6), done (7), face (8-10)
__device__ __forceinline__ uint32_t pack_meta(int level, int orient, int done, int face)
{
    return (uint32_t)level | ((uint32_t)orient << 5) | ((uint32_t)done << 7) | ((uint32_t)face << 8);
}
__device__ __forceinline__ int meta_level(uint32_t m) { return (int)(m & 31u); }
__device__ __forceinline__ int meta_orient(uint32_t m) { return (int)((m >> 5) & 3u); }
__device__ __forceinline__ int meta_done(uint32_t m) { return (int)((m >> 7) & 1u); }
__device__ __forceinline__ int meta_face(uint32_t m) { return (int)((m >> 8) & 7u); }

__device__ __forceinline__ int64_t tid64() { return (int64_t)blockIdx.x * blockDim.x + threadIdx.x; }

// (also zeroes the per-footprint flags and the list counters the setup
// kernels accumulate into: six fill launches fewer per covering)
__global__ void k_nverts(int64_t n, const int32_t *kind, const int64_t *voff, int64_t *nv, uint8_t *fan_fail,
                         uint8_t *not_inner, uint8_t *bad, unsigned int *c0, unsigned int *c1, unsigned int *c2)
{
    int64_t f = tid64();
    if (f == 0) *c0 = *c1 = *c2 = 0u;
    if (f >= n) return;
    nv[f] = kind[f] == DSSG_KIND_CIRCLE ? 20 : (voff[f + 1] - voff[f]);
    fan_fail[f] = not_inner[f] = bad[f] = 0;
}

// cos/sin of the 20 RegularLoop angles i * 2pi/20 (regular_loop.go), computed
// on the host with the same Go-math restatement (gomath.cuh is host+device).
__constant__ double c_circle_cos[20], c_circle_sin[20];

__device__ bool edge_inside_face(V3 a, V3 b, int face)
{
    if (xyz_face(a) != face || xyz_face(b) != face) return false;
    double u0, v0, u1, v1;
    valid_face_xyz_to_uv(face, a, u0, v0);
    valid_face_xyz_to_uv(face, b, u1, v1);
    const double lim = 1.0 - 1e-6;
    return __builtin_fabs(u0) <= lim && __builtin_fabs(v0) <= lim && __builtin_fabs(u1) <= lim &&
           __builtin_fabs(v1) <= lim;
}

struct FaceBox {
    double ulo, uhi, vlo, vhi;
};

// Coarse bound of footprint f on face fc (clipped edges, plus polyline vertex
// projections), expanded by the coarse padding.  Returns false if empty.
__device__ bool face_box(const V3 *p, int nv, uint8_t md, const double4 *clip_c, const uint8_t *cflags, int64_t base,
                         int ne, FaceBox &b, int fc)
{
    double ulo = 1e300, uhi = -1e300, vlo = 1e300, vhi = -1e300;
    bool any = false;
    for (int e = 0; e < ne; e++) {
        if (!(cflags[base + e] & 2)) continue;
        double4 c = clip_c[base + e];
        ulo = fmin(ulo, fmin(c.x, c.z));
        uhi = fmax(uhi, fmax(c.x, c.z));
        vlo = fmin(vlo, fmin(c.y, c.w));
        vhi = fmax(vhi, fmax(c.y, c.w));
        any = true;
    }
    if (md == MODE_POLYLINE) {
        for (int i = 0; i < nv; i++) {
            double u, v;
            if (face_xyz_to_uv(fc, p[i], u, v) && __builtin_fabs(u) <= 1 + kCoarsePad && __builtin_fabs(v) <= 1 + kCoarsePad) {
                ulo = fmin(ulo, u); uhi = fmax(uhi, u);
                vlo = fmin(vlo, v); vhi = fmax(vhi, v);
                any = true;
            }
        }
    }
    const double m = 1e-7;  // generous: the start region only has to contain the bound
    b = FaceBox{ulo - m, uhi + m, vlo - m, vhi + m};
    return any;
}

// Start cells for one face: <= 2x2 block of cells at the deepest level (<=13)
// whose i and j spans cover the bound.  Writes up to 4 (id, i0, j0, meta)
// sorted by id; returns the count.
__device__ int start_cells(const FaceBox &b, int fc, uint64_t *id, uint32_t *ii, uint32_t *jj, uint32_t *meta)
{
    double ulo = fmax(b.ulo, -1.0), uhi = fmin(b.uhi, 1.0), vlo = fmax(b.vlo, -1.0), vhi = fmin(b.vhi, 1.0);
    int i0 = st_to_ij(uv_to_st(ulo)), i1 = st_to_ij(uv_to_st(uhi));
    int j0 = st_to_ij(uv_to_st(vlo)), j1 = st_to_ij(uv_to_st(vhi));
    int L = kCoverLevel;
    while (L > 0 && (((i1 >> (kMaxLevel - L)) - (i0 >> (kMaxLevel - L))) > 1 || ((j1 >> (kMaxLevel - L)) - (j0 >> (kMaxLevel - L))) > 1))
        L--;
    int sh = kMaxLevel - L;
    int cnt = 0;
    for (int a = i0 >> sh; a <= (i1 >> sh); a++)
        for (int c = j0 >> sh; c <= (j1 >> sh); c++) {
            int o;
            uint64_t cid = cell_from_face_ij_level(fc, a << sh, c << sh, L, o);
            // insertion sort by id
            int k = cnt++;
            while (k > 0 && id[k - 1] > cid) {
                id[k] = id[k - 1]; ii[k] = ii[k - 1]; jj[k] = jj[k - 1]; meta[k] = meta[k - 1];
                k--;
            }
            id[k] = cid;
            ii[k] = (uint32_t)(a << sh);
            jj[k] = (uint32_t)(c << sh);
            meta[k] = pack_meta(L, o, 0, fc);
        }
    return cnt;
}

// ---------------------------------------------------------------------------
// Per-vertex pre-pass (FAST path).  The serial per-footprint work of loop
// construction is dominated by transcendental FP64 (Go's Cephes trig in
// PointFromLatLng and in every fan triangle's PointArea), so it is spread one
// thread per vertex slot: no divergence between footprints of different
// kind or size, and the per-footprint kernel only sums.
//
// k_circle_frames: RegularLoop's frame per circle (centre, ortho basis,
// cos/sin of the radius) -- regular_loop.go, computed once per circle.
struct CircleFrame {
    V3 c, c0, c1;
    double z, rr;
};
__global__ void k_circle_frames(int64_t n, const int32_t *kind, const int64_t *voff, const double *lat,
                                const double *lng, const float *radius_m, CircleFrame *fr)
{
    const int64_t f = tid64();
    if (f >= n || kind[f] != DSSG_KIND_CIRCLE) return;
    const V3 c = point_from_degrees(lat[voff[f]], lng[voff[f]]);
    const double radius = (double)radius_m[f] / DSS_RADIUS_EARTH_M;
    const V3 c1 = ortho(c), c0 = cross(c1, c);
    fr[f] = CircleFrame{c, c0, c1, go_cos(radius), go_sin(radius)};
}

// Owner footprint of every slot of a CSR layout (offs: n + 1 offsets; perm:
// the footprint of CSR position t, nullptr for footprint order).
__global__ void k_vowner(int64_t n, const int64_t *offs, uint32_t *vown, const uint32_t *perm = nullptr)
{
    const int64_t t = tid64();
    if (t >= n) return;
    const uint32_t f = perm ? perm[t] : (uint32_t)t;
    for (int64_t x = offs[t]; x < offs[t + 1]; x++) vown[x] = f;
}

// Vertex slots laid out in k_setup's footprint order (polygons, then
// circles): the per-slot kernels' waves then run one kind's path (k_verts:
// Cephes sincos for a polygon vertex, a frame product for a circle's), and
// k_setup's lanes read neighbouring slot ranges.
__global__ void k_perm_counts(int64_t n, const uint32_t *perm, const int64_t *nv, int64_t *nvp)
{
    const int64_t t = tid64();
    if (t < n) nvp[t] = nv[perm[t]];
}
__global__ void k_perm_offsets(int64_t n, const uint32_t *perm, const int64_t *xoffp, int64_t *xoff)
{
    const int64_t t = tid64();
    if (t < n) xoff[perm[t]] = xoffp[t];
    if (t == 0) xoff[n] = xoffp[n];
}

// One thread per vertex slot: S2 point of a polygon vertex
// (PointFromLatLng(LatLngFromDegrees)) or of a RegularLoop vertex.  A polygon
// vertex out of range (Q17: GeoPolygon.CalculateCovering's check precedes the
// count check) marks its footprint bad[f] (zeroed before), so k_setup reads
// one flag instead of re-walking the footprint's coordinates.
__global__ void k_verts(int64_t nx, const uint32_t *vown, const int32_t *kind, const int64_t *voff,
                        const double *lat, const double *lng, const int64_t *xoff, const CircleFrame *fr, V3 *xyz,
                        uint8_t *bad)
{
    const int64_t x = tid64();
    if (x >= nx) return;
    const uint32_t f = vown[x];
    const int i = (int)(x - xoff[f]);
    if (kind[f] == DSSG_KIND_CIRCLE) {
        const CircleFrame F = fr[f];
        const double px = F.rr * c_circle_cos[i], py = F.rr * c_circle_sin[i], pz = F.z;
        xyz[x] = normalize(v3(F.c0.x * px + F.c1.x * py + F.c.x * pz, F.c0.y * px + F.c1.y * py + F.c.y * pz,
                              F.c0.z * px + F.c1.z * py + F.c.z * pz));
    } else {
        const double la = lat[voff[f] + i], ln = lng[voff[f] + i];
        if (kind[f] == DSSG_KIND_POLYGON && (la > 90.0 || la < -90.0 || ln > 180.0 || ln < -180.0)) bad[f] = 1;
        xyz[x] = point_from_degrees(la, ln);
    }
}

// One thread per vertex slot of a loop candidate (n >= 3 slots): the (u,v)
// image of the vertex on the face of vertex 0 (the planar data k_setup keeps
// for single-face small loops) and whether edge (i, i+1) lies inside that
// face (any edge that does not clears the footprint's inner flag:
// not_inner[f] = 1).
__global__ void k_fan(int64_t nx, const uint32_t *vown, const int64_t *nslots, const int64_t *xoff, const V3 *xyz,
                      double2 *uv, uint8_t *not_inner)
{
    const int64_t x = tid64();
    if (x >= nx) return;
    const uint32_t f = vown[x];
    const int n = (int)nslots[f];
    const int i = (int)(x - xoff[f]);
    if (n < 3) return;
    const V3 *p = xyz + xoff[f];
    const int face0 = xyz_face(p[0]);
    double u, v;
    valid_face_xyz_to_uv(face0, p[i], u, v);  // = ClipToPaddedFace's same-face fast path
    uv[x] = make_double2(u, v);
    if (!edge_inside_face(p[i], p[i + 1 == n ? 0 : i + 1], face0)) not_inner[f] = 1;
}

// Fan-term orientation of a non-circle loop (n >= 3 vertices).  loop.go Area
// sums SignedArea over the fan (v0, vi, vi+1); when that sum is negative the
// area wraps to ~4 pi, exceeds the cap and the loop is reversed (Q4), so only
// the reversed fan's terms matter.  Each term is sign(det(a,b,c)) times the
// triangle's spherical excess E, and tan(E/2) = |det| / (1 + a.b + b.c + c.a):
// with every vertex within 0.05 rad of v0, E = |det|/2 to 0.2 %.  So
// D = sum det / 2 predicts the sign of the sum whenever |D| exceeds 5 % of
// sum |det| / 2 (plus an absolute floor far above rounding):
//   omode 0: sum > 0 and the area (loopAreaKm2, Q1) below the cap -> forward terms only;
//   omode 1: sum < 0 -> reversed terms only (the forward area is ~4 pi);
//   omode 2: undecided -> both, as loop.go computes them.
// tcnt = fan triangles to evaluate (k_fan_area tasks).
__global__ void k_orient(int64_t n, const int32_t *kind, const int64_t *nslots, const int64_t *xoff, const V3 *xyz,
                         uint8_t *omode, int64_t *tcnt)
{
    const int64_t f = tid64();
    if (f >= n) return;
    const int nv = (int)nslots[f];
    if (kind[f] == DSSG_KIND_CIRCLE || nv < 3) {
        omode[f] = 2;
        tcnt[f] = 0;
        return;
    }
    const V3 *p = xyz + xoff[f];
    const V3 a = p[0];
    double d = 0, dabs = 0;
    bool near = true;
    V3 b = p[1];
    near &= a.x * b.x + a.y * b.y + a.z * b.z >= 0.99875;  // cos(0.05)
    // a simple fan: every triangle (v0, vi, vi+1) and every (v0, v1, vi)
    // robustly of one orientation -- the rays from v0 turn one way through
    // less than a half turn, so the loop is simple (star-shaped from v0)
    const V3 a1 = cross(a, b);
    constexpr double kE = 2 * DSS_MAX_DET_ERR;
    bool pos = true, neg = true;
    for (int i = 1; i + 1 < nv; i++) {
        const V3 c = p[i + 1];
        near &= a.x * c.x + a.y * c.y + a.z * c.z >= 0.99875;
        const double t = a.x * (b.y * c.z - b.z * c.y) + a.y * (b.z * c.x - b.x * c.z) + a.z * (b.x * c.y - b.y * c.x);
        const double u = a1.x * c.x + a1.y * c.y + a1.z * c.z;  // det(v0, v1, vi)
        pos &= (t > kE) & (u > kE);
        neg &= (t < -kE) & (u < -kE);
        d += t;
        dabs += __builtin_fabs(t);
        b = c;
    }
    d *= 0.5;
    dabs *= 0.5;
    const double margin = 0.05 * dabs + 1e-13;
    int m = 2;
    if (near && d > margin && ((d * 1.1) * DSS_EARTH_AREA_KM2) / 4.0 * DSS_PI < DSS_MAX_AREA_KM2) m = 0;  // = fan_area_km2
    else if (near && d < -margin) m = 1;
    // bits 2, 3: the loop is a simple counter-clockwise / clockwise fan
    // within 0.05 rad of v0 (k_setup skips the origin walk of a simple
    // counter-clockwise loop whose cap excludes OriginPoint)
    omode[f] = (uint8_t)(m | (near && pos ? 4 : 0) | (near && neg ? 8 : 0));
    tcnt[f] = (int64_t)(nv - 2) * (m == 2 ? 2 : 1);
}

// One thread per fan triangle (grid-stride over the T = toff[n] tasks of
// k_orient): the loop.go surfaceIntegralFloat64(SignedArea) term of the loop
// as given (fwd, slot i = triangle (v0, vi, vi+1)) or of its reversal (rev,
// triangle (v[n-1], v[n-1-i], v[n-2-i])), i = 1 .. n-2.  The fan origin never
// moves for loops whose vertices all lie within DSS_SURFACE_MAX_LENGTH of the
// origin; any other loop, or an undecided sign, goes to the exact
// per-footprint path (fan_fail).
__global__ void k_fan_area(const int64_t *toff_end, const uint32_t *towner, const int64_t *toff, const uint8_t *omode,
                           const int64_t *nslots, const int64_t *xoff, const V3 *xyz, double *fwd, double *rev,
                           uint8_t *fan_fail)
{
    const int64_t T = *toff_end;
    for (int64_t t = tid64(); t < T; t += (int64_t)gridDim.x * blockDim.x) {
        const uint32_t f = towner[t];
        const int n = (int)nslots[f];
        const int k = n - 2;
        int j = (int)(t - toff[f]);
        const int m = omode[f] & 3;
        const bool r = m == 1 || (m == 2 && j >= k);
        if (m == 2 && j >= k) j -= k;
        const int i = 1 + j;
        const V3 *p = xyz + xoff[f];
        const V3 a = r ? p[n - 1] : p[0], b = r ? p[n - 1 - i] : p[i], c = r ? p[n - 2 - i] : p[i + 1];
        bool fail = angle(c, a) > DSS_SURFACE_MAX_LENGTH;
        const double v = fastp::signed_area(a, b, c, fail);
        (r ? rev : fwd)[xoff[f] + i] = v;
        if (fail) fan_fail[f] = 1;
    }
}

#ifndef DSS_SETUP_BATCH
#define DSS_SETUP_BATCH 4
#endif
constexpr int kSetupBatch = DSS_SETUP_BATCH;  // k_setup's per-footprint loads in flight (fan terms, (u,v) bound)

// loop.go Area from the precomputed fan terms (same summation order as
// surfaceIntegralFloat64), then loopAreaKm2.  Fails over to the exact path
// in the bands where Area consults IsNormalized.
__device__ __forceinline__ double fan_area_km2(const double *t, int n, bool &fail, bool rev_only = false)
{
    // terms loaded kSetupBatch at a time, summed in index order (the order of
    // surfaceIntegralFloat64, so the sum is bit-identical)
    double area = 0;
    for (int i0 = 1; i0 + 1 < n; i0 += kSetupBatch) {
        double x[kSetupBatch];
#pragma unroll
        for (int u = 0; u < kSetupBatch; u++) x[u] = t[i0 + u + 1 < n ? i0 + u : i0];
#pragma unroll
        for (int u = 0; u < kSetupBatch; u++)
            if (i0 + u + 1 < n) area += x[u];
    }
    const double max_error = DSS_TURN_ANGLE_ERR_PER_VERTEX * (double)n;
    // omode 1 skipped the forward sum (~ -area): its IsNormalized band
    // (|sum| < max_error) is excluded with a wide margin instead
    if (rev_only) fail |= area < 100 * max_error;
    if (area < 0) area += 4 * DSS_PI;
    if (area > 4 * DSS_PI) area = 4 * DSS_PI;
    if (area < 0) area = 0;
    fail |= area < max_error || area > (4 * DSS_PI - max_error);
    return (area * DSS_EARTH_AREA_KM2) / 4.0 * DSS_PI;
}

// The tail both setups share: a small loop inside one face (u,v bound
// [ulo, uhi] x [vlo, vhi] on face0) gets planar containment unless the bound
// comes near OriginPoint's projection (see planar_contains), and its start
// block (as k_start would choose it), if small enough, becomes the direct
// candidates' frame (FL_FAST).  Returns the flags to OR in.
__device__ __forceinline__ uint8_t direct_frame(int64_t f, int face0, double ulo, double uhi, double vlo, double vhi,
                                                uint64_t *st_id, uint32_t *st_i, uint32_t *st_j, uint32_t *finfo,
                                                uint4 *fbox, bool write)
{
    uint8_t fl = 0;
    bool near_origin = false;
    if (face0 == xyz_face(origin_point())) {
        double ou, ov;
        valid_face_xyz_to_uv(face0, origin_point(), ou, ov);
        near_origin = ou >= ulo - 1e-6 && ou <= uhi + 1e-6 && ov >= vlo - 1e-6 && ov <= vhi + 1e-6;
    }
    if (!near_origin) fl |= FL_PLANAR;
    const double m = 1e-7;
    FaceBox b{ulo - m, uhi + m, vlo - m, vhi + m};
    uint64_t id[4];
    uint32_t ii[4], jj[4], mt[4];
    const int k = start_cells(b, face0, id, ii, jj, mt);
    const int L = meta_level(mt[0]);
    if (k > 0 && L >= kFastMinLevel) {
        fl |= FL_FAST;
        if (!write) return fl;
        uint32_t info = (uint32_t)L | ((uint32_t)k << 5);
        for (int q = 0; q < k; q++) {
            st_id[4 * f + q] = id[q];
            st_i[4 * f + q] = ii[q];
            st_j[4 * f + q] = jj[q];
            info |= (uint32_t)meta_orient(mt[q]) << (8 + 2 * q);
        }
        finfo[f] = info;
        // level-13 (i, j) range of the padded bound: candidates outside it
        // are > 1e-7 (uv) from every vertex, so neither touch an edge nor
        // lie inside this single-face loop
        const int sh13 = kMaxLevel - kCoverLevel;
        fbox[f] = make_uint4((uint32_t)(st_to_ij(uv_to_st(fmax(b.ulo, -1.0))) >> sh13),
                             (uint32_t)(st_to_ij(uv_to_st(fmin(b.uhi, 1.0))) >> sh13),
                             (uint32_t)(st_to_ij(uv_to_st(fmax(b.vlo, -1.0))) >> sh13),
                             (uint32_t)(st_to_ij(uv_to_st(fmin(b.vhi, 1.0))) >> sh13));
    }
    return fl;
}

// One thread per footprint, triage-only predicates (no out-of-line exact
// arithmetic, so no call-ABI spills).  A footprint the triage cannot decide
// is appended to slow_list and redone by k_setup_exact, which strides over
// that list only.
__device__ __forceinline__ void setup_one(int64_t f, uint32_t *slow_list, unsigned int *slow_n, const int32_t *kind,
                                          const int64_t *voff, const double *lat, const double *lng,
                                          const float *radius_m, const int64_t *xoff, const V3 *xyz, int32_t *status, double *area_out,
                                          uint8_t *mode, uint8_t *origin_in, uint8_t *fmask, uint8_t *flags,
                                          int32_t *nvx, const double2 *uv, uint64_t *st_id, uint32_t *st_i,
                                          uint32_t *st_j, uint32_t *finfo, uint4 *fbox, const double *fwd,
                                          const double *rev, const uint8_t *fan_fail, const uint8_t *not_inner,
                                          const uint8_t *omode, uint8_t *rev_out, const uint8_t *bad_in,
                                          const CircleFrame *frames, bool all_exact)
{
    bool fail = all_exact;  // (a test knob: every footprint through k_setup_exact)
    auto bail = [&]() {
        if (fail) {
            // redone by k_setup_exact (which sets the reversal flag itself);
            // until then k_edge_counts sees nothing here
            slow_list[atomicAdd(slow_n, 1u)] = (uint32_t)f;
            mode[f] = MODE_NONE;
            flags[f] = 0;
            rev_out[f] = 0;
        }
        return fail;
    };
    if (bail()) return;
    rev_out[f] = 0;
    const int k = kind[f];
    const int64_t v0 = voff[f];
    const V3 *p = xyz + xoff[f];
    int st = DSSG_ST_OK;
    uint8_t md = MODE_NONE;
    double area = 0;
    int nv = 0;
    bool small = false;
    LoopView l{p, 0, false};
    if (k == DSSG_KIND_CIRCLE) {
        const double la = lat[v0], ln = lng[v0];
        const float r = radius_m[f];
        if (la > 90.0 || la < -90.0 || ln > 180.0 || ln < -180.0) st = DSSG_ST_BAD_COORD_SET;
        else if (!(r > 0)) st = DSSG_ST_RADIUS;
        else {
            // regular_loop.go RegularLoop(center, DistanceMetersToAngle(r), 20):
            // k_circle_frames + k_verts wrote the vertices
            const double radius = (double)r / DSS_RADIUS_EARTH_M;
            nv = 20;
            l.n = 20;
            // RegularLoop is simple and lies in its cap (centre, radius):
            // OriginPoint clearly outside the cap is outside the loop, which
            // is what initOriginAndBound's crossing walk finds there (the
            // circles' walks were ~0.05 of k_setup's 0.37 ms on configs[2])
            const CircleFrame &F = frames[f];
            const V3 o = origin_point();
            const bool far = radius > 1e-7 && radius < 0.5 &&
                             F.c.x * o.x + F.c.y * o.y + F.c.z * o.z < F.z - 1e-6 * F.rr - 1e-12;  // angle > radius + 1e-6
            if (far) l.origin_inside = false;
            else fastp::loop_init_origin(l, fail);
            if (bail()) return;
            md = MODE_LOOP;
            small = radius < 0.5;
        }
    } else {
        nv = (int)(voff[f + 1] - v0);
        // Q17: range check (flagged per vertex by k_verts) precedes the count check
        if (k == DSSG_KIND_POLYGON && bad_in[f]) st = DSSG_ST_BAD_COORD_SET;
        if (st == DSSG_ST_OK && nv < 3) st = DSSG_ST_NOT_ENOUGH_POINTS;
        if (st == DSSG_ST_OK) {
            fail |= fan_fail[f] != 0;
            l.n = nv;
            const int om = omode[f] & 3;  // k_orient: which fan terms exist
            // a simple loop within 0.05 rad of v0 (k_orient) is inside its
            // cap, so OriginPoint outside the cap is outside the loop once it
            // runs counter-clockwise -- initOriginAndBound's walk finds
            // "outside" there; the walk is skipped for the loop as given
            // (simple ccw) or for its reversal (simple cw)
            bool skip_fwd = false, skip_rev = false;
            const int sf = omode[f] >> 2;
            if (sf) {
                const V3 o = origin_point(), q = p[0];
                const bool ofar = q.x * o.x + q.y * o.y + q.z * o.z < 0.99875 - 1e-6;
                skip_fwd = ofar && (sf & 1);
                skip_rev = ofar && (sf & 2);
            }
            if (om == 1) {
                area = INFINITY;  // the forward sum is negative: ~4 pi, above the cap
            } else {
                if (skip_fwd) l.origin_inside = false;
                else fastp::loop_init_origin(l, fail);
                area = fan_area_km2(fwd + xoff[f], nv, fail);
            }
            if (om == 0 && area > DSS_MAX_AREA_KM2) fail = true;  // mispredicted: no reversed terms
            if (bail()) return;
            if (area > DSS_MAX_AREA_KM2) {
                // Q4's in-place reversal through a reversed view (LoopView.rev):
                // later kernels read it through rev_out, and k_reverse_list
                // moves only the descent footprints' vertices -- this thread's
                // serial walk of them cost 0.16 of k_setup's 0.55 ms on
                // configs[2]
                l.rev = true;
                rev_out[f] = 1;
                if (skip_rev) l.origin_inside = false;
                else fastp::loop_init_origin(l, fail);
                area = fan_area_km2(rev + xoff[f], nv, fail, om == 1);
                if (bail()) return;
            }
            if (area > DSS_MAX_AREA_KM2) st = DSSG_ST_AREA_TOO_LARGE;
            else if (area <= 0) md = MODE_POLYLINE;  // Q3: open polyline, no closing edge
            else { md = MODE_LOOP; small = true; }
        }
    }
    uint8_t mask = 0;
    bool inner = true;
    if (md == MODE_LOOP && !not_inner[f]) {  // k_fan: every edge lies inside the face of vertex 0
        mask = (uint8_t)(1u << xyz_face(p[0]));
    } else if (md != MODE_NONE) {
        const int ne = md == MODE_LOOP ? nv : nv - 1;
        const int face0 = xyz_face(p[0]);
        for (int e = 0; e < ne; e++) {
            const V3 a = p[e], b = p[(e + 1) % nv];
            if (edge_inside_face(a, b, face0)) { mask |= (uint8_t)(1u << face0); continue; }
            inner = false;
            for (int fc = 0; fc < 6; fc++) {
                double w[4];
                if (clip_to_padded_face(a, b, fc, kCoarsePad, w)) mask |= (uint8_t)(1u << fc);
            }
        }
        if (md == MODE_POLYLINE) {
            for (int i = 0; i < nv; i++)
                for (int fc = 0; fc < 6; fc++) {
                    double u, v;
                    if (face_xyz_to_uv(fc, p[i], u, v) && __builtin_fabs(u) <= 1 + kCoarsePad &&
                        __builtin_fabs(v) <= 1 + kCoarsePad)
                        mask |= (uint8_t)(1u << fc);
                }
        }
    }
    status[f] = st;
    area_out[f] = area;
    mode[f] = md;
    origin_in[f] = l.origin_inside ? 1 : 0;
    fmask[f] = mask;
    // bbox-limited start (per touched face, the bound of the edges clipped to
    // it) is valid for polylines (no interior) and for loops whose interior is
    // the small side: a small loop's part of a face is bounded by its clipped
    // edges and the face-boundary pieces between their clip points, which lie
    // in those points' bound (a face corner inside the part included, since
    // the part's boundary then reaches both face edges through it).
    uint8_t fl = (md == MODE_POLYLINE || (md == MODE_LOOP && small)) ? FL_SMALL : 0;
    if (md == MODE_LOOP && small && inner && __builtin_popcount(mask) == 1) {
        const double2 *uvp = uv + xoff[f];  // projected by k_fan
        double ulo = 1e300, uhi = -1e300, vlo = 1e300, vhi = -1e300;
        for (int i0 = 0; i0 < nv; i0 += kSetupBatch) {  // (a batch's loads in flight together; repeats are harmless)
            double2 w[kSetupBatch];
#pragma unroll
            for (int u = 0; u < kSetupBatch; u++) w[u] = uvp[i0 + u < nv ? i0 + u : i0];
#pragma unroll
            for (int u = 0; u < kSetupBatch; u++) {
                ulo = fmin(ulo, w[u].x); uhi = fmax(uhi, w[u].x); vlo = fmin(vlo, w[u].y); vhi = fmax(vhi, w[u].y);
            }
        }
        fl |= direct_frame(f, xyz_face(p[0]), ulo, uhi, vlo, vhi, st_id, st_i, st_j, finfo, fbox, true);
    }
    flags[f] = fl;
    nvx[f] = nv;
}

#ifndef DSS_SETUP_WPE
#define DSS_SETUP_WPE 1
#endif
constexpr int kSetupBlock = 64;  // (256-thread blocks: 0.306 -> 0.315 ms, profiles/r07n)
__global__ __launch_bounds__(kSetupBlock) __attribute__((amdgpu_waves_per_eu(DSS_SETUP_WPE))) void k_setup(
    uint32_t *slow_list, unsigned int *slow_n, int64_t n, const int32_t *kind, const int64_t *voff, const double *lat,
    const double *lng, const float *radius_m, const int64_t *xoff, const V3 *xyz, int32_t *status, double *area_out, uint8_t *mode,
    uint8_t *origin_in, uint8_t *fmask, uint8_t *flags, int32_t *nvx, const double2 *uv, uint64_t *st_id,
    uint32_t *st_i, uint32_t *st_j, uint32_t *finfo, uint4 *fbox, const double *fwd, const double *rev,
    const uint8_t *fan_fail, const uint8_t *not_inner, const uint8_t *omode, const uint32_t *perm, uint8_t *rev_out,
    const uint8_t *bad_in, const CircleFrame *frames, int all_exact)
{
    const int64_t t = tid64();
    if (t >= n) return;
    // polygons first, then circles: waves run one kind's path
    setup_one(perm[t], slow_list, slow_n, kind, voff, lat, lng, radius_m, xoff, xyz, status, area_out, mode, origin_in,
              fmask, flags, nvx, uv, st_id, st_i, st_j, finfo, fbox, fwd, rev, fan_fail, not_inner, omode, rev_out,
              bad_in, frames, all_exact != 0);
}

// ---------------------------------------------------------------------------
// The exact setup of the footprints the triage left undecided, one wave per
// listed footprint: setup_one's steps with the exact predicates of
// loopdev.cuh / s2dev.cuh (loop.go as written, no shortcuts), the per-vertex
// and per-edge loops spread over the lanes.
//  * Vertices: k_verts' S2 points (the same expressions as PointFromLatLng /
//    RegularLoop, -ffp-contract=off).
//  * The origin walk (initOriginAndBound -> bruteForceContainsPoint): each
//    lane tests its edges with a fresh EdgeCrosser restarted at the edge's
//    first vertex.  The chain's cached orientation of that vertex is the
//    same triage sign or its exact resolution, and every branch that reads
//    an undecided one resolves it the same way, so each edge's verdict is
//    the chain's; the wave counts the crossings by ballot.
//  * Area (surfaceIntegralFloat64(SignedArea)): when every vertex lies
//    within maxLength of v0 the fan origin never moves; the lanes compute
//    the terms and the wave sums them in index order -- the serial sum, bit
//    for bit.  Otherwise (and for IsNormalized's bands) the serial code.
//  * Q4's reversal through the reversed view and rev_out, as k_setup does.
//  * The face mask: edges over the lanes, bits OR-ed by ballot.
// One lane's serial exact walk of one footprint cost ~0.09 ms per configs[2]
// covering (profiles/r05ao), the whole GPU waiting on it.
__device__ bool wave_loop_contains(const LoopView &l, V3 pt, int lane)
{
    int cnt = 0;
    for (int i0 = 1; i0 <= l.n; i0 += 64) {
        const int i = i0 + lane;
        bool x = false;
        if (i <= l.n) {
            EdgeCrosser e;
            e.init(origin_point(), pt);
            e.restart_at(l.vertex(i - 1));
            x = e.edge_or_vertex_chain_crossing(l.vertex(i));
        }
        cnt += __popcll(__ballot(x));
    }
    return l.origin_inside != ((cnt & 1) != 0);
}

__device__ void wave_init_origin(LoopView &l, int lane)
{
    const V3 v0 = l.at(0), v1 = l.at(1), v2 = l.at(2);
    const bool v1_inside = !eq(v0, v1) && !eq(v2, v1) && angle_contains_vertex(v0, v1, v2);
    l.origin_inside = false;
    if (v1_inside != wave_loop_contains(l, v1, lane)) l.origin_inside = true;
}

// (the rare serial pieces out of line: inlined, they pushed the kernel to
// 256 VGPRs and scratch)
__device__ __noinline__ double serial_area_sum(const LoopView l) { return loop_signed_area_sum(l); }
__device__ __noinline__ bool serial_is_normalized(const LoopView l) { return loop_is_normalized(l); }
__device__ __noinline__ uint32_t clip_face_mask(V3 a, V3 b)
{
    uint32_t m = 0;
    for (int fc = 0; fc < 6; fc++) {
        double w4[4];
        if (clip_to_padded_face(a, b, fc, kCoarsePad, w4)) m |= 1u << fc;
    }
    return m;
}

// loop.go Area, then loopAreaKm2 (Q1)
__device__ double wave_area_km2(const LoopView &l, int lane)
{
    const int n = l.n;
    const V3 v0 = l.vertex(0);
    bool moves = false;
    for (int i = 2 + lane; i < n; i += 64) moves |= angle(l.vertex(i), v0) > DSS_SURFACE_MAX_LENGTH;
    double area = 0;
    if (__ballot(moves)) {
        area = serial_area_sum(l);  // (every lane: the serial walk)
    } else {
        for (int i0 = 1; i0 + 1 < n; i0 += 64) {
            const int i = i0 + lane;
            const double t = i + 1 < n ? signed_area(v0, l.vertex(i), l.vertex(i + 1)) : 0.0;
            const int cnt = min(64, n - 1 - i0);
            for (int u = 0; u < cnt; u++) area += __shfl(t, u);
        }
    }
    const double max_error = turning_angle_max_error(l);
    if (area < 0) area += 4 * DSS_PI;
    if (area > 4 * DSS_PI) area = 4 * DSS_PI;
    if (area < 0) area = 0;
    if (area < max_error && !serial_is_normalized(l)) area = 4 * DSS_PI;
    else if (area > (4 * DSS_PI - max_error) && serial_is_normalized(l)) area = 0;
    return (area * DSS_EARTH_AREA_KM2) / 4.0 * DSS_PI;
}

__device__ __forceinline__ double wave_min_d(double x)
{
    for (int o = 32; o > 0; o >>= 1) x = fmin(x, __shfl_xor(x, o));
    return x;
}
__device__ __forceinline__ double wave_max_d(double x)
{
    for (int o = 32; o > 0; o >>= 1) x = fmax(x, __shfl_xor(x, o));
    return x;
}

// k_setup_exact's fixed grid (4 x 64 threads measured the same, profiles/r07e)
constexpr int kExactGrid = 16, kExactBlock = 256;
__global__ __launch_bounds__(kExactBlock) void k_setup_exact(const uint32_t *slow_list, const unsigned int *slow_n,
                                                     const int32_t *kind, const int64_t *voff, const double *lat,
                                                     const double *lng, const float *radius_m, const int64_t *xoff,
                                                     const V3 *xyz, int32_t *status, double *area_out, uint8_t *mode,
                                                     uint8_t *origin_in, uint8_t *fmask, uint8_t *flags, int32_t *nvx,
                                                     const double2 *uv, uint64_t *st_id, uint32_t *st_i,
                                                     uint32_t *st_j, uint32_t *finfo, uint4 *fbox, uint8_t *rev_out,
                                                     const uint8_t *bad_in)
{
    const int lane = threadIdx.x & 63;
    const unsigned int ns = *slow_n;
    const int64_t nw = (int64_t)gridDim.x * (blockDim.x / 64);
    for (int64_t w = (int64_t)blockIdx.x * (blockDim.x / 64) + (threadIdx.x >> 6); w < (int64_t)ns; w += nw) {
        const int64_t f = slow_list[w];
        const int k = kind[f];
        const int64_t v0 = voff[f];
        int st = DSSG_ST_OK;
        uint8_t md = MODE_NONE;
        double area = 0;
        int nv = 0;
        bool small = false;
        LoopView l{xyz + xoff[f], 0, false};
        if (k == DSSG_KIND_CIRCLE) {
            const double la = lat[v0], ln = lng[v0];
            const float r = radius_m[f];
            if (la > 90.0 || la < -90.0 || ln > 180.0 || ln < -180.0) st = DSSG_ST_BAD_COORD_SET;
            else if (!(r > 0)) st = DSSG_ST_RADIUS;
            else {
                nv = l.n = 20;
                wave_init_origin(l, lane);
                md = MODE_LOOP;
                small = (double)r / DSS_RADIUS_EARTH_M < 0.5;
            }
        } else {
            nv = (int)(voff[f + 1] - v0);
            if (k == DSSG_KIND_POLYGON && bad_in[f]) st = DSSG_ST_BAD_COORD_SET;  // Q17
            if (st == DSSG_ST_OK && nv < 3) st = DSSG_ST_NOT_ENOUGH_POINTS;
            if (st == DSSG_ST_OK) {
                l.n = nv;
                // (the origin first, as the loop's construction runs it: Area's
                // IsNormalized bands read it through the pole containment)
                wave_init_origin(l, lane);
                area = wave_area_km2(l, lane);
                if (area > DSS_MAX_AREA_KM2) {  // Q4
                    l.rev = true;
                    wave_init_origin(l, lane);
                    area = wave_area_km2(l, lane);
                }
                if (area > DSS_MAX_AREA_KM2) st = DSSG_ST_AREA_TOO_LARGE;
                else if (area <= 0) md = MODE_POLYLINE;  // Q3
                else { md = MODE_LOOP; small = true; }
            }
        }
        uint32_t m = 0;
        bool out = false;
        if (md != MODE_NONE) {
            const int ne = md == MODE_LOOP ? nv : nv - 1;
            const int face0 = xyz_face(l.at(0));
            for (int e = lane; e < ne; e += 64) {
                const V3 a = l.at(e), b = l.at(e + 1 < nv ? e + 1 : 0);
                if (edge_inside_face(a, b, face0)) { m |= 1u << face0; continue; }
                out = true;
                m |= clip_face_mask(a, b);
            }
            if (md == MODE_POLYLINE)
                for (int i = lane; i < nv; i += 64)
                    for (int fc = 0; fc < 6; fc++) {
                        double u, v;
                        if (face_xyz_to_uv(fc, l.at(i), u, v) && __builtin_fabs(u) <= 1 + kCoarsePad &&
                            __builtin_fabs(v) <= 1 + kCoarsePad)
                            m |= 1u << fc;
                    }
        }
        uint8_t mask = 0;
        for (int fc = 0; fc < 6; fc++)
            if (__ballot((m >> fc) & 1u)) mask |= (uint8_t)(1u << fc);
        const bool inner = __ballot(out) == 0ull;
        uint8_t fl = (md == MODE_POLYLINE || (md == MODE_LOOP && small)) ? FL_SMALL : 0;
        if (md == MODE_LOOP && small && inner && __builtin_popcount(mask) == 1) {
            // (u,v) images on the face of vertex 0 (k_fan's, memory order: the
            // loop's one face whichever way it runs)
            const double2 *uvp = uv + xoff[f];
            double ulo = 1e300, uhi = -1e300, vlo = 1e300, vhi = -1e300;
            for (int i = lane; i < nv; i += 64) {
                const double2 w2 = uvp[i];
                ulo = fmin(ulo, w2.x); uhi = fmax(uhi, w2.x); vlo = fmin(vlo, w2.y); vhi = fmax(vhi, w2.y);
            }
            ulo = wave_min_d(ulo); uhi = wave_max_d(uhi); vlo = wave_min_d(vlo); vhi = wave_max_d(vhi);
            fl |= direct_frame(f, xyz_face(l.at(0)), ulo, uhi, vlo, vhi, st_id, st_i, st_j, finfo, fbox, lane == 0);
        }
        if (lane == 0) {
            status[f] = st;
            area_out[f] = area;
            mode[f] = md;
            origin_in[f] = l.origin_inside ? 1 : 0;
            fmask[f] = mask;
            flags[f] = fl;
            nvx[f] = nv;
            rev_out[f] = l.rev ? 1 : 0;
        }
    }
}

// Q4's in-place reversal, moved out of k_setup<true> (its serial walk of a
// lane's own footprint cost 0.16 of its 0.55 ms on configs[2]): the direct
// candidate kernels read a reversed loop through the rev flag (LoopView.rev,
// mirrored (u,v) staging), so only the descent footprints -- a few per batch,
// read by many kernels -- are reversed in memory here, one wave per listed
// footprint, lanes over its vertex pairs.
__global__ void k_reverse_list(const uint32_t *dlist, const unsigned int *dlist_n, const int64_t *xoff,
                               const int32_t *nvx, const uint8_t *rev_flag, V3 *xyz, double2 *uv)
{
    const unsigned int nl = *dlist_n;
    const int lane = threadIdx.x & 63;
    const int64_t nw = (int64_t)gridDim.x * (blockDim.x / 64);
    for (int64_t wi = (int64_t)blockIdx.x * (blockDim.x / 64) + (threadIdx.x >> 6); wi < (int64_t)nl; wi += nw) {
        const uint32_t f = dlist[wi];
        if (!rev_flag[f]) continue;
        const int64_t x0 = xoff[f];
        const int n = nvx[f];
        for (int i = lane; i < n / 2; i += 64) {
            const int64_t x = x0 + i, y = x0 + (n - 1 - i);
            const V3 a = xyz[x], b = xyz[y];
            xyz[x] = b;
            xyz[y] = a;
            const double2 c = uv[x], d = uv[y];
            uv[x] = d;
            uv[y] = c;
        }
    }
}

__device__ __forceinline__ int num_edges(uint8_t md, int nv) { return md == MODE_LOOP ? nv : (md == MODE_POLYLINE ? nv - 1 : 0); }

// Per footprint its clipped-edge items (descent footprints only), and the
// list of descent footprints (any order; one atomic per wave).
__global__ void k_edge_counts(int64_t n, const uint8_t *mode, const uint8_t *fmask, const uint8_t *flags, const int32_t *nvx,
                              int64_t *cnt, uint32_t *dlist, unsigned int *dlist_n)
{
    const int64_t f = tid64();
    bool desc = false;
    if (f < n) {
        desc = !(flags[f] & FL_FAST) && mode[f] != MODE_NONE;
        cnt[f] = desc ? (int64_t)__builtin_popcount(fmask[f]) * num_edges(mode[f], nvx[f]) : 0;
    }
    const unsigned long long m = __ballot(desc);
    if (!m) return;
    const int lane = threadIdx.x & 63, leader = __builtin_ctzll(m);
    unsigned int b = 0;
    if (lane == leader) b = atomicAdd(dlist_n, (unsigned int)__popcll(m));
    b = (unsigned int)__shfl((int)b, leader);
    if (desc) dlist[b + cmpct::lanes_below(m)] = (uint32_t)f;
}

// Clip every edge to every touched face (ascending face order), one thread
// per (footprint, touched face, edge) item: the few multi-face / big /
// polyline footprints of a batch carry up to 6 x 20 clips each, which one
// thread per footprint walked serially (0.17 ms on configs[2]).
__global__ void k_clip_items(int64_t ne_all, const uint32_t *eown, const int64_t *xoff, const V3 *xyz,
                             const uint8_t *mode, const uint8_t *fmask, const int32_t *nvx, const int64_t *eoff,
                             double4 *clip_f, double4 *clip_c, uint8_t *cflags)
{
    const int64_t k = tid64();
    if (k >= ne_all) return;
    const uint32_t f = eown[k];
    const int nv = nvx[f], ne = num_edges(mode[f], nv);
    const int64_t local = k - eoff[f];
    const int fi = (int)(local / ne), e = (int)(local - (int64_t)fi * ne);
    uint32_t fm = fmask[f];
    for (int q = 0; q < fi; q++) fm &= fm - 1;  // the fi-th touched face, ascending
    const int fc = __builtin_ctz(fm);
    const V3 *p = xyz + xoff[f];
    const V3 a = p[e], b = p[(e + 1) % nv];
    double uf[4], uc[4];
    const bool okf = clip_to_padded_face(a, b, fc, kFinePad, uf);
    const bool okc = clip_to_padded_face(a, b, fc, kCoarsePad, uc);
    clip_f[k] = make_double4(uf[0], uf[1], uf[2], uf[3]);
    clip_c[k] = make_double4(uc[0], uc[1], uc[2], uc[3]);
    cflags[k] = (uint8_t)((okf ? 1 : 0) | (okc ? 2 : 0));
}

// Face-cell id for face fc (level 0).
__device__ __forceinline__ uint64_t face_cell(int fc) { return ((uint64_t)fc << 61) | (1ull << 60); }

__device__ V3 node_center(int face, uint32_t i0, uint32_t j0, int level)
{
    // cellid.go faceSiTi / rawPoint: centre in (si, ti) = 2*i0 + size, exact.
    double size = (double)(1u << (kMaxLevel - level));
    const double half = 0.5 / (double)kMaxSize;
    double s = half * (2.0 * (double)i0 + size), t = half * (2.0 * (double)j0 + size);
    return normalize(face_uv_to_xyz(face, st_to_uv(s), st_to_uv(t)));
}

// Containment of a node centre that no loop edge comes near (the node is
// uniform, or a level-13 cell the padded edge test rejected): the centre is
// at least half a cell from every edge, so for a loop that lies inside one
// face the even-odd ray cast over the edges' gnomonic (u,v) images (great
// circles are straight lines there) decides it exactly.  Crossing parity is
// path independent, so it equals the parity S2 counts along OriginPoint->p
// (loop.go bruteForceContainsPoint), flipped by originInside; FL_PLANAR
// excludes loops whose bound surrounds OriginPoint's own projection.
__device__ __forceinline__ bool planar_contains(bool origin_inside, const double4 *clip, int ne, uint32_t i0, uint32_t j0,
                                                int level)
{
    double size = (double)(1u << (kMaxLevel - level));
    const double half = 0.5 / (double)kMaxSize;
    double uc = st_to_uv(half * (2.0 * (double)i0 + size)), vc = st_to_uv(half * (2.0 * (double)j0 + size));
    bool par = false;
    for (int e = 0; e < ne; e++) {
        double4 c = clip[e];
        if ((c.y > vc) != (c.w > vc)) {
            double x = c.x + (vc - c.y) * (c.z - c.x) / (c.w - c.y);
            if (uc < x) par = !par;
        }
    }
    return origin_inside != par;
}

// Count (pass 0) or write (pass 1) start nodes; big loops also get whole-face
// nodes for faces without edges whose centre the loop contains.
// A small descent footprint's start cell whose level-13 cells inside the
// footprint's per-face bound become start nodes at once (k_start13).
struct StartDesc {
    uint64_t id;   // the start cell
    int64_t w;     // its first output node
    uint32_t f, i, j, meta;
    uint4 box;     // the bound's level-13 (i0, i1, j0, j1)
};

template <int PASS>
__global__ __launch_bounds__(64) void k_start(int64_t nd, const uint32_t *dlist, const int64_t *xoff, const V3 *xyz, const uint8_t *mode, const uint8_t *fmask,
                        const uint8_t *flags, const uint8_t *origin_in, const int32_t *nvx, const int64_t *eoff,
                        const double4 *clip_c, const uint8_t *cflags, int64_t *cnt, const int64_t *soff,
                        uint32_t *nf, uint64_t *nid, uint32_t *ni, uint32_t *nj, uint32_t *nmeta, StartDesc *sdesc,
                        unsigned int *sdesc_n, unsigned int *xlist_n)
{
    const int64_t k = tid64();
    if (PASS == 0 && k == 0) *sdesc_n = *xlist_n = 0u;  // (pass 1 appends to the first, the descent to the second)
    if (k >= nd) return;
    const int64_t f = dlist[k];  // a descent footprint (k_edge_counts)
    uint8_t md = mode[f];
    int64_t c = 0;
    if (md != MODE_NONE && !(flags[f] & FL_FAST)) {
        int nv = nvx[f], ne = num_edges(md, nv);
        const V3 *p = xyz + xoff[f];
        LoopView l{p, nv, origin_in[f] != 0};
        int64_t w = PASS ? soff[f] : 0;
        int fi = 0;
        for (int fc = 0; fc < 6; fc++) {
            bool touched = (fmask[f] >> fc) & 1;
            if (!touched) {
                if (md == MODE_LOOP && !(flags[f] & FL_SMALL)) {
                    V3 ctr = node_center(fc, 0, 0, 0);
                    if (loop_contains(l, ctr)) {
                        if (PASS) {
                            nf[w] = (uint32_t)f; nid[w] = face_cell(fc); ni[w] = 0; nj[w] = 0;
                            nmeta[w] = pack_meta(0, fc & 1, 1, fc);
                            w++;
                        }
                        c++;
                    }
                }
                continue;
            }
            if (flags[f] & FL_SMALL) {
                FaceBox b;
                if (face_box(p, nv, md, clip_c, cflags, eoff[f] + (int64_t)fi * ne, ne, b, fc)) {
                    uint64_t id[4];
                    uint32_t ii[4], jj[4], mt[4];
                    int k = start_cells(b, fc, id, ii, jj, mt);
                    const int L = k > 0 ? meta_level(mt[0]) : 0;
                    if (k > 0 && L >= kFastMinLevel && L < kCoverLevel) {
                        // a small bound (<= 4 x 4^(13 - L) level-13 cells):
                        // its level-13 cells are the start nodes, in id order
                        // (start cells by id, Hilbert order inside each), so
                        // the descent decides them in one level instead of
                        // walking down from L -- every cell that can
                        // intersect the face part lies in the bound
                        const int sh13 = kMaxLevel - kCoverLevel;
                        const uint32_t i0 = (uint32_t)st_to_ij(uv_to_st(fmax(b.ulo, -1.0))) >> sh13,
                                       i1 = (uint32_t)st_to_ij(uv_to_st(fmin(b.uhi, 1.0))) >> sh13;
                        const uint32_t j0 = (uint32_t)st_to_ij(uv_to_st(fmax(b.vlo, -1.0))) >> sh13,
                                       j1 = (uint32_t)st_to_ij(uv_to_st(fmin(b.vhi, 1.0))) >> sh13;
                        // (the start cells cover the bound's cells: the
                        // count is the rectangle's; the write pass walks
                        // each start cell's Hilbert order, skipping every
                        // subtree outside the rectangle)
                        // (the start cells cover the bound's cells: each
                        // start cell's share is its intersection with the
                        // rectangle; k_start13 writes them, a wave per start
                        // cell, in Hilbert order)
                        const uint32_t span = 1u << (kCoverLevel - L);
                        for (int q = 0; q < k; q++) {
                            const uint32_t a0 = ii[q] >> sh13, b0 = jj[q] >> sh13;
                            const uint32_t x0 = max(a0, i0), x1 = min(a0 + span - 1, i1);
                            const uint32_t y0 = max(b0, j0), y1 = min(b0 + span - 1, j1);
                            const int64_t cq = x1 >= x0 && y1 >= y0 ? (int64_t)(x1 - x0 + 1) * (y1 - y0 + 1) : 0;
                            if (PASS && cq > 0) {
                                StartDesc sd;
                                sd.id = id[q];
                                sd.w = w;
                                sd.f = (uint32_t)f;
                                sd.i = ii[q];
                                sd.j = jj[q];
                                sd.meta = mt[q];
                                sd.box = make_uint4(i0, i1, j0, j1);
                                sdesc[atomicAdd(sdesc_n, 1u)] = sd;
                                w += cq;
                            }
                            c += cq;
                        }
                    } else {
                        if (PASS)
                            for (int q = 0; q < k; q++, w++) {
                                nf[w] = (uint32_t)f; nid[w] = id[q]; ni[w] = ii[q]; nj[w] = jj[q]; nmeta[w] = mt[q];
                            }
                        c += k;
                    }
                }
            } else {
                if (PASS) {
                    nf[w] = (uint32_t)f; nid[w] = face_cell(fc); ni[w] = 0; nj[w] = 0;
                    nmeta[w] = pack_meta(0, fc & 1, 0, fc);
                    w++;
                }
                c++;
            }
            fi++;
        }
    }
    if (!PASS) cnt[f] = c;
}

// The level-13 start nodes of k_start's listed start cells: a wave per start
// cell, lanes over its 4^(13 - L) descendants in Hilbert (= id) order, the
// ones inside the bound written contiguously from the cell's first node.
__global__ __launch_bounds__(256) void k_start13(const StartDesc *sdesc, const unsigned int *sdesc_n, uint32_t *nf,
                                                 uint64_t *nid, uint32_t *ni, uint32_t *nj, uint32_t *nmeta)
{
    const unsigned int n = *sdesc_n;
    const int lane = threadIdx.x & 63;
    const int64_t nw = (int64_t)gridDim.x * (blockDim.x / 64);
    const int sh13 = kMaxLevel - kCoverLevel;
    const uint64_t lsb13 = lsb_for_level(kCoverLevel);
    for (int64_t d = (int64_t)blockIdx.x * (blockDim.x / 64) + (threadIdx.x >> 6); d < (int64_t)n; d += nw) {
        const StartDesc sd = sdesc[d];
        const int L = meta_level(sd.meta), fc = meta_face(sd.meta);
        const uint32_t nd13 = 1u << (2 * (kCoverLevel - L));
        const uint64_t lsbL = lsb_for_level(L);
        int64_t w = sd.w;
        for (uint32_t r0 = 0; r0 < nd13; r0 += 64) {
            const uint32_t r = r0 + (uint32_t)lane;
            int o = meta_orient(sd.meta);
            uint32_t ci = sd.i, cj = sd.j;
            for (int l = L + 1; l <= kCoverLevel; l++) {
                const int digit = (int)((r >> (2 * (kCoverLevel - l))) & 3u);
                const int ij = pos_to_ij(o, digit);
                const uint32_t half = 1u << (kMaxLevel - l);
                if (ij >> 1) ci += half;
                if (ij & 1) cj += half;
                o ^= pos_to_orientation(digit);
            }
            const uint32_t c13 = ci >> sh13, d13 = cj >> sh13;
            const bool in = r < nd13 && c13 >= sd.box.x && c13 <= sd.box.y && d13 >= sd.box.z && d13 <= sd.box.w;
            const unsigned long long m = __ballot(in);
            if (in) {
                const int64_t p = w + (int64_t)cmpct::lanes_below(m);
                nf[p] = sd.f;
                nid[p] = sd.id - lsbL + lsb13 + (uint64_t)r * (lsb13 << 1);
                ni[p] = ci;
                nj[p] = cj;
                nmeta[p] = pack_meta(kCoverLevel, o, 0, fc);
            }
            w += (int64_t)__popcll(m);
        }
    }
}

// golang/geo polyline.go Polyline.IntersectsCell for a level-13 node.
__device__ bool polyline_intersects_cell(const V3 *p, int nv, int face, double ulo, double uhi, double vlo, double vhi)
{
    if (nv == 0) return false;
    const double m = DSS_DBL_EPS;  // cell.go ContainsPoint: uv bound expanded by dblEpsilon
    for (int i = 0; i < nv; i++) {
        double u, v;
        if (face_xyz_to_uv(face, p[i], u, v) && (ulo - m) <= u && u <= (uhi + m) && (vlo - m) <= v && v <= (vhi + m))
            return true;
    }
    V3 cv[4] = {normalize(face_uv_to_xyz(face, ulo, vlo)), normalize(face_uv_to_xyz(face, uhi, vlo)),
                normalize(face_uv_to_xyz(face, uhi, vhi)), normalize(face_uv_to_xyz(face, ulo, vhi))};
    for (int j = 0; j < 4; j++) {
        EdgeCrosser e;
        e.init(cv[j], cv[(j + 1) & 3]);
        e.restart_at(p[0]);
        for (int i = 1; i < nv; i++)
            if (e.chain_crossing_sign(p[i]) != DO_NOT_CROSS) return true;
    }
    return false;
}

// Classify each frontier node: 0 drop, 1 keep (done), 2 subdivide (4 children).
// The exact S2 paths (centre containment of a non-planar loop, a polyline's
// level-13 cell test) are deferred to k_expand_exact through a list, so this
// kernel does not carry their registers (248 VGPRs, 2 waves per SIMD, when
// they were inlined) for the planar majority.
__global__ __launch_bounds__(64) void k_expand_count(int64_t nn, const uint32_t *nf, const uint32_t *ni, const uint32_t *nj,
                               const uint32_t *nmeta, uint8_t *act, int64_t *cnt, const int64_t *xoff, const V3 *xyz,
                               const uint8_t *mode, const uint8_t *fmask, const uint8_t *origin_in, const int32_t *nvx,
                               const int64_t *eoff, const double4 *clip_f, const double4 *clip_c, const uint8_t *cflags,
                               const uint8_t *flags, uint32_t *xlist, unsigned int *xlist_n, int *any_open)
{
    const int64_t k = tid64();
    if (k == 0) *any_open = 0;  // (set by this level's k_expand_write)
    bool defer = false;
    if (k < nn) {
        const uint32_t m = nmeta[k];
        uint8_t a = 0;
        if (meta_done(m)) {
            a = 1;
        } else {
            const uint32_t f = nf[k];
            const int level = meta_level(m), face = meta_face(m);
            const uint8_t md = mode[f];
            const int nv = nvx[f], ne = num_edges(md, nv);
            const uint8_t mask = fmask[f];
            const int fi = __builtin_popcount((unsigned)mask & ((1u << face) - 1u));
            const int64_t base = eoff[f] + (int64_t)fi * ne;
            const uint32_t size = 1u << (kMaxLevel - level);
            const double ulo = st_to_uv((double)ni[k] / (double)kMaxSize),
                         uhi = st_to_uv((double)(ni[k] + size) / (double)kMaxSize);
            const double vlo = st_to_uv((double)nj[k] / (double)kMaxSize),
                         vhi = st_to_uv((double)(nj[k] + size) / (double)kMaxSize);
            const bool planar = (flags[f] & FL_PLANAR) != 0;
            // coarse test: a clipped edge (or a polyline vertex) within the
            // coarse padding of the node; a node it misses meets nothing
            auto coarse_hit = [&]() {
                const double pm = kCoarsePad;
                bool hit = false;
                for (int e = 0; e < ne && !hit; e++) {
                    if (!(cflags[base + e] & 2)) continue;
                    const double4 c = clip_c[base + e];
                    hit = edge_intersects_rect(c.x, c.y, c.z, c.w, ulo - pm, uhi + pm, vlo - pm, vhi + pm);
                }
                if (!hit && md == MODE_POLYLINE) {
                    const V3 *p = xyz + xoff[f];
                    for (int i = 0; i < nv && !hit; i++) {
                        double u, v;
                        hit = face_xyz_to_uv(face, p[i], u, v) && (ulo - pm) <= u && u <= (uhi + pm) && (vlo - pm) <= v &&
                              v <= (vhi + pm);
                    }
                }
                return hit;
            };
            if (level < kCoverLevel) {
                const bool hit = coarse_hit();
                if (hit) a = 2;
                else if (md == MODE_LOOP) {
                    if (planar) a = planar_contains(origin_in[f] != 0, clip_f + base, ne, ni[k], nj[k], level) ? 1 : 0;
                    else defer = true;
                } else a = 0;
            } else if (md == MODE_LOOP) {
                // loop.go IntersectsCell: padded edge test, else centre containment
                const double pm = kFinePad;
                bool in = false;
                for (int e = 0; e < ne && !in; e++) {
                    if (!(cflags[base + e] & 1)) continue;
                    const double4 c = clip_f[base + e];
                    in = edge_intersects_rect(c.x, c.y, c.z, c.w, ulo - pm, uhi + pm, vlo - pm, vhi + pm);
                }
                if (in) a = 1;
                else if (planar) a = planar_contains(origin_in[f] != 0, clip_f + base, ne, ni[k], nj[k], level) ? 1 : 0;
                else defer = true;
            } else if (coarse_hit()) {
                defer = true;  // polyline.go IntersectsCell
            } else {
                a = 0;  // (a level-13 start node of a small polyline's bound that no edge comes near)
            }
        }
        if (!defer) {
            act[k] = a;
            cnt[k] = a == 2 ? 4 : a;
        }
    }
    const unsigned long long dm = __ballot(defer);
    if (!dm) return;
    const int lane = threadIdx.x & 63, leader = __builtin_ctzll(dm);
    unsigned int b = 0;
    if (lane == leader) b = atomicAdd(xlist_n, (unsigned int)__popcll(dm));
    b = (unsigned int)__shfl((int)b, leader);
    if (defer) xlist[b + cmpct::lanes_below(dm)] = (uint32_t)k;
}

// The deferred nodes of k_expand_count: exact centre containment of a
// non-planar loop (drop / keep) or a polyline's level-13 cell test.  A fixed
// grid strides over the device-side list (no host sync).
__global__ __launch_bounds__(64) void k_expand_exact(const uint32_t *xlist, const unsigned int *xlist_n, const uint32_t *nf,
                                                     const uint32_t *ni, const uint32_t *nj, const uint32_t *nmeta,
                                                     uint8_t *act, int64_t *cnt, const int64_t *xoff, const V3 *xyz,
                                                     const uint8_t *mode, const uint8_t *origin_in, const int32_t *nvx)
{
    const int64_t nl = *xlist_n;
    for (int64_t t = tid64(); t < nl; t += (int64_t)gridDim.x * blockDim.x) {
        const uint32_t k = xlist[t];
        const uint32_t m = nmeta[k], f = nf[k];
        const int level = meta_level(m), face = meta_face(m);
        const V3 *p = xyz + xoff[f];
        const int nv = nvx[f];
        bool in;
        if (mode[f] == MODE_LOOP) {
            LoopView l{p, nv, origin_in[f] != 0};
            in = loop_contains(l, node_center(face, ni[k], nj[k], level));
        } else {
            const uint32_t size = 1u << (kMaxLevel - level);
            const double ulo = st_to_uv((double)ni[k] / (double)kMaxSize),
                         uhi = st_to_uv((double)(ni[k] + size) / (double)kMaxSize);
            const double vlo = st_to_uv((double)nj[k] / (double)kMaxSize),
                         vhi = st_to_uv((double)(nj[k] + size) / (double)kMaxSize);
            in = polyline_intersects_cell(p, nv, face, ulo, uhi, vlo, vhi);
        }
        act[k] = in ? 1 : 0;
        cnt[k] = in ? 1 : 0;
    }
}

__global__ void k_expand_write(int64_t nn, const uint32_t *nf, const uint64_t *nid, const uint32_t *ni, const uint32_t *nj,
                               const uint32_t *nmeta, const uint8_t *act, const int64_t *pos, uint32_t *of, uint64_t *oid,
                               uint32_t *oi, uint32_t *oj, uint32_t *ometa, int *any_open, unsigned int *xlist_n)
{
    int64_t k = tid64();
    if (k == 0) *xlist_n = 0u;  // the next level's list (this level's k_expand_exact has read it)
    if (k >= nn) return;
    uint8_t a = act[k];
    if (a == 0) return;
    int64_t w = pos[k];
    uint32_t m = nmeta[k];
    if (a == 1) {
        of[w] = nf[k]; oid[w] = nid[k]; oi[w] = ni[k]; oj[w] = nj[k];
        ometa[w] = m | (1u << 7);  // done
        return;
    }
    int level = meta_level(m), o = meta_orient(m), face = meta_face(m);
    uint64_t id = nid[k];
    uint64_t lsb = lsb_for_level(level);
    uint64_t child = id - lsb + (lsb >> 2);  // cellid.go ChildBegin
    uint32_t half = 1u << (kMaxLevel - level - 1);
    for (int c = 0; c < 4; c++, child += (lsb >> 1)) {
        int ij = pos_to_ij(o, c);
        of[w + c] = nf[k];
        oid[w + c] = child;
        oi[w + c] = ni[k] + ((ij >> 1) ? half : 0);
        oj[w + c] = nj[k] + ((ij & 1) ? half : 0);
        ometa[w + c] = pack_meta(level + 1, o ^ pos_to_orientation(c), 0, face);
    }
    *any_open = 1;
}

// Final items -> per-footprint counts.  A long footprint (a corridor) owns
// thousands of consecutive items, and same-address global atomics serialise
// (~88 per us): the block sums its items per footprint in LDS first (slot
// f - the block's first footprint; items out of that window go straight to
// HBM) and adds each sum with one global atomic.
constexpr int kItemBlock = 256;
__global__ __launch_bounds__(kItemBlock) void k_item_counts(int64_t nn, const uint32_t *nf, const uint32_t *nmeta,
                                                            int64_t *icnt, unsigned long long *fcnt, int *nbig)
{
    if (blockIdx.x == 0 && threadIdx.x == 0) *nbig = 0;  // (k_emit appends)
    __shared__ unsigned long long s_sum[kItemBlock];
    const int64_t k0 = (int64_t)blockIdx.x * kItemBlock, k = k0 + threadIdx.x;
    const uint32_t f0 = nf[k0];
    s_sum[threadIdx.x] = 0;
    __syncthreads();
    if (k < nn) {
        const int level = meta_level(nmeta[k]);
        const int64_t c = (int64_t)1 << (2 * (kCoverLevel - level));
        icnt[k] = c;
        const uint32_t f = nf[k], d = f - f0;
        if (d < (uint32_t)kItemBlock) atomicAdd(&s_sum[d], (unsigned long long)c);
        else atomicAdd(&fcnt[f], (unsigned long long)c);
    }
    __syncthreads();
    const unsigned long long v = s_sum[threadIdx.x];
    if (v) atomicAdd(&fcnt[f0 + threadIdx.x], v);
}

// Descent items are numbered among themselves (ipos); dpre[f] = descent cells
// of the footprints before f, offs[f] = all cells before f.
__device__ __forceinline__ int64_t item_pos(int64_t k, const uint32_t *nf, const int64_t *ipos, const int64_t *dpre,
                                            const int64_t *offs)
{
    const uint32_t f = nf[k];
    return offs[f] + (ipos[k] - dpre[f]);
}

__global__ void k_emit(int64_t nn, const uint32_t *nf, const uint64_t *nid, const uint32_t *nmeta, const int64_t *ipos,
                       const int64_t *dpre, const int64_t *offs, uint64_t *cells, uint32_t *big, int *nbig)
{
    int64_t k = tid64();
    if (k >= nn) return;
    int level = meta_level(nmeta[k]);
    int64_t c = (int64_t)1 << (2 * (kCoverLevel - level));
    uint64_t id = nid[k];
    if (c > 256) {
        big[atomicAdd(nbig, 1)] = (uint32_t)k;
        return;
    }
    uint64_t lsb13 = lsb_for_level(kCoverLevel);
    uint64_t first = id - cellid_lsb_dev(id) + lsb13;
    int64_t w = item_pos(k, nf, ipos, dpre, offs);
    for (int64_t q = 0; q < c; q++) cells[w + q] = first + (uint64_t)q * (lsb13 << 1);
}

// A fixed grid striding over the device count of big items (launched
// without reading the count back: no host sync after k_emit).
__global__ void k_emit_big(const uint32_t *big, const int *nbig, const uint32_t *nf, const uint64_t *nid,
                           const uint32_t *nmeta, const int64_t *ipos, const int64_t *dpre, const int64_t *offs,
                           uint64_t *cells)
{
    const int nb = *nbig;
    for (int b = blockIdx.x; b < nb; b += gridDim.x) {
        const uint32_t k = big[b];
        const int level = meta_level(nmeta[k]);
        const int64_t c = (int64_t)1 << (2 * (kCoverLevel - level));
        const uint64_t id = nid[k];
        const uint64_t lsb13 = lsb_for_level(kCoverLevel);
        const uint64_t first = id - cellid_lsb_dev(id) + lsb13;
        const int64_t w = item_pos(k, nf, ipos, dpre, offs);
        for (int64_t q = threadIdx.x; q < c; q += blockDim.x) cells[w + q] = first + (uint64_t)q * (lsb13 << 1);
    }
}

// ---------------------------------------------------------------------------
// Direct candidate path (FL_FAST footprints: single-face small loops whose
// padded bound lies in <= 4 start cells at level >= kFastMinLevel).  The
// candidates are the level-13 cells of the footprint's padded (i, j) bound
// (fbox; every one lies in a start cell), each tested exactly as
// k_expand_count tests a level-13 node.  A candidate's key is its index among
// the start cells' level-13 descendants in id order (start cell s, Hilbert
// position inside it), so a footprint's verdicts are two 256-bit masks
// (kept, undecided) whose bit order is the cell-id order of the output.
constexpr int kFpBlock = 256;  // threads of a k_cand_fp block (128: 0.29 -> 0.42 ms; 512: same, profiles/r07n)
constexpr int kFpPer = 64;     // footprints per k_cand_fp block (one wave loads them)

// Key of level-13 cell (i13, j13) of footprint f, or -1 outside its start
// cells (cannot happen for a cell of the bound).
__device__ __forceinline__ int rect_key(uint32_t i13, uint32_t j13, const uint32_t *sti, const uint32_t *stj,
                                        uint32_t info)
{
    const int L = (int)(info & 31u), k = (int)((info >> 5) & 7u), shL = kMaxLevel - L;
    const uint32_t i30 = i13 << (kMaxLevel - kCoverLevel), j30 = j13 << (kMaxLevel - kCoverLevel);
    int s = -1;
    for (int q = 0; q < k; q++)  // (unsigned wrap: a start cell above the cell gives a huge difference)
        if (((i30 - sti[q]) >> shL) == 0u && ((j30 - stj[q]) >> shL) == 0u) s = q;
    if (s < 0) return -1;
    int o = (int)((info >> (8 + 2 * s)) & 3u);
    uint32_t pos = 0;
    for (int l = L + 1; l <= kCoverLevel; l++) {
        const int ib = (int)((i30 >> (kMaxLevel - l)) & 1u), jb = (int)((j30 >> (kMaxLevel - l)) & 1u);
        const int p = ij_to_pos(o, (ib << 1) | jb);
        pos = (pos << 2) | (uint32_t)p;
        o ^= pos_to_orientation(p);
    }
    return (s << (2 * (kCoverLevel - L))) | (int)pos;
}

// Level-30 (i, j) corner, face and id of candidate `key` of footprint f.
__device__ __forceinline__ void key_cell(int key, uint32_t f, const uint64_t *st_id, const uint32_t *st_i,
                                         const uint32_t *st_j, uint32_t info, int &face, uint32_t &i, uint32_t &j,
                                         uint64_t &id)
{
    const int L = (int)(info & 31u);
    const int sh = 2 * (kCoverLevel - L);
    const int s = key >> sh;
    const uint32_t r = (uint32_t)key & ((1u << sh) - 1u);
    int o = (int)((info >> (8 + 2 * s)) & 3u);
    i = st_i[4 * f + s];
    j = st_j[4 * f + s];
    for (int l = L + 1; l <= kCoverLevel; l++) {
        const int digit = (int)((r >> (2 * (kCoverLevel - l))) & 3u);
        const int ij = pos_to_ij(o, digit);
        const uint32_t half = 1u << (kMaxLevel - l);
        if (ij >> 1) i += half;
        if (ij & 1) j += half;
        o ^= pos_to_orientation(digit);
    }
    const uint64_t sid = st_id[4 * f + s];
    const uint64_t lsb13 = lsb_for_level(kCoverLevel);
    face = (int)(sid >> 61);
    id = sid - lsb_for_level(L) + lsb13 + (uint64_t)r * (lsb13 << 1);  // cellid.go ChildBeginAtLevel + r steps
}

// loop.go IntersectsCell for a level-13 cell at level-30 corner (i, j): the
// padded edge test (stop at the first hit) and, for planar footprints,
// planar_contains's ray cast from the centre on the same (u,v) edge images --
// used only when no edge hits.  uc < a.x + (vc - a.y)(b.x - a.x)/(b.y - a.y),
// multiplied through by (b.y - a.y): an edge that misses the padded cell
// crosses v = vc at least half a cell (1.2e-4) from uc, so the rounding
// (~1e-16 relative) cannot flip the comparison.  0 / 1, or 2 = undecided
// (centre containment needs the exact S2 test: k_cand_exact).
__device__ __forceinline__ int cand_edges_uv(uint32_t i, uint32_t j, const double2 *up, int nv, bool planar,
                                             bool origin_in, bool rev)
{
    // (rev: a loop k_setup reversed without moving it, read mirrored)
    auto at = [&](int e) { return up[rev ? nv - 1 - e : e]; };
    double2 a = at(0);
    const uint32_t size = 1u << (kMaxLevel - kCoverLevel);
    const double ulo = st_to_uv((double)i / (double)kMaxSize), uhi = st_to_uv((double)(i + size) / (double)kMaxSize);
    const double vlo = st_to_uv((double)j / (double)kMaxSize), vhi = st_to_uv((double)(j + size) / (double)kMaxSize);
    const double pm = kFinePad;
    const double half = 0.5 / (double)kMaxSize, sz = (double)size;
    const double uc = st_to_uv(half * (2.0 * (double)i + sz)), vc = st_to_uv(half * (2.0 * (double)j + sz));
    bool in = false, par = false;
    for (int e = 0; e < nv; e++) {
        const double2 b = at(e + 1 < nv ? e + 1 : 0);
        if (edge_intersects_rect(a.x, a.y, b.x, b.y, ulo - pm, uhi + pm, vlo - pm, vhi + pm)) {
            in = true;
            break;
        }
        if ((a.y > vc) != (b.y > vc)) {
            const double d = b.y - a.y;
            const double lhs = (uc - a.x) * d, rhs = (vc - a.y) * (b.x - a.x);
            if (d > 0 ? lhs < rhs : lhs > rhs) par = !par;
        }
        a = b;
    }
    return in ? 1 : planar ? ((origin_in != par) ? 1 : 0) : 2;
}

// cand_edges_uv over LDS-staged loops of <= 64 vertices, two passes: a float
// prefilter over every edge (the vertices' (u,v) also staged as float2)
// marks the edges that can touch the cell's padded rect (both end points
// beyond one side of it, by more than 1e-6, cannot: float rounding of a
// vertex or a bound is < 1e-7 for |u|, |v| < 2) and the edges that can
// straddle the centre's row (both end points above, or below, vc by more
// than 1e-6 cannot); then only the marked edges run the exact tests, in the
// same double arithmetic -- the result is cand_edges_uv's.  NaN end points
// fail every float comparison, so their edges stay marked.
__device__ __forceinline__ int cand_edges_uv_f(uint32_t i, uint32_t j, const double2 *upg, bool rev,
                                               const float2 *upf, int nv, bool planar, bool origin_in)
{
    // (the exact tests read the loop from global memory; rev: a loop k_setup
    // reversed without moving it, read mirrored -- the float stage is in
    // loop order already)
    auto at = [&](int e) { return upg[rev ? nv - 1 - e : e]; };
    const uint32_t size = 1u << (kMaxLevel - kCoverLevel);
    const double ulo = st_to_uv((double)i / (double)kMaxSize), uhi = st_to_uv((double)(i + size) / (double)kMaxSize);
    const double vlo = st_to_uv((double)j / (double)kMaxSize), vhi = st_to_uv((double)(j + size) / (double)kMaxSize);
    const double pm = kFinePad;
    const double half = 0.5 / (double)kMaxSize, sz = (double)size;
    const double uc = st_to_uv(half * (2.0 * (double)i + sz)), vc = st_to_uv(half * (2.0 * (double)j + sz));
    constexpr float kSlack = 1e-6f;
    const float rlu = (float)(ulo - pm) - kSlack, rhu = (float)(uhi + pm) + kSlack;
    const float rlv = (float)(vlo - pm) - kSlack, rhv = (float)(vhi + pm) + kSlack;
    const float vcl = (float)vc - kSlack, vch = (float)vc + kSlack;
    unsigned long long near = 0, strad = 0;
    float2 a = upf[0];
    for (int e = 0; e < nv; e++) {
        const float2 b = upf[e + 1 < nv ? e + 1 : 0];
        const bool far = ((a.x < rlu) & (b.x < rlu)) | ((a.x > rhu) & (b.x > rhu)) | ((a.y < rlv) & (b.y < rlv)) |
                         ((a.y > rhv) & (b.y > rhv));
        const bool level = ((a.y > vch) & (b.y > vch)) | ((a.y < vcl) & (b.y < vcl));
        near |= (unsigned long long)!far << e;
        strad |= (unsigned long long)!level << e;
        a = b;
    }
    while (near) {
        const int e = __builtin_ctzll(near);
        near &= near - 1;
        const double2 x = at(e), y = at(e + 1 < nv ? e + 1 : 0);
        if (edge_intersects_rect(x.x, x.y, y.x, y.y, ulo - pm, uhi + pm, vlo - pm, vhi + pm)) return 1;
    }
    if (!planar) return 2;
    bool par = false;
    while (strad) {
        const int e = __builtin_ctzll(strad);
        strad &= strad - 1;
        const double2 x = at(e), y = at(e + 1 < nv ? e + 1 : 0);
        if ((x.y > vc) != (y.y > vc)) {
            const double d = y.y - x.y;
            const double lhs = (uc - x.x) * d, rhs = (vc - x.y) * (y.x - x.x);
            if (d > 0 ? lhs < rhs : lhs > rhs) par = !par;
        }
    }
    return (origin_in != par) ? 1 : 0;
}

// One block per kFpPer consecutive footprints: wave 0 loads their bounds,
// start cells and flags into LDS (one round trip for the block, none per
// candidate), the block stages their (u,v) vertices, then its threads stride
// over the block's bound cells (footprint by LDS search, cell by position in
// its bound) and set key bits in the footprints' LDS masks.  Wave 0 writes the
// kept masks, and lists the footprints with undecided bits for k_cand_exact.
__global__ __launch_bounds__(kFpBlock) void k_cand_fp(int64_t n, const uint8_t *flags, const uint4 *fbox,
                                                      const uint32_t *finfo, const uint32_t *st_i,
                                                      const uint32_t *st_j, const int64_t *xoff, const int32_t *nvx,
                                                      const double2 *uv, const uint8_t *origin_in,
                                                      const uint8_t *rev_flag, unsigned long long *fkm,
                                                      unsigned long long *fum, uint32_t *ulist, unsigned int *ulist_n,
                                                      const uint32_t *perm)
{
    __shared__ uint4 s_bx[kFpPer];
    __shared__ uint32_t s_info[kFpPer], s_sti[kFpPer][4], s_stj[kFpPer][4];
    __shared__ int s_cb[kFpPer + 1], s_vb[kFpPer], s_nv[kFpPer], s_fl[kFpPer], s_vp[kFpPer + 1];
    __shared__ int64_t s_xo[kFpPer];
    __shared__ unsigned long long s_km[kFpPer][4], s_um[kFpPer][4];
    __shared__ float2 s_uvf[kCandStageV];  // the block's (u,v) vertices in float (cand_edges_uv_f's prefilter)
    const int t = threadIdx.x, lane = t & 63;
    const int64_t F0 = (int64_t)blockIdx.x * kFpPer;
    if (t < kFpPer) {
        // footprints in k_setup's order (polygons, then circles): a block's
        // loops are of one kind, so a wave's edge walks are of similar length
        const int64_t f = F0 + t < n ? (int64_t)perm[F0 + t] : n;
        const bool fast = f < n && (flags[f] & FL_FAST);
        uint32_t cnt = 0, nvv = 0;
        if (fast) {
            const uint4 bx = fbox[f];
            s_bx[t] = bx;
            s_info[t] = finfo[f];
#pragma unroll
            for (int q = 0; q < 4; q++) {
                s_sti[t][q] = st_i[4 * f + q];
                s_stj[t][q] = st_j[4 * f + q];
            }
            s_xo[t] = xoff[f];
            nvv = (uint32_t)nvx[f];
            s_fl[t] = ((flags[f] & FL_PLANAR) ? 1 : 0) | (origin_in[f] ? 2 : 0) | (rev_flag[f] ? 4 : 0);
            cnt = (bx.y - bx.x + 1) * (bx.w - bx.z + 1);
        }
        s_nv[t] = (int)nvv;
#pragma unroll
        for (int q = 0; q < 4; q++) s_km[t][q] = s_um[t][q] = 0ull;
        // candidate and vertex prefixes over the block's footprints (wave scans)
        uint32_t ci = cnt, vi = nvv;
        for (int o = 1; o < 64; o <<= 1) {
            const uint32_t a = (uint32_t)__shfl_up((int)ci, o), b = (uint32_t)__shfl_up((int)vi, o);
            if (lane >= o) {
                ci += a;
                vi += b;
            }
        }
        s_cb[t + 1] = (int)ci;
        if (t == 0) s_cb[0] = 0;
        s_vb[t] = vi <= (uint32_t)kCandStageV ? (int)(vi - nvv) : -1;  // LDS offset, or -1: read from global
        s_vp[t] = (int)(vi - nvv);
        if (t == kFpPer - 1) s_vp[kFpPer] = (int)vi;
    }
    __syncthreads();
    // the block's staged vertices, all threads over them (vertex -> footprint
    // by LDS search: the last footprint whose prefix is <= k holds it), so a
    // block of small footprints (configs[3]'s 4-gons) does not walk them one
    // footprint per wave
    const int nvs = min(s_vp[kFpPer], kCandStageV);
    for (int k = t; k < nvs; k += kFpBlock) {
        int lo = 0, hi = kFpPer;  // s_vp[lo] <= k < s_vp[hi]
        while (hi - lo > 1) {
            const int mid = (lo + hi) >> 1;
            if (s_vp[mid] <= k) lo = mid;
            else hi = mid;
        }
        const int i = k - s_vp[lo];
        const double2 w = uv[s_xo[lo] + ((s_fl[lo] & 4) ? s_nv[lo] - 1 - i : i)];  // a reversed loop staged in its order
        s_uvf[k] = make_float2((float)w.x, (float)w.y);
    }
    __syncthreads();
    const int total = s_cb[kFpPer];
    for (int k = t; k < total; k += kFpBlock) {
        // (round 6: an LDS candidate -> footprint byte map and a magic-number
        // division instead of this search and d / w measured slower, 0.294
        // -> 0.315 ms, profiles/r07e)
        int lo = 0, hi = kFpPer;  // s_cb[lo] <= k < s_cb[hi]
        while (hi - lo > 1) {
            const int mid = (lo + hi) >> 1;
            if (s_cb[mid] <= k) lo = mid;
            else hi = mid;
        }
        const uint4 bx = s_bx[lo];
        const uint32_t w = bx.y - bx.x + 1, d = (uint32_t)(k - s_cb[lo]);
        const uint32_t dj = d / w, i13 = bx.x + (d - dj * w), j13 = bx.z + dj;
        const uint32_t info = s_info[lo];
        const int key = rect_key(i13, j13, s_sti[lo], s_stj[lo], info);
        if (key < 0) continue;
        const int vb = s_vb[lo], fl = s_fl[lo];
        // (staged vertices are in loop order already; unstaged ones are read
        // through the reversal)
        const double2 *up = uv + s_xo[lo];
        const int nvf = s_nv[lo];
        const int v = vb >= 0 && nvf <= 64
                          ? cand_edges_uv_f(i13 << (kMaxLevel - kCoverLevel), j13 << (kMaxLevel - kCoverLevel), up,
                                            (fl & 4) != 0, s_uvf + vb, nvf, (fl & 1) != 0, (fl & 2) != 0)
                          : cand_edges_uv(i13 << (kMaxLevel - kCoverLevel), j13 << (kMaxLevel - kCoverLevel), up, nvf,
                                          (fl & 1) != 0, (fl & 2) != 0, (fl & 4) != 0);
        if (v == 1) atomicOr(&s_km[lo][key >> 6], 1ull << (key & 63));
        else if (v == 2) atomicOr(&s_um[lo][key >> 6], 1ull << (key & 63));
    }
    __syncthreads();
    if (t < kFpPer) {
        const int64_t f = F0 + t < n ? (int64_t)perm[F0 + t] : n;
        const bool has = f < n && s_cb[t + 1] > s_cb[t];
        if (has) {
            ulonglong2 *km = reinterpret_cast<ulonglong2 *>(fkm + 4 * f);
            km[0] = make_ulonglong2(s_km[t][0], s_km[t][1]);
            km[1] = make_ulonglong2(s_km[t][2], s_km[t][3]);
        }
        const bool und = has && (s_um[t][0] | s_um[t][1] | s_um[t][2] | s_um[t][3]) != 0ull;
        const unsigned long long um = __ballot(und);
        if (um) {
            unsigned int base = 0;
            if (lane == 0) base = atomicAdd(ulist_n, (unsigned int)__popcll(um));
            base = (unsigned int)__shfl((int)base, 0);
            if (und) {
                ulist[base + cmpct::lanes_below(um)] = (uint32_t)f;
                ulonglong2 *u = reinterpret_cast<ulonglong2 *>(fum + 4 * f);
                u[0] = make_ulonglong2(s_um[t][0], s_um[t][1]);
                u[1] = make_ulonglong2(s_um[t][2], s_um[t][3]);
            }
        }
    }
}

// Undecided candidates: exact S2 containment of the cell centre.  One wave
// per listed footprint (a fixed grid strides over the list, so a batch with
// none costs one small launch), lane = key within a mask word; the wave folds
// its results into the footprint's kept mask.
__global__ __launch_bounds__(256) void k_cand_exact(const uint32_t *ulist, const unsigned int *ulist_n,
                                                    const uint64_t *st_id, const uint32_t *st_i, const uint32_t *st_j,
                                                    const uint32_t *finfo, const int64_t *xoff, const V3 *xyz,
                                                    const int32_t *nvx, const uint8_t *origin_in,
                                                    const uint8_t *rev_flag, unsigned long long *fkm,
                                                    const unsigned long long *fum)
{
    const unsigned int nl = *ulist_n;
    const int lane = threadIdx.x & 63;
    const int64_t nw = (int64_t)gridDim.x * (blockDim.x / 64);
    for (int64_t wi = (int64_t)blockIdx.x * (blockDim.x / 64) + (threadIdx.x >> 6); wi < (int64_t)nl; wi += nw) {
        const uint32_t f = ulist[wi];
        const uint32_t info = finfo[f];
        for (int q = 0; q < 4; q++) {
            const unsigned long long um = fum[4 * (int64_t)f + q];
            if (!um) continue;
            bool in = false;
            if ((um >> lane) & 1ull) {
                int face;
                uint32_t i, j;
                uint64_t id;
                key_cell(64 * q + lane, f, st_id, st_i, st_j, info, face, i, j, id);
                LoopView l{xyz + xoff[f], nvx[f], origin_in[f] != 0, rev_flag[f] != 0};
                in = loop_contains(l, node_center(face, i, j, kCoverLevel));
            }
            const unsigned long long m = __ballot(in);
            if (lane == 0 && m) fkm[4 * (int64_t)f + q] |= m;
        }
    }
}

// Per-footprint cell counts: kept direct candidates plus the descent count
// the item atomics left in dcnt.
__global__ void k_counts(int64_t n, const uint8_t *flags, const unsigned long long *fkm,
                         const unsigned long long *dcnt, int64_t *total, int64_t *dc64)
{
    const int64_t f = tid64();
    if (f >= n) return;
    int64_t c = 0;
    if (flags[f] & FL_FAST) {
        const ulonglong2 *km = reinterpret_cast<const ulonglong2 *>(fkm + 4 * f);
        const ulonglong2 a = km[0], b = km[1];
        c = __popcll(a.x) + __popcll(a.y) + __popcll(b.x) + __popcll(b.y);
    }
    total[f] = c + (int64_t)dcnt[f];
    dc64[f] = (int64_t)dcnt[f];
}

// The kept direct candidates of a footprint at its CSR offset, in id order
// (keys ascend with the cell id).  One wave per 64 footprints emits their
// cells 64 at a time: output j of the wave belongs to the last lane whose
// exclusive count prefix is <= j (a 6-step search over the lanes) and is the
// (j - prefix)-th set bit of that lane's 256-bit mask, so the trip count is
// the wave's mean count, not its largest, and neighbouring lanes store to
// neighbouring cells.
__global__ __launch_bounds__(kBlock) void k_cand_emit(int64_t n, const uint8_t *flags, const unsigned long long *fkm,
                                                      const uint64_t *st_id, const uint32_t *finfo,
                                                      const int64_t *offs, uint64_t *cells)
{
    const int lane = (int)(threadIdx.x & 63);
    const int64_t f = tid64();
    if (f - lane >= n) return;  // whole waves
    unsigned long long m0 = 0, m1 = 0, m2 = 0, m3 = 0;
    if (f < n && (flags[f] & FL_FAST)) {
        const ulonglong2 *km = reinterpret_cast<const ulonglong2 *>(fkm + 4 * f);
        const ulonglong2 a = km[0], b = km[1];
        m0 = a.x, m1 = a.y, m2 = b.x, m3 = b.y;
    }
    const int c = __popcll(m0) + __popcll(m1) + __popcll(m2) + __popcll(m3);
    int incl = c;
    for (int o = 1; o < 64; o <<= 1) {
        const int y = __shfl_up(incl, o);
        if (lane >= o) incl += y;
    }
    const int excl = incl - c, T = __shfl(incl, 63);
    if (T == 0) return;
    const int64_t w0 = c ? offs[f] : 0;
    const int L0 = c ? (int)(finfo[f] & 31u) : kCoverLevel;
    const uint64_t lsb13 = lsb_for_level(kCoverLevel);
    for (int base = 0; base < T; base += 64) {  // uniform trip count: every lane shuffles
        const int j = base + lane;
        int o = 0;
#pragma unroll
        for (int step = 32; step > 0; step >>= 1)
            if (__shfl(excl, o + step) <= j) o += step;  // o + step <= 63
        int k = j - __shfl(excl, o);
        const unsigned long long a0 = __shfl(m0, o), a1 = __shfl(m1, o), a2 = __shfl(m2, o), a3 = __shfl(m3, o);
        const int64_t w = __shfl(w0, o) + k;
        const int L = __shfl(L0, o);
        if (j >= T) continue;
        // the k-th set bit, in (word, bit) order
        int q = 0;
        unsigned long long mk = a0;
        if (k >= __popcll(mk)) { k -= __popcll(mk); mk = a1; q = 1;
            if (k >= __popcll(mk)) { k -= __popcll(mk); mk = a2; q = 2;
                if (k >= __popcll(mk)) { k -= __popcll(mk); mk = a3; q = 3; } } }
        int bit = 0;
#pragma unroll
        for (int wdt = 32; wdt > 0; wdt >>= 1) {
            const int lo = __popcll(mk & ((1ull << wdt) - 1));
            if (k >= lo) { k -= lo; mk >>= wdt; bit += wdt; }
        }
        const int cc = 64 * q + bit, sh = 2 * (kCoverLevel - L);
        const uint64_t r = (uint64_t)(cc & ((1 << sh) - 1));
        cells[w] = st_id[4 * (f - lane + o) + (cc >> sh)] - lsb_for_level(L) + lsb13 + r * (lsb13 << 1);
    }
}

__global__ void k_u64_to_i64(int64_t n, const unsigned long long *a, int64_t *b)
{
    int64_t k = tid64();
    if (k < n) b[k] = (int64_t)a[k];
}

// ===========================================================================
// Wave path: one wavefront per footprint (north_star "one wavefront per
// footprint, LDS-staged polygon vertices").  The per-thread pipeline above
// spreads a footprint over ~15 launches and re-reads its vertices from L2 per
// candidate; here one wave does the whole covering of a footprint the triage
// decides, with the loop staged in LDS:
//   lanes = vertices   S2 points (Go Cephes trig), RegularLoop vertices,
//                      (u,v) images on the face of vertex 0, the inner test;
//   lanes = triangles  k_orient's determinants, then Loop.Area's fan terms
//                      (fastp::signed_area) -- summed in surfaceIntegral order
//                      by every lane from LDS (bit-identical area);
//   lanes = edges      loop.go initOriginAndBound's crossing count
//                      (EdgeCrosser chain, each edge from its own restart);
//   lanes = candidates the level-13 descendants of the <= 4 start cells, each
//                      tested against every (u,v) edge in LDS (broadcast reads).
// Every decision is the one setup_one<true> / k_cand_test_c would make; what
// they would send to the exact path (triage fails, undecided orientation,
// polylines, multi-face / big / near-origin loops, > kWaveV vertices) is
// flagged `slow` and covered by run_general as one compacted sub-batch.
constexpr int kWaveV = 128;   // vertex cap of the wave path (LDS: 48 B per vertex)
constexpr int kWaveFp = 4;    // footprints (waves) per block
struct WaveRec {              // a wave-path footprint's kept candidates
    uint64_t st_id[4];        // start cells (sorted), level L
    unsigned long long mask[4];  // kept bits over the <= 256 candidates, in id order
    uint32_t info;            // L | k << 5
    uint32_t pad;
};


__global__ __launch_bounds__(64 * kWaveFp) void k_cover_wave(int64_t n, const int32_t *kind, const int64_t *voff,
                                                            const double *lat, const double *lng,
                                                            const float *radius_m, int32_t *status, double *area_out,
                                                            int64_t *cnt, WaveRec *rec, uint8_t *slow)
{
    __shared__ V3 s_p[kWaveFp][kWaveV];
    __shared__ double2 s_uv[kWaveFp][kWaveV];
    __shared__ double s_t[kWaveFp][kWaveV];
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    const int64_t f = (int64_t)blockIdx.x * kWaveFp + w;
    if (f >= n) return;  // wave-uniform
    V3 *p = s_p[w];
    double2 *uvp = s_uv[w];
    double *tt = s_t[w];
    const int k = kind[f];
    const int64_t v0 = voff[f];
    int st = DSSG_ST_OK, nv = 0;
    bool go_slow = false;
    double area = 0;
    auto finish = [&](int64_t c) {
        if (lane == 0) {
            status[f] = st;
            area_out[f] = area;
            cnt[f] = go_slow ? 0 : c;
            slow[f] = go_slow ? 1 : 0;
        }
    };
    // ---- inputs: range / count / radius checks (pkg/models/geo.go:224-268, Q17), S2 points
    if (k == DSSG_KIND_CIRCLE) {
        const double la = lat[v0], ln = lng[v0];
        const float r = radius_m[f];
        if (la > 90.0 || la < -90.0 || ln > 180.0 || ln < -180.0) st = DSSG_ST_BAD_COORD_SET;
        else if (!(r > 0)) st = DSSG_ST_RADIUS;
        else {
            nv = 20;
            const double radius = (double)r / DSS_RADIUS_EARTH_M;
            if (!(radius < 0.5)) {
                go_slow = true;  // not a small loop
            } else if (lane < 20) {  // k_circle_frames + k_verts, per lane
                const V3 c = point_from_degrees(la, ln);
                const V3 c1 = ortho(c), c0 = cross(c1, c);
                const double z = go_cos(radius), rr = go_sin(radius);
                const double px = rr * c_circle_cos[lane], py = rr * c_circle_sin[lane], pz = z;
                p[lane] = normalize(v3(c0.x * px + c1.x * py + c.x * pz, c0.y * px + c1.y * py + c.y * pz,
                                       c0.z * px + c1.z * py + c.z * pz));
            }
        }
    } else {
        nv = (int)(voff[f + 1] - v0);
        if (k == DSSG_KIND_POLYGON) {
            bool bad = false;
            for (int i = lane; i < nv; i += 64) {
                const double la = lat[v0 + i], ln = lng[v0 + i];
                bad |= la > 90.0 || la < -90.0 || ln > 180.0 || ln < -180.0;
            }
            if (__ballot(bad)) st = DSSG_ST_BAD_COORD_SET;
        }
        if (st == DSSG_ST_OK && nv < 3) st = DSSG_ST_NOT_ENOUGH_POINTS;
        if (st == DSSG_ST_OK) {
            if (nv > kWaveV) go_slow = true;
            else
                for (int i = lane; i < nv; i += 64) p[i] = point_from_degrees(lat[v0 + i], lng[v0 + i]);
        }
    }
    if (st != DSSG_ST_OK || go_slow) {
        finish(0);
        return;
    }
    __builtin_amdgcn_wave_barrier();
    // ---- (u,v) on the face of vertex 0; every edge inside that face (k_fan)
    const int face0 = xyz_face(p[0]);
    bool outer = false;
    for (int i = lane; i < nv; i += 64) {
        double u, v;
        valid_face_xyz_to_uv(face0, p[i], u, v);
        uvp[i] = make_double2(u, v);
        outer |= !edge_inside_face(p[i], p[i + 1 == nv ? 0 : i + 1], face0);
    }
    if (__ballot(outer)) {
        go_slow = true;
        finish(0);
        return;
    }
    bool fail = false;
    if (k != DSSG_KIND_CIRCLE) {
        // ---- k_orient: fan determinants per lane, summed in order by every lane
        const V3 a = p[0];
        bool far = false;
        for (int i = 1 + lane; i < nv; i += 64) {
            const V3 c = p[i];
            far |= !(a.x * c.x + a.y * c.y + a.z * c.z >= 0.99875);  // cos(0.05)
            if (i + 1 < nv) {
                const V3 b = c, cc = p[i + 1];
                tt[i] = a.x * (b.y * cc.z - b.z * cc.y) + a.y * (b.z * cc.x - b.x * cc.z) + a.z * (b.x * cc.y - b.y * cc.x);
            }
        }
        const bool near = __ballot(far) == 0ull;
        __builtin_amdgcn_wave_barrier();
        double d = 0, dabs = 0;
        for (int i = 1; i + 1 < nv; i++) {
            const double t = tt[i];
            d += t;
            dabs += __builtin_fabs(t);
        }
        d *= 0.5;
        dabs *= 0.5;
        const double margin = 0.05 * dabs + 1e-13;
        int om = 2;
        if (near && d > margin && ((d * 1.1) * DSS_EARTH_AREA_KM2) / 4.0 * DSS_PI < DSS_MAX_AREA_KM2) om = 0;
        else if (near && d < -margin) om = 1;
        if (om == 2) {  // both orientations' terms would be needed: the general path
            go_slow = true;
            finish(0);
            return;
        }
        __builtin_amdgcn_wave_barrier();
        // ---- k_fan_area: the needed orientation's terms, one lane per triangle
        bool fl = false;
        for (int j = lane; j < nv - 2; j += 64) {
            const int i = 1 + j;
            const V3 ta = om == 1 ? p[nv - 1] : p[0], tb = om == 1 ? p[nv - 1 - i] : p[i],
                     tc = om == 1 ? p[nv - 2 - i] : p[i + 1];
            bool f1 = angle(tc, ta) > DSS_SURFACE_MAX_LENGTH;
            const double v = fastp::signed_area(ta, tb, tc, f1);
            tt[i] = v;
            fl |= f1;
        }
        fail = __ballot(fl) != 0ull;
        __builtin_amdgcn_wave_barrier();
        if (om == 0) {
            area = fan_area_km2(tt, nv, fail);
            if (area > DSS_MAX_AREA_KM2) fail = true;  // mispredicted: no reversed terms
        } else {
            area = INFINITY;  // the forward sum is negative: ~4 pi, above the cap
        }
        if (fail) {
            go_slow = true;
            finish(0);
            return;
        }
        if (area > DSS_MAX_AREA_KM2) {  // Q4: reverse in place (points and their (u,v) images)
            for (int i = lane; i < nv / 2; i += 64) {
                const int j = nv - 1 - i;
                const V3 x = p[i];
                p[i] = p[j];
                p[j] = x;
                const double2 y = uvp[i];
                uvp[i] = uvp[j];
                uvp[j] = y;
            }
            __builtin_amdgcn_wave_barrier();
            area = fan_area_km2(tt, nv, fail, true);
            if (fail) {
                go_slow = true;
                finish(0);
                return;
            }
        }
        if (area > DSS_MAX_AREA_KM2) {
            st = DSSG_ST_AREA_TOO_LARGE;
            finish(0);
            return;
        }
        if (area <= 0) {  // Q3: open polyline (general path)
            go_slow = true;
            finish(0);
            return;
        }
    }
    // ---- loop.go initOriginAndBound on the final loop: v1's wedge vs the
    // crossings of OriginPoint -> v1 with every edge (one lane per edge)
    const V3 P0 = p[0], P1 = p[1], P2 = p[2];
    const bool v1_inside = !eq(P0, P1) && !eq(P2, P1) && fastp::angle_contains_vertex(P0, P1, P2, fail);
    EdgeCrosser ex;
    ex.init(origin_point(), P1);
    bool par = false, fl = false;
    for (int i = 1 + lane; i <= nv; i += 64) {
        EdgeCrosser y = ex;
        y.c = p[i - 1];
        y.acb = -triage_sign(y.a, y.b, y.c);  // restart_at(v[i-1])
        par ^= fastp::edge_or_vertex_chain_crossing(y, p[i == nv ? 0 : i], fl);
    }
    fail |= __ballot(fl) != 0ull;
    const bool contains_v1 = (__popcll(__ballot(par)) & 1) != 0;
    const bool origin_in = v1_inside != contains_v1;
    if (fail) {
        go_slow = true;
        finish(0);
        return;
    }
    // ---- (u,v) bound, planar test, start cells (setup_one's FL_FAST block)
    double ulo = 1e300, uhi = -1e300, vlo = 1e300, vhi = -1e300;
    for (int i = lane; i < nv; i += 64) {
        const double2 q = uvp[i];
        ulo = fmin(ulo, q.x);
        uhi = fmax(uhi, q.x);
        vlo = fmin(vlo, q.y);
        vhi = fmax(vhi, q.y);
    }
    ulo = wave_min_d(ulo);
    uhi = wave_max_d(uhi);
    vlo = wave_min_d(vlo);
    vhi = wave_max_d(vhi);
    bool near_origin = false;
    if (face0 == xyz_face(origin_point())) {
        double ou, ov;
        valid_face_xyz_to_uv(face0, origin_point(), ou, ov);
        near_origin = ou >= ulo - 1e-6 && ou <= uhi + 1e-6 && ov >= vlo - 1e-6 && ov <= vhi + 1e-6;
    }
    const double m = 1e-7;
    const FaceBox b{ulo - m, uhi + m, vlo - m, vhi + m};
    uint64_t sid[4];
    uint32_t si[4], sj[4], smt[4];
    const int kc = start_cells(b, face0, sid, si, sj, smt);
    const int L = kc > 0 ? meta_level(smt[0]) : 0;
    if (near_origin || kc == 0 || L < kFastMinLevel) {
        go_slow = true;
        finish(0);
        return;
    }
    const int sh13 = kMaxLevel - kCoverLevel;
    const uint32_t bx0 = (uint32_t)(st_to_ij(uv_to_st(fmax(b.ulo, -1.0))) >> sh13),
                   bx1 = (uint32_t)(st_to_ij(uv_to_st(fmin(b.uhi, 1.0))) >> sh13),
                   by0 = (uint32_t)(st_to_ij(uv_to_st(fmax(b.vlo, -1.0))) >> sh13),
                   by1 = (uint32_t)(st_to_ij(uv_to_st(fmin(b.vhi, 1.0))) >> sh13);
    // ---- candidates, one per lane: bound, then the padded edge test and the
    // planar centre ray cast over the LDS edges (cand_edges)
    const int sh = 2 * (kCoverLevel - L);
    const int nc = kc << sh;
    unsigned long long km[4] = {0, 0, 0, 0};
    const uint32_t size = 1u << (kMaxLevel - kCoverLevel);
    const double pm = kFinePad;
    const double half = 0.5 / (double)kMaxSize, sz = (double)size;
    for (int c0 = 0; c0 < nc; c0 += 64) {
        const int c = c0 + lane;
        bool keep = false;
        if (c < nc) {
            const int s = c >> sh;
            const uint32_t r = (uint32_t)(c & ((1 << sh) - 1));
            int o = meta_orient(smt[s]);
            uint32_t i = si[s], j = sj[s];
            for (int l = L + 1; l <= kCoverLevel; l++) {
                const int digit = (int)((r >> (2 * (kCoverLevel - l))) & 3u);
                const int ij = pos_to_ij(o, digit);
                const uint32_t hf = 1u << (kMaxLevel - l);
                if (ij >> 1) i += hf;
                if (ij & 1) j += hf;
                o ^= pos_to_orientation(digit);
            }
            const uint32_t i13 = i >> sh13, j13 = j >> sh13;
            if (!(i13 < bx0 || i13 > bx1 || j13 < by0 || j13 > by1)) {
                const double culo = st_to_uv((double)i / (double)kMaxSize),
                             cuhi = st_to_uv((double)(i + size) / (double)kMaxSize);
                const double cvlo = st_to_uv((double)j / (double)kMaxSize),
                             cvhi = st_to_uv((double)(j + size) / (double)kMaxSize);
                const double uc = st_to_uv(half * (2.0 * (double)i + sz)), vc = st_to_uv(half * (2.0 * (double)j + sz));
                bool in = false, pr = false;
                double2 a = uvp[0];
                for (int e = 0; e < nv; e++) {
                    const double2 q = uvp[e + 1 < nv ? e + 1 : 0];
                    if (edge_intersects_rect(a.x, a.y, q.x, q.y, culo - pm, cuhi + pm, cvlo - pm, cvhi + pm)) {
                        in = true;
                        break;
                    }
                    if ((a.y > vc) != (q.y > vc)) {
                        const double dd = q.y - a.y;
                        const double lhs = (uc - a.x) * dd, rhs = (vc - a.y) * (q.x - a.x);
                        if (dd > 0 ? lhs < rhs : lhs > rhs) pr = !pr;
                    }
                    a = q;
                }
                keep = in || (origin_in != pr);
            }
        }
        const unsigned long long bm = __ballot(keep);
        km[0] = (c0 >> 6) == 0 ? bm : km[0];
        km[1] = (c0 >> 6) == 1 ? bm : km[1];
        km[2] = (c0 >> 6) == 2 ? bm : km[2];
        km[3] = (c0 >> 6) == 3 ? bm : km[3];
    }
    const int64_t total = __popcll(km[0]) + __popcll(km[1]) + __popcll(km[2]) + __popcll(km[3]);
    if (lane < 4) {
        WaveRec &R = rec[f];
        R.st_id[lane] = lane < kc ? sid[lane] : 0;
        R.mask[lane] = lane == 0 ? km[0] : lane == 1 ? km[1] : lane == 2 ? km[2] : km[3];
        if (lane == 0) {
            R.info = (uint32_t)L | ((uint32_t)kc << 5);
            R.pad = 0;
        }
    }
    finish(total);
}

// Wave-path footprints' cells at their CSR offsets (one thread per footprint,
// kept candidates in id order).
__global__ void k_emit_wave(int64_t n, const uint8_t *slow, const WaveRec *rec, const int64_t *offs, uint64_t *cells)
{
    const int64_t f = tid64();
    if (f >= n || slow[f]) return;
    int64_t w = offs[f];
    if (offs[f + 1] == w) return;
    const WaveRec R = rec[f];
    const int L = (int)(R.info & 31u);
    const int sh = 2 * (kCoverLevel - L);
    const uint64_t lsbL = lsb_for_level(L), lsb13 = lsb_for_level(kCoverLevel);
    for (int q = 0; q < 4; q++) {
        unsigned long long mk = R.mask[q];
        while (mk) {
            const int c = 64 * q + __builtin_ctzll(mk);
            mk &= mk - 1;
            const int s = c >> sh;
            const uint64_t r = (uint64_t)(c & ((1 << sh) - 1));
            cells[w++] = R.st_id[s] - lsbL + lsb13 + r * (lsb13 << 1);  // cellid.go ChildBeginAtLevel + r steps
        }
    }
}

// The slow footprints as their own batch (kind, radius, vertex counts) ...
__global__ void k_slow_gather(int64_t ns, const uint32_t *list, const int32_t *kind, const int64_t *voff,
                              const float *radius_m, int32_t *skind, float *srad, int64_t *snv)
{
    const int64_t k = tid64();
    if (k >= ns) return;
    const uint32_t f = list[k];
    skind[k] = kind[f];
    srad[k] = radius_m[f];
    snv[k] = voff[f + 1] - voff[f];
}
// ... and their vertices (one wave per slow footprint).
__global__ void k_slow_verts(int64_t ns, const uint32_t *list, const int64_t *voff, const double *lat, const double *lng,
                             const int64_t *svoff, double *slat, double *slng)
{
    const int64_t k = (int64_t)blockIdx.x * (blockDim.x / 64) + (threadIdx.x >> 6);
    if (k >= ns) return;
    const uint32_t f = list[k];
    const int64_t a = voff[f], nv = voff[f + 1] - a, b = svoff[k];
    for (int64_t i = threadIdx.x & 63; i < nv; i += 64) {
        slat[b + i] = lat[a + i];
        slng[b + i] = lng[a + i];
    }
}
// The general pipeline's answers back to their footprints.
__global__ void k_slow_scatter(int64_t ns, const uint32_t *list, const int32_t *sstat, const double *sarea,
                               const int64_t *soffs, int32_t *status, double *area, int64_t *cnt)
{
    const int64_t k = tid64();
    if (k >= ns) return;
    const uint32_t f = list[k];
    status[f] = sstat[k];
    area[f] = sarea[k];
    cnt[f] = soffs[k + 1] - soffs[k];
}
// The slow footprints' cells into the merged CSR (one wave per footprint).
__global__ void k_slow_cells(int64_t ns, const uint32_t *list, const int64_t *soffs, const uint64_t *scells,
                             const int64_t *offs, uint64_t *cells)
{
    const int64_t k = (int64_t)blockIdx.x * (blockDim.x / 64) + (threadIdx.x >> 6);
    if (k >= ns) return;
    const int64_t a = soffs[k], c = soffs[k + 1] - a, b = offs[list[k]];
    for (int64_t i = threadIdx.x & 63; i < c; i += 64) cells[b + i] = scells[a + i];
}

struct PredSlow {
    const uint8_t *slow;
    __device__ bool operator()(int64_t i) const { return slow[i] != 0; }
};
struct EmitSlow {
    uint32_t *list;
    __device__ void operator()(int64_t i, int64_t r) const { list[r] = (uint32_t)i; }
};

}  // namespace

// ---------------------------------------------------------------- host side
void CoverEngine::run(int64_t n, const int32_t *kind, const int64_t *voff, const double *lat, const double *lng,
                      const float *radius_m, hipStream_t s, dssg_cells *out)
{
    // the wave path is one launch with few host syncs, but a wave per
    // footprint runs the per-footprint (uniform) work on all 64 lanes: at 1M
    // footprints it took 6.5 ms against the general pipeline's 2.1 ms, so it
    // serves the small, launch-bound batches of the per-request path only
    if (!wave_ || n == 0 || n > wave_max_) {
        last_slow_ = n;
        run_general(n, kind, voff, lat, lng, radius_m, s, out);
        return;
    }
    init_tables(s);
    int32_t *status = w_status_.ensure(n + 1);
    double *area = w_area_.ensure(n + 1);
    int64_t *cnt = w_cnt_.ensure(n + 1), *offs = w_offs_.ensure(n + 1), *dtot = w_tot_.ensure(2);
    WaveRec *rec = (WaveRec *)w_rec_.ensure(sizeof(WaveRec) * (size_t)(n + 1));
    uint8_t *slow = w_slow_.ensure(n + 1);
    hipLaunchKernelGGL(k_cover_wave, dim3(grid_for(n, kWaveFp)), dim3(64 * kWaveFp), 0, s, n, kind, voff, lat, lng,
                       radius_m, status, area, cnt, rec, slow);
    // counts and slow flags to the host (the batch is small): offsets and
    // total there, one sync; only a batch with slow footprints takes the
    // device compaction and the general pipeline below
    h_cnt_.resize((size_t)n);
    h_slow_.resize((size_t)n);
    DSS_HIP(hipMemcpyAsync(h_cnt_.data(), cnt, sizeof(int64_t) * (size_t)n, hipMemcpyDeviceToHost, s));
    DSS_HIP(hipMemcpyAsync(h_slow_.data(), slow, (size_t)n, hipMemcpyDeviceToHost, s));
    DSS_HIP(hipStreamSynchronize(s));
    bool any_slow = false;
    for (int64_t i = 0; i < n && !any_slow; i++) any_slow = h_slow_[i] != 0;
    if (!any_slow) {
        last_slow_ = 0;
        // pinned staging of the offsets; its previous upload (maybe on
        // another stream) has finished once h_ev_ has
        if (h_ev_) DSS_HIP(hipEventSynchronize(h_ev_));
        else DSS_HIP(hipEventCreateWithFlags(&h_ev_, hipEventDisableTiming));
        if (h_offs_cap_ < n + 1) {
            if (h_offs_) DSS_HIP(hipHostFree(h_offs_));
            h_offs_cap_ = std::max<int64_t>(2 * (n + 1), 4096);
            DSS_HIP(hipHostMalloc((void **)&h_offs_, sizeof(int64_t) * (size_t)h_offs_cap_, hipHostMallocDefault));
        }
        h_offs_[0] = 0;
        for (int64_t i = 0; i < n; i++) h_offs_[i + 1] = h_offs_[i] + h_cnt_[i];
        const int64_t total = h_offs_[n];
        DSS_HIP(hipMemcpyAsync(offs, h_offs_, sizeof(int64_t) * (size_t)(n + 1), hipMemcpyHostToDevice, s));
        DSS_HIP(hipEventRecord(h_ev_, s));
        uint64_t *cells = w_cells_.ensure(total + 1);
        hipLaunchKernelGGL(k_emit_wave, dim3(grid_for(n, kBlock)), dim3(kBlock), 0, s, n, slow, rec, offs, cells);
        out->n = n;
        out->offs = offs;
        out->cells = cells;
        out->status = status;
        out->area_km2 = area;
        out->total_cells = total;
        return;
    }
    // the footprints the wave path left: one sub-batch through the general pipeline
    uint32_t *list = s_list_.ensure(n + 1);
    int64_t ns = 0;
    compact_if(n, PredSlow{slow}, EmitSlow{list}, tmp_, tmp2_, s, dtot, &ns);
    last_slow_ = ns;
    dssg_cells sub{};
    if (ns > 0) {
        int32_t *skind = s_kind_.ensure(ns + 1);
        float *srad = s_rad_.ensure(ns + 1);
        int64_t *snv = s_nv_.ensure(ns + 1), *svoff = s_voff_.ensure(ns + 1);
        hipLaunchKernelGGL(k_slow_gather, dim3(grid_for(ns, kBlock)), dim3(kBlock), 0, s, ns, list, kind, voff, radius_m,
                           skind, srad, snv);
        exclusive_scan_i64(snv, svoff, ns, tmp_, s);
        int64_t snx = 0;
        DSS_HIP(hipMemcpyAsync(&snx, svoff + ns, sizeof(int64_t), hipMemcpyDeviceToHost, s));
        DSS_HIP(hipStreamSynchronize(s));
        double *slat = s_lat_.ensure(snx + 1), *slng = s_lng_.ensure(snx + 1);
        hipLaunchKernelGGL(k_slow_verts, dim3(grid_for(ns, kBlock / 64)), dim3(kBlock), 0, s, ns, list, voff, lat, lng,
                           svoff, slat, slng);
        run_general(ns, skind, svoff, slat, slng, srad, s, &sub);
        hipLaunchKernelGGL(k_slow_scatter, dim3(grid_for(ns, kBlock)), dim3(kBlock), 0, s, ns, list, sub.status,
                           sub.area_km2, sub.offs, status, area, cnt);
    }
    exclusive_scan_i64(cnt, offs, n, tmp_, s);
    int64_t total = 0;
    DSS_HIP(hipMemcpyAsync(&total, offs + n, sizeof(int64_t), hipMemcpyDeviceToHost, s));
    DSS_HIP(hipStreamSynchronize(s));
    uint64_t *cells = w_cells_.ensure(total + 1);
    hipLaunchKernelGGL(k_emit_wave, dim3(grid_for(n, kBlock)), dim3(kBlock), 0, s, n, slow, rec, offs, cells);
    if (ns > 0)
        hipLaunchKernelGGL(k_slow_cells, dim3(grid_for(ns, kBlock / 64)), dim3(kBlock), 0, s, ns, list, sub.offs,
                           sub.cells, offs, cells);
    out->n = n;
    out->offs = offs;
    out->cells = cells;
    out->status = status;
    out->area_km2 = area;
    out->total_cells = total;
}

int64_t *CoverEngine::mailbox()
{
    if (!mail_h_) {
        DSS_HIP(hipHostMalloc((void **)&mail_h_, 16 * sizeof(int64_t), hipHostMallocMapped | hipHostMallocCoherent));
        DSS_HIP(hipHostGetDevicePointer((void **)&mail_d_, mail_h_, 0));
    }
    return mail_d_;
}

void CoverEngine::init_tables(hipStream_t s)
{
    if (tables_) return;
    // RegularLoop angles, bit-identical host evaluation of the Go math
    double cs[20], sn[20];
    const double step = 2 * DSS_PI / 20.0;
    for (int i = 0; i < 20; i++) {
        const double ang = (double)i * step;
        cs[i] = go_cos(ang);
        sn[i] = go_sin(ang);
    }
    DSS_HIP(hipMemcpyToSymbolAsync(HIP_SYMBOL(c_circle_cos), cs, sizeof(cs), 0, hipMemcpyHostToDevice, s));
    DSS_HIP(hipMemcpyToSymbolAsync(HIP_SYMBOL(c_circle_sin), sn, sizeof(sn), 0, hipMemcpyHostToDevice, s));
    tables_ = true;
}

void CoverEngine::run_general(int64_t n, const int32_t *kind, const int64_t *voff, const double *lat,
                              const double *lng, const float *radius_m, hipStream_t s, dssg_cells *out)
{
    const unsigned B = kBlock;
    out->n = n;
    init_tables(s);
    int64_t *nv = cnt_.ensure(n + 1);
    int64_t *xoff = xoff_.ensure(n + 1);
    int32_t *status = status_.ensure(n + 1);
    double *area = area_.ensure(n + 1);
    uint8_t *mode = mode_.ensure(n + 1), *orig = orig_.ensure(n + 1), *fmask = fmask_.ensure(n + 1),
            *flags = flags_.ensure(n + 1);
    int32_t *nvx = nvx_.ensure(n + 1);
    int64_t *offs = offs_.ensure(n + 1);
    if (n == 0) {
        DSS_HIP(hipMemsetAsync(offs, 0, sizeof(int64_t), s));
        out->offs = offs; out->cells = cells_.ensure(1); out->status = status; out->area_km2 = area; out->total_cells = 0;
        return;
    }
    uint8_t *fan_fail = fanf_.ensure(n + 1), *not_inner = ninner_.ensure(n + 1), *bad = badv_.ensure(n + 1);
    unsigned int *slow_n = slow_n_.ensure(1), *dlist_n = dlist_n_.ensure(1), *ulist_n = ulist_n_.ensure(1);
    hipLaunchKernelGGL(k_nverts, dim3(grid_for(n, B)), dim3(B), 0, s, n, kind, voff, nv, fan_fail, not_inner, bad,
                       slow_n, dlist_n, ulist_n);
    int64_t *mail = mailbox();  // [0] vertices [1] edge items [2] descent [3] exact setups [4] start nodes
                                // [5] next frontier [6] open [7] cells
    volatile const int64_t *mh = mail_h_;
    uint32_t *perm = perm_.ensure(n + 1);
    partition_polygons_first(kind, perm, fcnt_.ensure(n + 2), n, tmp_, tmp2_, s);
    int64_t *xoffp = xoff;
    if (slot_order_) {
        int64_t *nvp = nvp_.ensure(n + 1);
        xoffp = xoffp_.ensure(n + 1);
        hipLaunchKernelGGL(k_perm_counts, dim3(grid_for(n, B)), dim3(B), 0, s, n, perm, nv, nvp);
        exclusive_scan_i64(nvp, xoffp, n, tmp_, s, mail + 0);
        hipLaunchKernelGGL(k_perm_offsets, dim3(grid_for(n, B)), dim3(B), 0, s, n, perm, xoffp, xoff);
    } else {
        exclusive_scan_i64(nv, xoff, n, tmp_, s, mail + 0);
    }
    DSS_HIP(hipStreamSynchronize(s));
    const int64_t nx = mh[0];
    V3 *xyz = (V3 *)xyz_.ensure((size_t)nx * 3 + 3);
    double2 *uv = uv_.ensure(nx + 1);
    uint64_t *st_id = st_id_.ensure(4 * n + 4);
    uint32_t *st_i = st_i_.ensure(4 * n + 4), *st_j = st_j_.ensure(4 * n + 4), *finfo = finfo_.ensure(n + 1);
    uint4 *fbox = fbox_.ensure(n + 1);
    uint32_t *slow = slow_.ensure(n + 1);
    CircleFrame *frames = (CircleFrame *)frames_.ensure(sizeof(CircleFrame) * (n + 1));
    uint32_t *vown = vown_.ensure(nx + 1);
    double *fwd = fwd_.ensure(nx + 1), *rev = rev_.ensure(nx + 1);
    uint8_t *omode = omode_.ensure(n + 1);
    int64_t *tcnt = tcnt_.ensure(n + 1), *toff = toff_.ensure(n + 2);
    uint32_t *towner = towner_.ensure(2 * nx + 1);  // <= 2 (n - 2) tasks per loop
    // per-vertex pre-pass: frames, owners, S2 points, fan terms
    hipLaunchKernelGGL(k_circle_frames, dim3(grid_for(n, B)), dim3(B), 0, s, n, kind, voff, lat, lng, radius_m, frames);
    hipLaunchKernelGGL(k_vowner, dim3(grid_for(n, B)), dim3(B), 0, s, n, xoffp, vown, slot_order_ ? perm : nullptr);
    if (nx > 0) {
        hipLaunchKernelGGL(k_verts, dim3(grid_for(nx, B)), dim3(B), 0, s, nx, vown, kind, voff, lat, lng, xoff, frames, xyz,
                           bad);
        // (k_fan fused into k_verts -- neighbours by shuffle, recomputed across
        // wave edges -- measured slower: 0.355 against 0.317 ms, r05v)
        hipLaunchKernelGGL(k_fan, dim3(grid_for(nx, B)), dim3(B), 0, s, nx, vown, nv, xoff, xyz, uv, not_inner);
    }
    // fan triangle terms of Loop.Area: orientation first, then one thread per
    // triangle actually needed (no lanes idle on circles or on the orientation
    // that is never summed)
    hipLaunchKernelGGL(k_orient, dim3(grid_for(n, B)), dim3(B), 0, s, n, kind, nv, xoff, xyz, omode, tcnt);
    exclusive_scan_i64(tcnt, toff, n, tmp_, s);
    hipLaunchKernelGGL(k_vowner, dim3(grid_for(n, B)), dim3(B), 0, s, n, toff, towner, nullptr);
    hipLaunchKernelGGL(k_fan_area, dim3(std::min<int64_t>(grid_for(2 * nx + 1, B), 2048)), dim3(B), 0, s, toff + n,
                       towner, toff, omode, nv, xoff, xyz, fwd, rev, fan_fail);
    uint8_t *rev_flag = revf_.ensure(n + 1);
    hipLaunchKernelGGL(k_setup, dim3(grid_for(n, kSetupBlock)), dim3(kSetupBlock), 0, s, slow, slow_n, n, kind, voff, lat, lng, radius_m,
                       xoff, xyz, status, area, mode, orig, fmask, flags, nvx, uv, st_id, st_i, st_j, finfo, fbox, fwd,
                       rev, fan_fail, not_inner, omode, perm, rev_flag, bad, frames, all_exact_ ? 1 : 0);
    int64_t *eoff = eoff_.ensure(n + 1);
    uint32_t *dlist = dlist_.ensure(n + 1);
    int64_t ne = 0;
    unsigned int nd_u = 0, ns_u = 0;
    // the exact setup of whatever the triage left (~1 footprint per 1M on
    // configs[2]), launched without reading the count back: a fixed grid of
    // waves strides over the device list (empty, it costs one small launch),
    // then per footprint its clipped-edge items and the descent list, and one
    // sync for their totals
    hipLaunchKernelGGL(k_setup_exact, dim3(kExactGrid), dim3(kExactBlock), 0, s, slow, slow_n, kind, voff, lat, lng, radius_m, xoff,
                       xyz, status, area, mode, orig, fmask, flags, nvx, uv, st_id, st_i, st_j, finfo, fbox, rev_flag,
                       bad);
    hipLaunchKernelGGL(k_edge_counts, dim3(grid_for(n, B)), dim3(B), 0, s, n, mode, fmask, flags, nvx, nv, dlist, dlist_n);
    exclusive_scan_i64(nv, eoff, n, tmp_, s, mail + 1);
    mail_counters(dlist_n, slow_n, nullptr, mail + 2, s);
    DSS_HIP(hipStreamSynchronize(s));
    ne = mh[1];
    nd_u = (unsigned int)mh[2];
    ns_u = (unsigned int)mh[3];
    const int64_t nd = nd_u;  // descent footprints (big, multi-face, polyline): the only ones k_start visits
    if (nd > 0)
        hipLaunchKernelGGL(k_reverse_list, dim3((unsigned)std::min<int64_t>((nd + 3) / 4, 1024)), dim3(256), 0, s, dlist,
                           dlist_n, xoff, nvx, rev_flag, xyz, uv);
    if (std::getenv("DSS_COVER_STATS")) {
        fprintf(stderr, "[cover] n %lld vertices %lld clipped edges %lld descent %lld exact-setup %u\n", (long long)n,
                (long long)nx, (long long)ne, (long long)nd, ns_u);
        // (the exact setup's footprints: kind, vertex count, status, mode, flags)
        for (unsigned int i = 0; i < ns_u && i < 8; i++) {
            uint32_t f = 0;
            int32_t k = 0, st = 0, nvv = 0;
            uint8_t md = 0, fl = 0;
            DSS_HIP(hipMemcpy(&f, slow + i, sizeof(f), hipMemcpyDeviceToHost));
            DSS_HIP(hipMemcpy(&k, kind + f, sizeof(k), hipMemcpyDeviceToHost));
            DSS_HIP(hipMemcpy(&st, status + f, sizeof(st), hipMemcpyDeviceToHost));
            DSS_HIP(hipMemcpy(&nvv, nvx + f, sizeof(nvv), hipMemcpyDeviceToHost));
            DSS_HIP(hipMemcpy(&md, mode + f, 1, hipMemcpyDeviceToHost));
            DSS_HIP(hipMemcpy(&fl, flags + f, 1, hipMemcpyDeviceToHost));
            fprintf(stderr, "[cover]   exact-setup footprint %u: kind %d vertices %d status %d mode %d flags %d\n", f, k,
                    nvv, st, (int)md, (int)fl);
        }
    }
    // direct candidates (most footprints): the cells of each one's bound,
    // tested now, compacted after the counts
    unsigned long long *fkm = kmask_.ensure(8 * (n + 1)), *fum = fkm + 4 * (n + 1);
    uint32_t *ulist = ulist_.ensure(n + 1);
    hipLaunchKernelGGL(k_cand_fp, dim3(grid_for(n, kFpPer)), dim3(kFpBlock), 0, s, n, flags, fbox, finfo, st_i, st_j,
                       xoff, nvx, uv, orig, rev_flag, fkm, fum, ulist, ulist_n, perm);
    hipLaunchKernelGGL(k_cand_exact, dim3((unsigned)std::min<int64_t>(grid_for(n, B / 64), 1024)), dim3(B), 0, s, ulist,
                       ulist_n, st_id, st_i, st_j, finfo, xoff, xyz, nvx, orig, rev_flag, fkm, fum);
    // hierarchical descent for the rest (big, multi-face, polyline footprints)
    double4 *clip_f = clipf_.ensure(ne + 1), *clip_c = clipc_.ensure(ne + 1);
    uint8_t *cflags = cflags_.ensure(ne + 1);
    if (ne > 0) {
        uint32_t *eown = eown_.ensure(ne + 1);
        hipLaunchKernelGGL(k_vowner, dim3(grid_for(n, B)), dim3(B), 0, s, n, eoff, eown, nullptr);
        hipLaunchKernelGGL(k_clip_items, dim3(grid_for(ne, B)), dim3(B), 0, s, ne, eown, xoff, xyz, mode, fmask, nvx, eoff,
                           clip_f, clip_c, cflags);
    }
    int64_t *soff = soff_.ensure(n + 1);
    int64_t nn = 0;
    // the descent's list counters, zeroed by the kernel before the one that
    // appends to them (k_start<0>: start descriptors and the first level's
    // exact list; k_expand_count / _write: the open flag, the next list;
    // k_item_counts: the big items) -- no fill launches
    unsigned int *sdesc_n = sdesc_n_.ensure(1), *xlist_n = xlist_n_.ensure(1);
    int *any_open = flag_.ensure(1);
    if (nd > 0) {  // (none: no start nodes, no second sync)
        DSS_HIP(hipMemsetAsync(nv, 0, sizeof(int64_t) * n, s));
        hipLaunchKernelGGL(k_start<0>, dim3(grid_for(nd, 64)), dim3(64), 0, s, nd, dlist, xoff, xyz, mode, fmask, flags,
                           orig, nvx, eoff, clip_c, cflags, nv, soff, nullptr, nullptr, nullptr, nullptr, nullptr, nullptr,
                           sdesc_n, xlist_n);
        exclusive_scan_i64(nv, soff, n, tmp_, s, mail + 4);
        DSS_HIP(hipStreamSynchronize(s));
        nn = mh[4];
    }
    int cur = 0;
    Frontier *F = &fr_[cur];
    F->ensure(nn + 1);
    if (nn > 0) {
        StartDesc *sdesc = (StartDesc *)sdesc_.ensure(sizeof(StartDesc) * (size_t)(24 * nd + 1));
        hipLaunchKernelGGL(k_start<1>, dim3(grid_for(nd, 64)), dim3(64), 0, s, nd, dlist, xoff, xyz, mode, fmask, flags,
                           orig, nvx, eoff, clip_c, cflags, nullptr, soff, F->f.p, F->id.p, F->i.p, F->j.p, F->meta.p,
                           sdesc, sdesc_n, nullptr);
        hipLaunchKernelGGL(k_start13, dim3((unsigned)std::min<int64_t>((24 * nd + 3) / 4, 1024)), dim3(256), 0, s, sdesc,
                           sdesc_n, F->f.p, F->id.p, F->i.p, F->j.p, F->meta.p);
    }
    for (int iter = 0; iter < 32 && nn > 0; iter++) {
        uint8_t *act = act_.ensure(nn + 1);
        int64_t *c = ncnt_.ensure(nn + 1);
        int64_t *pos = npos_.ensure(nn + 1);
        uint32_t *xlist = xlist_.ensure(nn + 1);
        hipLaunchKernelGGL(k_expand_count, dim3(grid_for(nn, 64)), dim3(64), 0, s, nn, F->f.p, F->i.p, F->j.p, F->meta.p,
                           act, c, xoff, xyz, mode, fmask, orig, nvx, eoff, clip_f, clip_c, cflags, flags, xlist, xlist_n,
                           any_open);
        hipLaunchKernelGGL(k_expand_exact, dim3((unsigned)std::min<int64_t>(grid_for(nn, 64), 1024)), dim3(64), 0, s, xlist,
                           xlist_n, F->f.p, F->i.p, F->j.p, F->meta.p, act, c, xoff, xyz, mode, orig, nvx);
        exclusive_scan_i64(c, pos, nn, tmp_, s, mail + 5);
        Frontier *G = &fr_[cur ^ 1];
        G->ensure(4 * nn + 1);  // <= 4 children per node: no host round trip before the write
        hipLaunchKernelGGL(k_expand_write, dim3(grid_for(nn, B)), dim3(B), 0, s, nn, F->f.p, F->id.p, F->i.p, F->j.p,
                           F->meta.p, act, pos, G->f.p, G->id.p, G->i.p, G->j.p, G->meta.p, any_open, xlist_n);
        mail_counters(reinterpret_cast<const unsigned int *>(any_open), nullptr, nullptr, mail + 6, s);
        DSS_HIP(hipStreamSynchronize(s));
        const int64_t nn2 = mh[5];
        const int open = (int)mh[6];
        cur ^= 1;
        F = G;
        nn = nn2;
        if (!open) break;
    }
    // per-footprint counts (direct: from the scan; descent: item atomics) -> CSR
    unsigned long long *dcnt = fcnt_.ensure(n + 1);
    DSS_HIP(hipMemsetAsync(dcnt, 0, sizeof(unsigned long long) * (n + 1), s));
    int64_t *icnt = ncnt_.ensure(nn + 1), *ipos = npos_.ensure(nn + 1);
    if (nn > 0)
        hipLaunchKernelGGL(k_item_counts, dim3(grid_for(nn, kItemBlock)), dim3(kItemBlock), 0, s, nn, F->f.p, F->meta.p,
                           icnt, dcnt, any_open /* = nbig */);
    int64_t *tot64 = fc64_.ensure(n + 1), *dc64 = dc64_.ensure(n + 1), *dpre = dpre_.ensure(n + 1);
    hipLaunchKernelGGL(k_counts, dim3(grid_for(n, B)), dim3(B), 0, s, n, flags, fkm, dcnt, tot64, dc64);
    exclusive_scan_i64(tot64, offs, n, tmp_, s, mail + 7);
    if (nn > 0) {
        exclusive_scan_i64(icnt, ipos, nn, tmp_, s);
        exclusive_scan_i64(dc64, dpre, n, tmp_, s);
    }
    DSS_HIP(hipStreamSynchronize(s));
    const int64_t total = mh[7];
    uint64_t *cells = cells_.ensure(total + 1);
    hipLaunchKernelGGL(k_cand_emit, dim3(grid_for(n, B)), dim3(B), 0, s, n, flags, fkm, st_id, finfo, offs, cells);
    if (nn > 0) {
        uint32_t *big = big_.ensure(nn + 1);
        int *nbig = any_open;  // (the flag word, zeroed by k_item_counts)
        hipLaunchKernelGGL(k_emit, dim3(grid_for(nn, B)), dim3(B), 0, s, nn, F->f.p, F->id.p, F->meta.p, ipos, dpre, offs,
                           cells, big, nbig);
        hipLaunchKernelGGL(k_emit_big, dim3((unsigned)std::min<int64_t>(nn, 256)), dim3(256), 0, s, big,
                           (const int *)nbig, F->f.p, F->id.p, F->meta.p, ipos, dpre, offs, cells);
    }
    out->offs = offs;
    out->cells = cells;
    out->status = status;
    out->area_km2 = area;
    out->total_cells = total;
}

}  // namespace dss
