// S2 geometry primitives for the gfx950 covering kernels.
//
// Semantics restated from github.com/golang/geo v0.0.0-20190916061304-5b978397cfec
// (pinned by reference go.mod:15; not vendored).  File names below are that
// package's.  All arithmetic is float64 with -ffp-contract=off; exact signs
// (s2/predicates.go computes them with big.Float) use floating-point
// expansions whose products are exact via explicit FMA.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "gomath.cuh"

namespace dss {
namespace s2 {

using namespace gomath;

struct V3 {
    double x, y, z;
};
DSS_HD V3 v3(double x, double y, double z) { return V3{x, y, z}; }
DSS_HD V3 add(V3 a, V3 b) { return v3(a.x + b.x, a.y + b.y, a.z + b.z); }
DSS_HD V3 sub(V3 a, V3 b) { return v3(a.x - b.x, a.y - b.y, a.z - b.z); }
DSS_HD V3 mul(V3 a, double m) { return v3(m * a.x, m * a.y, m * a.z); }
DSS_HD double dot(V3 a, V3 b) { return a.x * b.x + a.y * b.y + a.z * b.z; }
DSS_HD V3 cross(V3 a, V3 b) { return v3(a.y * b.z - a.z * b.y, a.z * b.x - a.x * b.z, a.x * b.y - a.y * b.x); }
DSS_HD double norm(V3 a) { return __builtin_sqrt(dot(a, a)); }
DSS_HD bool eq(V3 a, V3 b) { return a.x == b.x && a.y == b.y && a.z == b.z; }
// r3/vector.go Normalize
DSS_HD V3 normalize(V3 a)
{
    double n2 = dot(a, a);
    if (n2 == 0) return v3(0, 0, 0);
    return mul(a, 1 / __builtin_sqrt(n2));
}
// r3/vector.go LargestComponent (0=X, 1=Y, 2=Z)
DSS_HD int largest(V3 v)
{
    double ax = __builtin_fabs(v.x), ay = __builtin_fabs(v.y), az = __builtin_fabs(v.z);
    if (ax > ay) return ax > az ? 0 : 2;
    return ay > az ? 1 : 2;
}
// r3/vector.go Ortho
DSS_HD V3 ortho(V3 v)
{
    int k = largest(v);
    V3 ov = v3(k == 1 ? 1.0 : 0.012, k == 2 ? 1.0 : 0.0053, k == 0 ? 1.0 : 0.00457);
    return normalize(cross(v, ov));
}
// r3/vector.go Angle
DSS_HD double angle(V3 a, V3 b) { return go_atan2(norm(cross(a, b)), dot(a, b)); }
// r3/vector.go Cmp
DSS_HD int cmp(V3 a, V3 b)
{
    if (a.x != b.x) return a.x < b.x ? -1 : 1;
    if (a.y != b.y) return a.y < b.y ? -1 : 1;
    if (a.z != b.z) return a.z < b.z ? -1 : 1;
    return 0;
}
// point.go PointCross
DSS_HD V3 point_cross(V3 p, V3 op)
{
    V3 x = cross(add(p, op), sub(op, p));
    if (x.x == 0 && x.y == 0 && x.z == 0) return ortho(p);
    return x;
}
// point.go OriginPoint
DSS_HD V3 origin_point() { return v3(-0.0099994664350250197, 0.0025924542609324121, 0.99994664350250195); }

// latlng.go PointFromLatLng(LatLngFromDegrees(lat, lng))
DSS_HD V3 point_from_degrees(double lat, double lng)
{
    double phi = lat * DSS_DEGREE, theta = lng * DSS_DEGREE;
    double cosphi = go_cos(phi);
    return v3(go_cos(theta) * cosphi, go_sin(theta) * cosphi, go_sin(phi));
}

// ------------------------------------------------------------- exact signs
namespace exact {
DSS_HD void two_sum(double a, double b, double &x, double &y)
{
    x = a + b;
    double bv = x - a, av = x - bv;
    y = (a - av) + (b - bv);
}
DSS_HD void two_prod(double a, double b, double &x, double &y)
{
    x = a * b;
    y = __builtin_fma(a, b, -x);
}
// Grow-expansion of `n` arbitrary terms into a nonoverlapping expansion of
// increasing magnitude; returns the sign of the sum (sign of the largest
// component).  n <= 24 on every call site.
DSS_HD int sum_sign(const double *t, int n)
{
    double e[24];
    int m = 0;
    for (int i = 0; i < n; i++) {
        double q = t[i];
        for (int k = 0; k < m; k++) {
            double s, err;
            two_sum(q, e[k], s, err);
            e[k] = err;
            q = s;
        }
        e[m++] = q;
    }
    for (int k = m - 1; k >= 0; k--) {
        if (e[k] > 0) return 1;
        if (e[k] < 0) return -1;
    }
    return 0;
}
// sign(a*b - c*d), exact
DSS_HD int diff_prod_sign(double a, double b, double c, double d)
{
    double t[4];
    two_prod(a, b, t[1], t[0]);
    two_prod(c, d, t[3], t[2]);
    t[2] = -t[2];
    t[3] = -t[3];
    return sum_sign(t, 4);
}
DSS_HD int fsgn(double x) { return (x > 0) - (x < 0); }
}  // namespace exact

enum { CLOCKWISE = -1, INDETERMINATE = 0, COUNTERCLOCKWISE = 1 };

// predicates.go triageSign
DSS_HD int triage_sign(V3 a, V3 b, V3 c)
{
    double det = dot(cross(a, b), c);
    if (det > DSS_MAX_DET_ERR) return COUNTERCLOCKWISE;
    if (det < -DSS_MAX_DET_ERR) return CLOCKWISE;
    return INDETERMINATE;
}

// predicates.go exactSign + symbolicallyPerturbedSign
__host__ __device__ __noinline__ inline int exact_sign(V3 a, V3 b, V3 c)
{
    using namespace exact;
    int perm = 1;
    V3 t;
    if (cmp(a, b) > 0) { t = a; a = b; b = t; perm = -perm; }
    if (cmp(b, c) > 0) { t = b; b = c; c = t; perm = -perm; }
    if (cmp(a, b) > 0) { t = a; a = b; b = t; perm = -perm; }
    // det = a . (b x c): 6 triple products, each expanded exactly (4 terms).
    double terms[24];
    double bx[3][4];  // (b x c) components as 4-term expansions
    two_prod(b.y, c.z, bx[0][1], bx[0][0]);
    two_prod(b.z, c.y, bx[0][3], bx[0][2]);
    two_prod(b.z, c.x, bx[1][1], bx[1][0]);
    two_prod(b.x, c.z, bx[1][3], bx[1][2]);
    two_prod(b.x, c.y, bx[2][1], bx[2][0]);
    two_prod(b.y, c.x, bx[2][3], bx[2][2]);
    const double ac[3] = {a.x, a.y, a.z};
    int n = 0;
    for (int k = 0; k < 3; k++)
        for (int q = 0; q < 4; q++) {
            double s = q < 2 ? bx[k][q] : -bx[k][q];
            double p, e;
            two_prod(s, ac[k], p, e);
            terms[n++] = e;
            terms[n++] = p;
        }
    int ds = sum_sign(terms, 24);
    if (ds != 0) return perm * ds;
    // symbolic perturbation (inputs sorted, b x c exact)
    double bc2[4] = {bx[2][0], bx[2][1], -bx[2][2], -bx[2][3]};
    double bc1[4] = {bx[1][0], bx[1][1], -bx[1][2], -bx[1][3]};
    double bc0[4] = {bx[0][0], bx[0][1], -bx[0][2], -bx[0][3]};
    int s;
    if ((s = sum_sign(bc2, 4)) != 0) return perm * s;                  // da.z
    if ((s = sum_sign(bc1, 4)) != 0) return perm * s;                  // da.y
    if ((s = sum_sign(bc0, 4)) != 0) return perm * s;                  // da.x
    if ((s = diff_prod_sign(c.x, a.y, c.y, a.x)) != 0) return perm * s; // db.z
    if ((s = fsgn(c.x)) != 0) return perm * s;                         // db.z*da.y
    if ((s = -fsgn(c.y)) != 0) return perm * s;                        // db.z*da.x
    if ((s = diff_prod_sign(c.z, a.x, c.x, a.z)) != 0) return perm * s; // db.y
    if ((s = fsgn(c.z)) != 0) return perm * s;                         // db.y*da.x
    if ((s = diff_prod_sign(a.x, b.y, a.y, b.x)) != 0) return perm * s; // dc.z
    if ((s = -fsgn(b.x)) != 0) return perm * s;                        // dc.z*da.y
    if ((s = fsgn(b.y)) != 0) return perm * s;                         // dc.z*da.x
    if ((s = fsgn(a.x)) != 0) return perm * s;                         // dc.z*db.y
    return perm;                                                        // dc.z*db.y*da.x
}

// predicates.go expensiveSign (stableSign only short-cuts to the exact sign)
DSS_HD int expensive_sign(V3 a, V3 b, V3 c)
{
    if (eq(a, b) || eq(b, c) || eq(c, a)) return INDETERMINATE;
    return exact_sign(a, b, c);
}
// predicates.go RobustSign
DSS_HD int robust_sign(V3 a, V3 b, V3 c)
{
    int s = triage_sign(a, b, c);
    return s != INDETERMINATE ? s : expensive_sign(a, b, c);
}
// predicates.go OrderedCCW
DSS_HD bool ordered_ccw(V3 a, V3 b, V3 c, V3 o)
{
    int sum = 0;
    if (robust_sign(b, o, a) != CLOCKWISE) sum++;
    if (robust_sign(c, o, b) != CLOCKWISE) sum++;
    if (robust_sign(a, o, c) == COUNTERCLOCKWISE) sum++;
    return sum >= 2;
}
// edge_crossings.go VertexCrossing
DSS_HD bool vertex_crossing(V3 a, V3 b, V3 c, V3 d)
{
    if (eq(a, b) || eq(c, d)) return false;
    if (eq(a, c)) return eq(b, d) || ordered_ccw(ortho(a), d, b, a);
    if (eq(b, d)) return ordered_ccw(ortho(b), c, a, b);
    if (eq(a, d)) return eq(b, c) || ordered_ccw(ortho(a), c, b, a);
    if (eq(b, c)) return ordered_ccw(ortho(b), d, a, b);
    return false;
}
// AngleContainsVertex
DSS_HD bool angle_contains_vertex(V3 a, V3 b, V3 c) { return !ordered_ccw(ortho(b), c, a, b); }

// edge_crosser.go
enum { DO_NOT_CROSS = -1, MAYBE_CROSS = 0, CROSS = 1 };
struct EdgeCrosser {
    V3 a, b, a_tangent, b_tangent, c;
    int acb;
    DSS_HD void init(V3 a_, V3 b_)
    {
        a = a_;
        b = b_;
        V3 n = point_cross(a_, b_);
        a_tangent = cross(a_, n);
        b_tangent = cross(n, b_);
        c = v3(0, 0, 0);
        acb = 0;
    }
    DSS_HD void restart_at(V3 c_)
    {
        c = c_;
        acb = -triage_sign(a, b, c_);
    }
    __host__ __device__ __noinline__ int crossing_sign_slow(V3 d, int bda)
    {
        int result;
        const double max_error = (1.5 + 1 / __builtin_sqrt(3.0)) * DSS_DBL_EPS;
        if ((dot(c, a_tangent) > max_error && dot(d, a_tangent) > max_error) ||
            (dot(c, b_tangent) > max_error && dot(d, b_tangent) > max_error)) {
            result = DO_NOT_CROSS;
        } else if (eq(a, c) || eq(a, d) || eq(b, c) || eq(b, d)) {
            result = MAYBE_CROSS;
        } else if (eq(a, b) || eq(c, d)) {
            result = DO_NOT_CROSS;
        } else {
            if (acb == INDETERMINATE) acb = -expensive_sign(a, b, c);
            if (bda == INDETERMINATE) bda = expensive_sign(a, b, d);
            if (bda != acb) result = DO_NOT_CROSS;
            else if (-robust_sign(c, d, b) != acb) result = DO_NOT_CROSS;
            else if (robust_sign(c, d, a) != acb) result = DO_NOT_CROSS;
            else result = CROSS;
        }
        c = d;
        acb = -bda;
        return result;
    }
    DSS_HD int chain_crossing_sign(V3 d)
    {
        int bda = triage_sign(a, b, d);
        if (acb == -bda && bda != INDETERMINATE) {
            c = d;
            acb = -bda;
            return DO_NOT_CROSS;
        }
        return crossing_sign_slow(d, bda);
    }
    DSS_HD bool edge_or_vertex_chain_crossing(V3 d)
    {
        V3 c0 = c;
        int s = chain_crossing_sign(d);
        if (s == DO_NOT_CROSS) return false;
        if (s == CROSS) return true;
        return vertex_crossing(a, b, c0, d);
    }
};

// ------------------------------------------------- triage-only predicates
// Variants for the hot kernels: they never reach the exact arithmetic
// (exact_sign / crossing_sign_slow are out-of-line calls whose ABI spills
// would dominate a one-thread-per-footprint kernel).  A case the triage
// cannot decide sets `fail`; the caller then recomputes that footprint on
// the exact path.  Whenever `fail` stays false the result equals the exact
// predicate's (triage_sign is exact when it decides).
namespace fastp {
DSS_HD int robust_sign(V3 a, V3 b, V3 c, bool &fail)
{
    int s = triage_sign(a, b, c);
    // expensive_sign answers INDETERMINATE itself for repeated points (the
    // closed rings of the prober fixtures); only the rest needs exact_sign
    if (s == INDETERMINATE && !(eq(a, b) || eq(b, c) || eq(c, a))) fail = true;
    return s;
}
DSS_HD bool ordered_ccw(V3 a, V3 b, V3 c, V3 o, bool &fail)
{
    int sum = 0;
    if (robust_sign(b, o, a, fail) != CLOCKWISE) sum++;
    if (robust_sign(c, o, b, fail) != CLOCKWISE) sum++;
    if (robust_sign(a, o, c, fail) == COUNTERCLOCKWISE) sum++;
    return sum >= 2;
}
DSS_HD bool vertex_crossing(V3 a, V3 b, V3 c, V3 d, bool &fail)
{
    if (eq(a, b) || eq(c, d)) return false;
    if (eq(a, c)) return eq(b, d) || ordered_ccw(ortho(a), d, b, a, fail);
    if (eq(b, d)) return ordered_ccw(ortho(b), c, a, b, fail);
    if (eq(a, d)) return eq(b, c) || ordered_ccw(ortho(a), c, b, a, fail);
    if (eq(b, c)) return ordered_ccw(ortho(b), d, a, b, fail);
    return false;
}
DSS_HD bool angle_contains_vertex(V3 a, V3 b, V3 c, bool &fail) { return !ordered_ccw(ortho(b), c, a, b, fail); }
// EdgeCrosser::chain_crossing_sign with crossing_sign_slow inlined minus
// its expensive_sign calls.
DSS_HD int chain_crossing_sign(EdgeCrosser &x, V3 d, bool &fail)
{
    const int bda = triage_sign(x.a, x.b, d);
    if (x.acb == -bda && bda != INDETERMINATE) {
        x.c = d;
        x.acb = -bda;
        return DO_NOT_CROSS;
    }
    int result;
    const double max_error = (1.5 + 1 / __builtin_sqrt(3.0)) * DSS_DBL_EPS;
    if ((dot(x.c, x.a_tangent) > max_error && dot(d, x.a_tangent) > max_error) ||
        (dot(x.c, x.b_tangent) > max_error && dot(d, x.b_tangent) > max_error)) {
        result = DO_NOT_CROSS;
    } else if (eq(x.a, x.c) || eq(x.a, d) || eq(x.b, x.c) || eq(x.b, d)) {
        result = MAYBE_CROSS;
    } else if (eq(x.a, x.b) || eq(x.c, d)) {
        result = DO_NOT_CROSS;
    } else if (x.acb == INDETERMINATE || bda == INDETERMINATE) {
        fail = true;
        result = DO_NOT_CROSS;
    } else if (bda != x.acb) {
        result = DO_NOT_CROSS;
    } else if (-robust_sign(x.c, d, x.b, fail) != x.acb) {
        result = DO_NOT_CROSS;
    } else if (robust_sign(x.c, d, x.a, fail) != x.acb) {
        result = DO_NOT_CROSS;
    } else {
        result = CROSS;
    }
    x.c = d;
    x.acb = -bda;
    return result;
}
DSS_HD bool edge_or_vertex_chain_crossing(EdgeCrosser &x, V3 d, bool &fail)
{
    const V3 c0 = x.c;
    const int s = chain_crossing_sign(x, d, fail);
    if (s == DO_NOT_CROSS) return false;
    if (s == CROSS) return true;
    return vertex_crossing(x.a, x.b, c0, d, fail);
}
}  // namespace fastp

// ------------------------------------------------------------ projections
// stuv.go (quadratic projection)
constexpr int kMaxLevel = 30;
constexpr int kMaxSize = 1 << kMaxLevel;
constexpr int kCoverLevel = 13;  // pkg/geo/s2.go:19-22 min = max level

DSS_HD double st_to_uv(double s)
{
    if (s >= 0.5) return DSS_ONE_THIRD * (4 * s * s - 1);
    return DSS_ONE_THIRD * (1 - 4 * (1 - s) * (1 - s));
}
DSS_HD double uv_to_st(double u)
{
    if (u >= 0) return 0.5 * __builtin_sqrt(1 + 3 * u);
    return 1 - 0.5 * __builtin_sqrt(1 - 3 * u);
}
DSS_HD int st_to_ij(double s)
{
    double f = __builtin_floor((double)kMaxSize * s);
    if (!(f >= 0)) return 0;  // also NaN
    if (f > (double)(kMaxSize - 1)) return kMaxSize - 1;
    return (int)f;
}
DSS_HD int xyz_face(V3 r)
{
    int f = largest(r);
    double c = f == 0 ? r.x : (f == 1 ? r.y : r.z);
    return c < 0 ? f + 3 : f;
}
DSS_HD void valid_face_xyz_to_uv(int face, V3 r, double &u, double &v)
{
    switch (face) {
    case 0: u = r.y / r.x; v = r.z / r.x; break;
    case 1: u = -r.x / r.y; v = r.z / r.y; break;
    case 2: u = -r.x / r.z; v = -r.y / r.z; break;
    case 3: u = r.z / r.x; v = r.y / r.x; break;
    case 4: u = r.z / r.y; v = -r.x / r.y; break;
    default: u = -r.y / r.z; v = -r.x / r.z; break;
    }
}
DSS_HD bool face_xyz_to_uv(int face, V3 p, double &u, double &v)
{
    double c = (face % 3 == 0) ? p.x : (face % 3 == 1 ? p.y : p.z);
    if (face < 3 ? !(c > 0) : !(c < 0)) return false;
    valid_face_xyz_to_uv(face, p, u, v);
    return true;
}
DSS_HD V3 face_uv_to_xyz(int face, double u, double v)
{
    switch (face) {
    case 0: return v3(1, u, v);
    case 1: return v3(-u, 1, v);
    case 2: return v3(-u, -v, 1);
    case 3: return v3(-1, -v, -u);
    case 4: return v3(v, -1, -u);
    default: return v3(v, u, -1);
    }
}
DSS_HD V3 face_xyz_to_uvw(int face, V3 p)
{
    switch (face) {
    case 0: return v3(p.y, p.z, p.x);
    case 1: return v3(-p.x, p.z, p.y);
    case 2: return v3(-p.x, -p.y, p.z);
    case 3: return v3(-p.z, -p.y, -p.x);
    case 4: return v3(-p.z, p.x, -p.y);
    default: return v3(p.y, p.x, -p.z);
    }
}

// ----------------------------------------------------------- edge clipping
// edge_clipping.go
DSS_HD bool uvw_intersects_face(V3 n)
{
    double u = __builtin_fabs(n.x), v = __builtin_fabs(n.y), w = __builtin_fabs(n.z);
    return (v >= w - u) && (u >= w - v);
}
DSS_HD bool uvw_intersects_opposite_edges(V3 n)
{
    double u = __builtin_fabs(n.x), v = __builtin_fabs(n.y), w = __builtin_fabs(n.z);
    double d = __builtin_fabs(u - v);
    if (d != w) return d >= w;
    return u >= v ? (u - w >= v) : (v - w >= u);
}
DSS_HD int uvw_exit_axis(V3 n)
{
    if (uvw_intersects_opposite_edges(n)) return __builtin_fabs(n.x) >= __builtin_fabs(n.y) ? 1 : 0;
    int x = __builtin_signbit(n.x) ? 1 : 0, y = __builtin_signbit(n.y) ? 1 : 0, z = __builtin_signbit(n.z) ? 1 : 0;
    return ((x ^ y ^ z) == 0) ? 1 : 0;
}
DSS_HD void uvw_exit_point(V3 n, int axis, double &pu, double &pv)
{
    if (axis == 0) {
        double u = n.y > 0 ? 1.0 : -1.0;
        pu = u;
        pv = (-u * n.x - n.z) / n.y;
    } else {
        double v = n.x < 0 ? 1.0 : -1.0;
        pu = (-v * n.y - n.z) / n.x;
        pv = v;
    }
}
DSS_HD int clip_destination(V3 a, V3 b, V3 scaled_n, V3 a_tan, V3 b_tan, double scale_uv, double &ou, double &ov)
{
    double u, v;
    if (b.z > 0) {
        u = b.x / b.z;
        v = b.y / b.z;
        if (go_max(__builtin_fabs(u), __builtin_fabs(v)) <= DSS_MAX_SAFE_UV_COORD) {
            ou = u;
            ov = v;
            return 0;
        }
    }
    uvw_exit_point(scaled_n, uvw_exit_axis(scaled_n), u, v);
    u = scale_uv * u;
    v = scale_uv * v;
    V3 p = v3(u, v, 1.0);
    int score = 0;
    if (dot(sub(p, a), a_tan) < 0) score = 2;
    else if (dot(sub(p, b), b_tan) < 0) score = 1;
    if (score > 0) {
        if (b.z <= 0) score = 3;
        else { u = b.x / b.z; v = b.y / b.z; }
    }
    ou = u;
    ov = v;
    return score;
}
// edge_clipping.go ClipToPaddedFace -> uv = (au, av, bu, bv)
DSS_HD bool clip_to_padded_face(V3 a, V3 b, int f, double padding, double *uv)
{
    if (xyz_face(a) == f && xyz_face(b) == f) {
        valid_face_xyz_to_uv(f, a, uv[0], uv[1]);
        valid_face_xyz_to_uv(f, b, uv[2], uv[3]);
        return true;
    }
    V3 norm_uvw = face_xyz_to_uvw(f, point_cross(a, b));
    V3 a_uvw = face_xyz_to_uvw(f, a);
    V3 b_uvw = face_xyz_to_uvw(f, b);
    double scale_uv = 1 + padding;
    V3 scaled_n = v3(scale_uv * norm_uvw.x, scale_uv * norm_uvw.y, norm_uvw.z);
    if (!uvw_intersects_face(scaled_n)) return false;
    norm_uvw = normalize(norm_uvw);
    V3 a_tan = cross(norm_uvw, a_uvw);
    V3 b_tan = cross(b_uvw, norm_uvw);
    int as = clip_destination(b_uvw, a_uvw, mul(scaled_n, -1), b_tan, a_tan, scale_uv, uv[0], uv[1]);
    int bs = clip_destination(a_uvw, b_uvw, scaled_n, a_tan, b_tan, scale_uv, uv[2], uv[3]);
    return as + bs < 3;
}
// edge_clipping.go edgeIntersectsRect; rect = [ulo,uhi] x [vlo,vhi]
DSS_HD bool edge_intersects_rect(double au, double av, double bu, double bv, double ulo, double uhi, double vlo,
                                 double vhi)
{
    double blu = au < bu ? au : bu, bhu = au > bu ? au : bu;
    double blv = av < bv ? av : bv, bhv = av > bv ? av : bv;
    if (bu != bu || au != au) { blu = au; bhu = au; }  // NaN: keep Go's AddPoint order semantics
    bool xi = (ulo <= blu) ? (blu <= uhi && blu <= bhu) : (ulo <= bhu && ulo <= uhi);
    bool yi = (vlo <= blv) ? (blv <= vhi && blv <= bhv) : (vlo <= bhv && vlo <= vhi);
    if (!(xi && yi)) return false;
    double nx = -(bv - av), ny = bu - au;
    bool i = nx >= 0, j = ny >= 0;
    double mx = nx * ((i ? uhi : ulo) - au) + ny * ((j ? vhi : vlo) - av);
    double mn = nx * ((i ? ulo : uhi) - au) + ny * ((j ? vlo : vhi) - av);
    return (mx >= 0) && (mn <= 0);
}

// ------------------------------------------------------------ Hilbert / ids
// cellid.go: position <-> (i, j) per level, no lookup tables needed because
// the kernels only walk one level at a time.
// kIJtoPos = {{0,1,3,2},{0,3,1,2},{2,3,1,0},{2,1,3,0}}, kPosToIJ =
// {{0,1,3,2},{0,2,3,1},{3,2,0,1},{3,1,0,2}}, kPosToOrientation = {1,0,0,3},
// packed 2 bits per entry, 8 bits per orientation row.
DSS_HD int ij_to_pos(int orientation, int ij) { return (int)((0x361E9CB4u >> (8 * orientation + 2 * ij)) & 3u); }
DSS_HD int pos_to_ij(int orientation, int pos) { return (int)((0x874B78B4u >> (8 * orientation + 2 * pos)) & 3u); }
DSS_HD int pos_to_orientation(int pos) { return (int)((0xC1u >> (2 * pos)) & 3u); }  // {1,0,0,3}

DSS_HD uint64_t lsb_for_level(int level) { return 1ull << (2 * (kMaxLevel - level)); }
DSS_HD uint64_t cellid_lsb_dev(uint64_t id) { return id & (~id + 1); }

// cellid.go cellIDFromFaceIJ truncated to `level`, plus the Hilbert
// orientation of that cell (needed to enumerate its children in id order).
DSS_HD uint64_t cell_from_face_ij_level(int face, int i, int j, int level, int &orientation)
{
    int o = face & 1;
    uint64_t pos = 0;
    for (int l = 1; l <= level; l++) {
        int ib = (i >> (kMaxLevel - l)) & 1, jb = (j >> (kMaxLevel - l)) & 1;
        int p = ij_to_pos(o, (ib << 1) | jb);
        pos = (pos << 2) | (uint64_t)p;
        o ^= pos_to_orientation(p);
    }
    orientation = o;
    // id = face<<61 | pos << (61 - 2*level) | lsb
    uint64_t lsb = lsb_for_level(level);
    return ((uint64_t)face << 61) | (pos << (2 * (kMaxLevel - level) + 1)) | lsb;
}
}  // namespace s2
}  // namespace dss
