// s2.Loop pieces the DSS covering path needs, for one footprint per thread.
//
// Restated from golang/geo v0.0.0-20190916061304-5b978397cfec s2/loop.go
// (initOriginAndBound, bruteForceContainsPoint, Area, surfaceIntegral,
// IsNormalized, TurningAngle, turningAngleMaxError), s2/point_measures.go
// (PointArea, GirardArea, SignedArea, TurnAngle), s2/rect_bounder.go and the
// s1/r1 interval arithmetic it uses.  Vertices live in global memory.
// The loop bound is only consulted by IsNormalized, which Area only calls for
// near-zero or near-4*pi areas, so it is computed lazily here.
#pragma once
#include "s2dev.cuh"

namespace dss {
namespace s2 {

struct LoopView {
    const V3 *v;
    int n;
    bool origin_inside;
    bool rev = false;  // the loop is v[n-1], ..., v[0]: Q4's reversal without moving the vertices
    DSS_HD V3 vertex(int i) const
    {
        const int k = i % n;
        return v[rev ? n - 1 - k : k];
    }
    DSS_HD V3 at(int i) const { return v[rev ? n - 1 - i : i]; }  // 0 <= i < n
};

// loop.go bruteForceContainsPoint
DSS_HD bool loop_contains(const LoopView &l, V3 p)
{
    EdgeCrosser e;
    e.init(origin_point(), p);
    e.restart_at(l.vertex(0));
    bool inside = l.origin_inside;
    for (int i = 1; i <= l.n; i++) inside = inside != e.edge_or_vertex_chain_crossing(l.vertex(i));
    return inside;
}

// loop.go initOriginAndBound (origin part; n >= 3 on every DSS path)
DSS_HD void loop_init_origin(LoopView &l)
{
    bool v1_inside = !eq(l.v[0], l.v[1]) && !eq(l.v[2], l.v[1]) && angle_contains_vertex(l.v[0], l.v[1], l.v[2]);
    l.origin_inside = false;
    if (v1_inside != loop_contains(l, l.v[1])) l.origin_inside = true;
}

// -------------------------------------------------------- interval algebra
struct Ival {
    double lo, hi;
};
namespace iv {
DSS_HD Ival s1_empty() { return Ival{DSS_PI, -DSS_PI}; }
DSS_HD Ival s1_full() { return Ival{-DSS_PI, DSS_PI}; }
DSS_HD bool s1_is_full(Ival i) { return i.lo == -DSS_PI && i.hi == DSS_PI; }
DSS_HD bool s1_is_empty(Ival i) { return i.lo == DSS_PI && i.hi == -DSS_PI; }
DSS_HD bool s1_inverted(Ival i) { return i.lo > i.hi; }
DSS_HD double s1_length(Ival i)
{
    double l = i.hi - i.lo;
    if (l >= 0) return l;
    l += 2 * DSS_PI;
    return l > 0 ? l : -1;
}
DSS_HD bool s1_fast_contains(Ival i, double p)
{
    if (s1_inverted(i)) return (p >= i.lo || p <= i.hi) && !s1_is_empty(i);
    return p >= i.lo && p <= i.hi;
}
DSS_HD double pos_dist(double a, double b)
{
    double d = b - a;
    if (d >= 0) return d;
    return (b + DSS_PI) - (a - DSS_PI);
}
DSS_HD Ival s1_add_point(Ival i, double p)
{
    if (__builtin_fabs(p) > DSS_PI) return i;
    if (p == -DSS_PI) p = DSS_PI;
    if (s1_fast_contains(i, p)) return i;
    if (s1_is_empty(i)) return Ival{p, p};
    if (pos_dist(p, i.lo) < pos_dist(i.hi, p)) return Ival{p, i.hi};
    return Ival{i.lo, p};
}
DSS_HD bool s1_contains_interval(Ival i, Ival o)
{
    if (s1_inverted(i)) {
        if (s1_inverted(o)) return o.lo >= i.lo && o.hi <= i.hi;
        return (o.lo >= i.lo || o.hi <= i.hi) && !s1_is_empty(i);
    }
    if (s1_inverted(o)) return s1_is_full(i) || s1_is_empty(o);
    return o.lo >= i.lo && o.hi <= i.hi;
}
DSS_HD Ival s1_union(Ival i, Ival o)
{
    if (s1_is_empty(o)) return i;
    if (s1_fast_contains(i, o.lo)) {
        if (s1_fast_contains(i, o.hi)) return s1_contains_interval(i, o) ? i : s1_full();
        return Ival{i.lo, o.hi};
    }
    if (s1_fast_contains(i, o.hi)) return Ival{o.lo, i.hi};
    if (s1_is_empty(i) || s1_fast_contains(o, i.lo)) return o;
    if (pos_dist(o.hi, i.lo) < pos_dist(i.hi, o.lo)) return Ival{o.lo, i.hi};
    return Ival{i.lo, o.hi};
}
DSS_HD bool r1_empty(Ival i) { return i.lo > i.hi; }
DSS_HD Ival r1_add(Ival i, double p)
{
    if (r1_empty(i)) return Ival{p, p};
    if (p < i.lo) return Ival{p, i.hi};
    if (p > i.hi) return Ival{i.lo, p};
    return i;
}
DSS_HD Ival r1_union(Ival i, Ival o)
{
    if (r1_empty(i)) return o;
    if (r1_empty(o)) return i;
    return Ival{go_min(i.lo, o.lo), go_max(i.hi, o.hi)};
}
}  // namespace iv

// math.Remainder(x, 2*Pi) for the interval endpoints s1.Interval.Expanded
// sees: they come from atan2, so |x| <= Pi, where the IEEE remainder is x
// itself (a quotient of +-0.5 rounds to the even 0).
DSS_HD double rem_2pi(double x)
{
    if (__builtin_fabs(x) <= DSS_PI) return x;
    double q = __builtin_rint(x / (2 * DSS_PI));  // not reached on the DSS path
    return x - q * (2 * DSS_PI);
}

// rect_bounder.go RectBounder.AddPoint over the closed vertex chain, then
// RectBound() (expanded by 2*dblEpsilon in latitude, PolarClosure).
// Returns the longitude interval length; pole containment adjusts it in
// loop_bound_lng_length below (loop.go initBound).
DSS_HD double point_lat(V3 p) { return go_atan2(p.z, __builtin_sqrt(p.x * p.x + p.y * p.y)); }
DSS_HD double point_lng(V3 p) { return go_atan2(p.y, p.x); }

__host__ __device__ __noinline__ inline double loop_bound_lng_length(const LoopView &l)
{
    using namespace iv;
    Ival lat{1, 0}, lng = s1_empty();
    V3 a = v3(0, 0, 0);
    double alat = 0, alng = 0;
    for (int k = 0; k <= l.n; k++) {
        V3 b = l.vertex(k);
        double blat = point_lat(b), blng = point_lng(b);
        bool valid = __builtin_fabs(blat) <= DSS_PI_2 && __builtin_fabs(blng) <= DSS_PI;
        if (r1_empty(lat)) {
            a = b;
            alat = blat;
            alng = blng;
            if (valid) { lat = r1_add(lat, blat); lng = s1_add_point(lng, blng); }
            continue;
        }
        V3 nn = cross(sub(a, b), add(a, b));
        double n_norm = norm(nn);
        if (n_norm < 1.91346e-15) {
            if (dot(a, b) < 0) {
                lat = Ival{-DSS_PI_2, DSS_PI_2};
                lng = s1_full();
            } else {
                Ival plat{alat, alat}, plng{alng, alng};
                if (valid) { plat = r1_add(plat, blat); plng = s1_add_point(plng, blng); }
                lat = r1_union(lat, plat);
                lng = s1_union(lng, plng);
            }
            a = b;
            alat = blat;
            alng = blng;
            continue;
        }
        Ival lng_ab = s1_add_point(s1_add_point(s1_empty(), alng), blng);
        if (s1_length(lng_ab) >= DSS_PI_MINUS_2EPS) lng_ab = s1_full();
        Ival lat_ab = r1_add(Ival{alat, alat}, blat);
        V3 m = cross(nn, v3(0, 0, 1));
        double ma = dot(m, a), mb = dot(m, b);
        double m_error = 6.06638e-16 * n_norm + 6.83174e-31;
        if (ma * mb < 0 || __builtin_fabs(ma) <= m_error || __builtin_fabs(mb) <= m_error) {
            double max_lat = go_min(go_atan2(__builtin_sqrt(nn.x * nn.x + nn.y * nn.y), __builtin_fabs(nn.z)) + DSS_THREE_EPS,
                                    DSS_PI_2);
            double lat_budget = 2 * go_asin(0.5 * norm(sub(a, b)) * go_sin(max_lat));
            double max_delta = 0.5 * (lat_budget - (lat_ab.hi - lat_ab.lo)) + DSS_DBL_EPS;
            if (ma <= m_error && mb >= -m_error) lat_ab.hi = go_min(max_lat, lat_ab.hi + max_delta);
            if (mb <= m_error && ma >= -m_error) lat_ab.lo = go_max(-max_lat, lat_ab.lo - max_delta);
        }
        a = b;
        alat = blat;
        alng = blng;
        lat = r1_union(lat, lat_ab);
        lng = s1_union(lng, lng_ab);
    }
    // RectBound(): lat expanded by 2*eps and clamped; lng Expanded(0).
    if (!r1_empty(lat)) { lat.lo = lat.lo - DSS_TWO_EPS; lat.hi = lat.hi + DSS_TWO_EPS; }
    if (!s1_is_empty(lng) && s1_length(lng) + 2 * DSS_DBL_EPS >= 2 * DSS_PI) lng = s1_full();
    else if (!s1_is_empty(lng)) {
        Ival r{rem_2pi(lng.lo), rem_2pi(lng.hi)};
        if (r.lo <= -DSS_PI) r.lo = DSS_PI;
        lng = r;
    }
    if (r1_empty(lat) || s1_is_empty(lng)) return -1;  // EmptyRect: Lng length of EmptyInterval
    lat.lo = go_max(lat.lo, -DSS_PI_2);
    lat.hi = go_min(lat.hi, DSS_PI_2);
    if (lat.lo == -DSS_PI_2 || lat.hi == DSS_PI_2) lng = s1_full();
    // loop.go initBound: north pole inside -> full longitude; south pole only
    // changes latitude.
    if (loop_contains(l, v3(0, 0, 1))) lng = s1_full();
    return s1_length(lng);
}

// point_measures.go
DSS_HD double girard_area(V3 a, V3 b, V3 c)
{
    V3 ab = point_cross(a, b), bc = point_cross(b, c), ac = point_cross(a, c);
    double area = angle(ab, ac) - angle(ab, bc) + angle(bc, ac);
    return area < 0 ? 0 : area;
}
DSS_HD double point_area(V3 a, V3 b, V3 c)
{
    double sa = angle(b, c), sb = angle(c, a), sc = angle(a, b);
    double s = 0.5 * (sa + sb + sc);
    if (s >= 3e-4) {
        double dmin = s - go_max(sa, go_max(sb, sc));
        if (dmin < 1e-2 * s * s * s * s * s) {
            double area = girard_area(a, b, c);
            if (dmin < s * 0.1 * area) return area;
        }
    }
    return 4 * go_atan(__builtin_sqrt(go_max(0.0, go_tan(0.5 * s) * go_tan(0.5 * (s - sa)) * go_tan(0.5 * (s - sb)) *
                                                      go_tan(0.5 * (s - sc)))));
}
DSS_HD double signed_area(V3 a, V3 b, V3 c) { return (double)robust_sign(a, b, c) * point_area(a, b, c); }

// loop.go surfaceIntegralFloat64(SignedArea)
DSS_HD double loop_signed_area_sum(const LoopView &l)
{
    const double max_length = DSS_SURFACE_MAX_LENGTH;
    double sum = 0;
    V3 v0 = l.vertex(0), origin = v0;
    for (int i = 1; i + 1 < l.n; i++) {
        V3 vi = l.vertex(i), vi1 = l.vertex(i + 1);
        if (angle(vi1, origin) > max_length) {
            V3 old = origin;
            if (eq(origin, v0)) {
                origin = normalize(point_cross(v0, vi));
            } else if (angle(vi, v0) < max_length) {
                origin = v0;
            } else {
                origin = cross(v0, old);
                sum += signed_area(v0, old, origin);
            }
            sum += signed_area(old, vi, origin);
        }
        sum += signed_area(origin, vi, vi1);
    }
    if (!eq(origin, v0)) sum += signed_area(origin, l.vertex(l.n - 1), v0);
    return sum;
}
DSS_HD double turn_angle(V3 a, V3 b, V3 c)
{
    double ang = angle(point_cross(a, b), point_cross(b, c));
    return robust_sign(a, b, c) == COUNTERCLOCKWISE ? ang : -ang;
}
DSS_HD double turning_angle_max_error(const LoopView &l) { return DSS_TURN_ANGLE_ERR_PER_VERTEX * (double)l.n; }
// loop.go TurningAngle (Kahan summation from canonicalFirstVertex)
DSS_HD double loop_turning_angle(const LoopView &l)
{
    int n = l.n, first = 0, dir;
    for (int i = 1; i < n; i++)
        if (cmp(l.vertex(i), l.vertex(first)) == -1) first = i;
    if (cmp(l.vertex(first + 1), l.vertex(first + n - 1)) == -1) dir = 1;
    else { first += n; dir = -1; }
    int i = first;
    double sum = turn_angle(l.vertex((i + n - dir) % n), l.vertex(i), l.vertex((i + dir) % n));
    double comp = 0;
    for (int cnt = n; cnt - 1 > 0; cnt--) {
        i += dir;
        double a = turn_angle(l.vertex(i - dir), l.vertex(i), l.vertex(i + dir));
        double old = sum;
        a += comp;
        sum += a;
        comp = (old - sum) + a;
    }
    return (double)dir * (sum + comp);
}
DSS_HD bool loop_is_normalized(const LoopView &l)
{
    if (loop_bound_lng_length(l) < DSS_PI) return true;
    return loop_turning_angle(l) >= -turning_angle_max_error(l);
}
// loop.go Area
DSS_HD double loop_area(const LoopView &l)
{
    double area = loop_signed_area_sum(l);
    double max_error = turning_angle_max_error(l);
    if (area < 0) area += 4 * DSS_PI;
    if (area > 4 * DSS_PI) area = 4 * DSS_PI;
    if (area < 0) area = 0;
    if (area < max_error && !loop_is_normalized(l)) return 4 * DSS_PI;
    if (area > (4 * DSS_PI - max_error) && loop_is_normalized(l)) return 0;
    return area;
}
// pkg/geo/s2.go:89-95 loopAreaKm2 -- (Area * E) / 4.0 * math.Pi (quirk Q1)
DSS_HD double loop_area_km2(const LoopView &l) { return (loop_area(l) * DSS_EARTH_AREA_KM2) / 4.0 * DSS_PI; }

// ------------------------------------------------- triage-only loop pieces
// (s2dev.cuh fastp): same results as the exact versions above whenever
// `fail` stays false; Area fails over to the exact path in the two bands
// where loop.go Area consults IsNormalized (the loop bound).
namespace fastp {
DSS_HD bool loop_contains(const LoopView &l, V3 p, bool &fail)
{
    EdgeCrosser e;
    e.init(origin_point(), p);
    e.restart_at(l.at(0));
    bool inside = l.origin_inside;
    // vertices loaded 4 at a time (independent loads in flight together; the
    // chain itself is evaluated in order, as loop.go does)
    for (int i0 = 1; i0 <= l.n; i0 += 4) {
        V3 q[4];
#pragma unroll
        for (int u = 0; u < 4; u++) {
            const int i = i0 + u <= l.n ? i0 + u : l.n;
            q[u] = l.at(i == l.n ? 0 : i);
        }
#pragma unroll
        for (int u = 0; u < 4; u++)
            if (i0 + u <= l.n) inside = inside != edge_or_vertex_chain_crossing(e, q[u], fail);
    }
    return inside;
}
DSS_HD void loop_init_origin(LoopView &l, bool &fail)
{
    const V3 v0 = l.at(0), v1 = l.at(1), v2 = l.at(2);
    bool v1_inside = !eq(v0, v1) && !eq(v2, v1) && angle_contains_vertex(v0, v1, v2, fail);
    l.origin_inside = false;
    if (v1_inside != loop_contains(l, v1, fail)) l.origin_inside = true;
}
DSS_HD double signed_area(V3 a, V3 b, V3 c, bool &fail) { return (double)robust_sign(a, b, c, fail) * point_area(a, b, c); }
DSS_HD double loop_signed_area_sum(const LoopView &l, bool &fail)
{
    const double max_length = DSS_SURFACE_MAX_LENGTH;
    double sum = 0;
    V3 v0 = l.vertex(0), origin = v0;
    for (int i = 1; i + 1 < l.n; i++) {
        V3 vi = l.vertex(i), vi1 = l.vertex(i + 1);
        if (angle(vi1, origin) > max_length) {
            V3 old = origin;
            if (eq(origin, v0)) {
                origin = normalize(point_cross(v0, vi));
            } else if (angle(vi, v0) < max_length) {
                origin = v0;
            } else {
                origin = cross(v0, old);
                sum += signed_area(v0, old, origin, fail);
            }
            sum += signed_area(old, vi, origin, fail);
        }
        sum += signed_area(origin, vi, vi1, fail);
    }
    if (!eq(origin, v0)) sum += signed_area(origin, l.vertex(l.n - 1), v0, fail);
    return sum;
}
DSS_HD double loop_area_km2(const LoopView &l, bool &fail)
{
    double area = loop_signed_area_sum(l, fail);
    const double max_error = turning_angle_max_error(l);
    if (area < 0) area += 4 * DSS_PI;
    if (area > 4 * DSS_PI) area = 4 * DSS_PI;
    if (area < 0) area = 0;
    fail |= area < max_error || area > (4 * DSS_PI - max_error);
    return (area * DSS_EARTH_AREA_KM2) / 4.0 * DSS_PI;
}
}  // namespace fastp

}  // namespace s2
}  // namespace dss
