/* ORACLE / TEST INFRASTRUCTURE ONLY -- never linked into the product path.
 * Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may
 * load the library built from this file.
 *
 * CPU restatement of the subset of github.com/golang/geo
 * v0.0.0-20190916061304-5b978397cfec (reference go.mod:15, go.sum:58-59; not
 * vendored in /root/reference and not present in this image) that the DSS
 * covering path calls:
 *   - s2.PointFromLatLng / LatLngFromDegrees      (pkg/geo/s2.go:160, pkg/models/geo.go:235,262)
 *   - s2.LoopFromPoints, Loop.Area, Loop.IntersectsCell, Loop.ContainsPoint (pkg/geo/s2.go:94,100,108,121)
 *   - s2.Polyline.IntersectsCell                  (pkg/geo/s2.go:118-119)
 *   - s2.RegularLoop                              (pkg/models/geo.go:234-238)
 *   - s2.RegionCoverer{MinLevel:13,MaxLevel:13}.Covering (pkg/geo/s2.go:30-35)
 * Each function below names the golang/geo file it restates.  Everything is
 * float64 with no FMA contraction (Go 1.14/amd64), see gomath.h.
 *
 * Documented deviation ("pure" IntersectsCell): golang/geo's
 * Loop.IntersectsCell consults the loop's ShapeIndex (Disjoint / Subdivided /
 * index-cell shortcuts) before doing the padded edge test and the
 * cell-centre containment test that are restated here.  Both agree except for
 * cells whose padded bound lies within ~1e-15 (u,v) of a loop edge (about
 * 6 nm on the ground), see SURVEY.md s8(c) "Residual risk" and DESIGN.md.
 *
 * Parity pin: pkg/models/geo_test.go:10-55 (20-cell KAT) and the status-level
 * fixtures of pkg/geo/s2_test.go, checked in tests/test_oracle_kat.py.
 */
#include <stdint.h>
#include <stdlib.h>
#include <string.h>
#include <math.h>

#include "gomath.h"
#include "oracle.h"

/* ------------------------------------------------------------------ r3 */
typedef struct { double x, y, z; } V3;

static inline V3 v3(double x, double y, double z) { V3 r = {x, y, z}; return r; }
static inline V3 v_add(V3 a, V3 b) { return v3(a.x + b.x, a.y + b.y, a.z + b.z); }
static inline V3 v_sub(V3 a, V3 b) { return v3(a.x - b.x, a.y - b.y, a.z - b.z); }
static inline V3 v_mul(V3 a, double m) { return v3(m * a.x, m * a.y, m * a.z); }
static inline double v_dot(V3 a, V3 b) { return a.x * b.x + a.y * b.y + a.z * b.z; }
static inline V3 v_cross(V3 a, V3 b)
{
    return v3(a.y * b.z - a.z * b.y, a.z * b.x - a.x * b.z, a.x * b.y - a.y * b.x);
}
static inline double v_norm2(V3 a) { return v_dot(a, a); }
static inline double v_norm(V3 a) { return sqrt(v_dot(a, a)); }
static inline int v_eq(V3 a, V3 b) { return a.x == b.x && a.y == b.y && a.z == b.z; }
/* r3/vector.go Normalize: multiply by 1/sqrt(n2) */
static inline V3 v_normalize(V3 a)
{
    double n2 = v_norm2(a);
    if (n2 == 0) return v3(0, 0, 0);
    return v_mul(a, 1 / sqrt(n2));
}
/* r3/vector.go LargestComponent: 0=X 1=Y 2=Z */
static inline int v_largest(V3 v)
{
    double ax = fabs(v.x), ay = fabs(v.y), az = fabs(v.z);
    if (ax > ay) return ax > az ? 0 : 2;
    return ay > az ? 1 : 2;
}
/* r3/vector.go Ortho */
static V3 v_ortho(V3 v)
{
    V3 ov = v3(0.012, 0.0053, 0.00457);
    switch (v_largest(v)) {
    case 0: ov.z = 1; break;
    case 1: ov.x = 1; break;
    default: ov.y = 1; break;
    }
    return v_normalize(v_cross(v, ov));
}
/* r3/vector.go Angle: atan2(|v x ov|, v . ov) */
static inline double v_angle(V3 a, V3 b) { return go_atan2(v_norm(v_cross(a, b)), v_dot(a, b)); }
/* r3/vector.go Cmp (lexicographic) */
static inline int v_cmp(V3 a, V3 b)
{
    if (a.x < b.x) return -1;
    if (a.x > b.x) return 1;
    if (a.y < b.y) return -1;
    if (a.y > b.y) return 1;
    if (a.z < b.z) return -1;
    if (a.z > b.z) return 1;
    return 0;
}
/* s2/point.go PointCross */
static V3 point_cross(V3 p, V3 op)
{
    V3 x = v_cross(v_add(p, op), v_sub(op, p));
    if (x.x == 0 && x.y == 0 && x.z == 0) return v_ortho(p);
    return x;
}

/* ------------------------------------------------- exact arithmetic
 * Shewchuk expansions (Dekker split; exact without FMA contraction).  Used to
 * obtain the exact sign that s2/predicates.go computes with big.Float.     */
#define SPLITTER 134217729.0
static inline void two_sum(double a, double b, double *x, double *y)
{
    *x = a + b;
    double bv = *x - a, av = *x - bv;
    *y = (a - av) + (b - bv);
}
static inline void split(double a, double *hi, double *lo)
{
    double c = SPLITTER * a, ab = c - a;
    *hi = c - ab;
    *lo = a - *hi;
}
static inline void two_prod(double a, double b, double *x, double *y)
{
    *x = a * b;
    double ahi, alo, bhi, blo;
    split(a, &ahi, &alo);
    split(b, &bhi, &blo);
    double err1 = *x - (ahi * bhi), err2 = err1 - (alo * bhi), err3 = err2 - (ahi * blo);
    *y = (alo * blo) - err3;
}
/* h = e + f as a nonoverlapping expansion of increasing magnitude (zero
 * eliminated): Shewchuk's Grow-Expansion applied to every input term in turn,
 * starting from the empty expansion, so the inputs need not be normalized. */
static int exp_sum(int elen, const double *e, int flen, const double *f, double *h)
{
    double tmp[64];
    int n = 0;
    for (int i = 0; i < elen + flen; i++) {
        double q = i < elen ? e[i] : f[i - elen];
        for (int k = 0; k < n; k++) {
            double s, err;
            two_sum(q, tmp[k], &s, &err);
            tmp[k] = err;
            q = s;
        }
        tmp[n++] = q;
    }
    int m = 0;
    for (int k = 0; k < n; k++)
        if (tmp[k] != 0) h[m++] = tmp[k];
    return m;
}
static int exp_scale(int elen, const double *e, double b, double *h)
{
    double terms[64];
    int n = 0;
    for (int i = 0; i < elen; i++) {
        double p, err;
        two_prod(e[i], b, &p, &err);
        terms[n++] = err;
        terms[n++] = p;
    }
    return exp_sum(n, terms, 0, terms, h);
}
static int exp_sign(int n, const double *e)
{
    /* After the grow-expansion every component is nonoverlapping and increasing
     * in magnitude, so the last nonzero component carries the sign. */
    for (int i = n - 1; i >= 0; i--) {
        if (e[i] > 0) return 1;
        if (e[i] < 0) return -1;
    }
    return 0;
}
/* exact a*b - c*d as an expansion (<=4 terms) */
static int exp_diff_prod(double a, double b, double c, double d, double *h)
{
    double t1[2], t2[2];
    two_prod(a, b, &t1[1], &t1[0]);
    two_prod(c, d, &t2[1], &t2[0]);
    t2[0] = -t2[0];
    t2[1] = -t2[1];
    return exp_sum(2, t1, 2, t2, h);
}

/* ----------------------------------------------------------- predicates
 * s2/predicates.go                                                     */
enum { CLOCKWISE = -1, INDETERMINATE = 0, COUNTERCLOCKWISE = 1 };

static int triage_sign(V3 a, V3 b, V3 c)
{
    double det = v_dot(v_cross(a, b), c);
    if (det > ORC_MAX_DET_ERR) return COUNTERCLOCKWISE;
    if (det < -ORC_MAX_DET_ERR) return CLOCKWISE;
    return INDETERMINATE;
}

static inline int fsgn(double x) { return (x > 0) - (x < 0); }

/* predicates.go symbolicallyPerturbedSign (inputs sorted lexicographically) */
static int symbolically_perturbed_sign(V3 a, V3 b, V3 c, const double bc[3][4], const int bcn[3])
{
    int s;
    double h[8];
    int n;
    if ((s = exp_sign(bcn[2], bc[2])) != 0) return s; /* da.z */
    if ((s = exp_sign(bcn[1], bc[1])) != 0) return s; /* da.y */
    if ((s = exp_sign(bcn[0], bc[0])) != 0) return s; /* da.x */
    n = exp_diff_prod(c.x, a.y, c.y, a.x, h);
    if ((s = exp_sign(n, h)) != 0) return s; /* db.z */
    if ((s = fsgn(c.x)) != 0) return s;  /* db.z * da.y */
    if ((s = -fsgn(c.y)) != 0) return s; /* db.z * da.x */
    n = exp_diff_prod(c.z, a.x, c.x, a.z, h);
    if ((s = exp_sign(n, h)) != 0) return s; /* db.y */
    if ((s = fsgn(c.z)) != 0) return s;  /* db.y * da.x */
    n = exp_diff_prod(a.x, b.y, a.y, b.x, h);
    if ((s = exp_sign(n, h)) != 0) return s; /* dc.z */
    if ((s = -fsgn(b.x)) != 0) return s; /* dc.z * da.y */
    if ((s = fsgn(b.y)) != 0) return s;  /* dc.z * da.x */
    if ((s = fsgn(a.x)) != 0) return s;  /* dc.z * db.y */
    return 1;                                          /* dc.z * db.y * da.x */
}

/* predicates.go exactSign */
static int exact_sign(V3 a, V3 b, V3 c, int perturb)
{
    int perm = 1;
    V3 pa = a, pb = b, pc = c, t;
    if (v_cmp(pa, pb) > 0) { t = pa; pa = pb; pb = t; perm = -perm; }
    if (v_cmp(pb, pc) > 0) { t = pb; pb = pc; pc = t; perm = -perm; }
    if (v_cmp(pa, pb) > 0) { t = pa; pa = pb; pb = t; perm = -perm; }
    /* b x c exactly */
    double bc[3][4];
    int bcn[3];
    bcn[0] = exp_diff_prod(pb.y, pc.z, pb.z, pc.y, bc[0]);
    bcn[1] = exp_diff_prod(pb.z, pc.x, pb.x, pc.z, bc[1]);
    bcn[2] = exp_diff_prod(pb.x, pc.y, pb.y, pc.x, bc[2]);
    double s0[16], s1[16], s2[16], t01[32], det[48];
    int n0 = exp_scale(bcn[0], bc[0], pa.x, s0);
    int n1 = exp_scale(bcn[1], bc[1], pa.y, s1);
    int n2 = exp_scale(bcn[2], bc[2], pa.z, s2);
    int n01 = exp_sum(n0, s0, n1, s1, t01);
    int nd = exp_sum(n01, t01, n2, s2, det);
    int ds = exp_sign(nd, det);
    if (ds == 0 && perturb) ds = symbolically_perturbed_sign(pa, pb, pc, (const double(*)[4])bc, bcn);
    return perm * ds;
}

/* predicates.go expensiveSign: equal points -> Indeterminate; otherwise the
 * exact sign (stableSign only short-cuts to the same exact answer). */
static int expensive_sign(V3 a, V3 b, V3 c)
{
    if (v_eq(a, b) || v_eq(b, c) || v_eq(c, a)) return INDETERMINATE;
    return exact_sign(a, b, c, 1);
}

/* predicates.go RobustSign */
static int robust_sign(V3 a, V3 b, V3 c)
{
    int s = triage_sign(a, b, c);
    if (s == INDETERMINATE) s = expensive_sign(a, b, c);
    return s;
}

/* predicates.go OrderedCCW */
static int ordered_ccw(V3 a, V3 b, V3 c, V3 o)
{
    int sum = 0;
    if (robust_sign(b, o, a) != CLOCKWISE) sum++;
    if (robust_sign(c, o, b) != CLOCKWISE) sum++;
    if (robust_sign(a, o, c) == COUNTERCLOCKWISE) sum++;
    return sum >= 2;
}

/* edge_crossings.go VertexCrossing */
static int vertex_crossing(V3 a, V3 b, V3 c, V3 d)
{
    if (v_eq(a, b) || v_eq(c, d)) return 0;
    if (v_eq(a, c)) return v_eq(b, d) || ordered_ccw(v_ortho(a), d, b, a);
    if (v_eq(b, d)) return ordered_ccw(v_ortho(b), c, a, b);
    if (v_eq(a, d)) return v_eq(b, c) || ordered_ccw(v_ortho(a), c, b, a);
    if (v_eq(b, c)) return ordered_ccw(v_ortho(b), d, a, b);
    return 0;
}

/* loop.go / edge_crossings.go AngleContainsVertex */
static int angle_contains_vertex(V3 a, V3 b, V3 c) { return !ordered_ccw(v_ortho(b), c, a, b); }

/* ------------------------------------------------------- EdgeCrosser
 * s2/edge_crosser.go                                                   */
enum { DO_NOT_CROSS = -1, MAYBE_CROSS = 0, CROSS = 1 };
typedef struct {
    V3 a, b, a_tangent, b_tangent, c;
    int acb;
} EdgeCrosser;

static void ec_init(EdgeCrosser *e, V3 a, V3 b)
{
    V3 norm = point_cross(a, b);
    e->a = a;
    e->b = b;
    e->a_tangent = v_cross(a, norm);
    e->b_tangent = v_cross(norm, b);
    e->acb = 0;
    e->c = v3(0, 0, 0);
}
static void ec_restart(EdgeCrosser *e, V3 c)
{
    e->c = c;
    e->acb = -triage_sign(e->a, e->b, c);
}
static int ec_crossing_sign_slow(EdgeCrosser *e, V3 d, int bda)
{
    int result;
    const double max_error = (1.5 + 1 / sqrt(3.0)) * ORC_DBL_EPS;
    if ((v_dot(e->c, e->a_tangent) > max_error && v_dot(d, e->a_tangent) > max_error) ||
        (v_dot(e->c, e->b_tangent) > max_error && v_dot(d, e->b_tangent) > max_error)) {
        result = DO_NOT_CROSS;
        goto done;
    }
    if (v_eq(e->a, e->c) || v_eq(e->a, d) || v_eq(e->b, e->c) || v_eq(e->b, d)) {
        result = MAYBE_CROSS;
        goto done;
    }
    if (v_eq(e->a, e->b) || v_eq(e->c, d)) {
        result = DO_NOT_CROSS;
        goto done;
    }
    if (e->acb == INDETERMINATE) e->acb = -expensive_sign(e->a, e->b, e->c);
    if (bda == INDETERMINATE) bda = expensive_sign(e->a, e->b, d);
    if (bda != e->acb) { result = DO_NOT_CROSS; goto done; }
    {
        int cbd = -robust_sign(e->c, d, e->b);
        if (cbd != e->acb) { result = DO_NOT_CROSS; goto done; }
        int dac = robust_sign(e->c, d, e->a);
        if (dac != e->acb) { result = DO_NOT_CROSS; goto done; }
    }
    result = CROSS;
done:
    /* the deferred assignments in crossingSign */
    e->c = d;
    e->acb = -bda;
    return result;
}
static int ec_chain_crossing_sign(EdgeCrosser *e, V3 d)
{
    int bda = triage_sign(e->a, e->b, d);
    if (e->acb == -bda && bda != INDETERMINATE) {
        e->c = d;
        e->acb = -bda;
        return DO_NOT_CROSS;
    }
    return ec_crossing_sign_slow(e, d, bda);
}
static int ec_edge_or_vertex_chain_crossing(EdgeCrosser *e, V3 d)
{
    V3 c = e->c;
    int s = ec_chain_crossing_sign(e, d);
    if (s == DO_NOT_CROSS) return 0;
    if (s == CROSS) return 1;
    return vertex_crossing(e->a, e->b, c, d);
}

/* ------------------------------------------------------ projections
 * s2/stuv.go                                                          */
#define MAX_LEVEL 30
#define MAX_SIZE (1 << MAX_LEVEL)

static inline double st_to_uv(double s)
{
    if (s >= 0.5) return ORC_ONE_THIRD * (4 * s * s - 1);
    return ORC_ONE_THIRD * (1 - 4 * (1 - s) * (1 - s));
}
static inline double uv_to_st(double u)
{
    if (u >= 0) return 0.5 * sqrt(1 + 3 * u);
    return 1 - 0.5 * sqrt(1 - 3 * u);
}
static inline int st_to_ij(double s)
{
    double f = floor(MAX_SIZE * s);
    /* Go: int(math.Floor(...)) then clamp */
    long long v = (long long)f;
    if (v < 0) v = 0;
    if (v > MAX_SIZE - 1) v = MAX_SIZE - 1;
    return (int)v;
}
static inline double ij_to_st_min(int i) { return (double)i / (double)MAX_SIZE; }
static inline int xyz_face(V3 r)
{
    int f = v_largest(r);
    if (f == 0 && r.x < 0) f += 3;
    else if (f == 1 && r.y < 0) f += 3;
    else if (f == 2 && r.z < 0) f += 3;
    return f;
}
static inline void valid_face_xyz_to_uv(int face, V3 r, double *u, double *v)
{
    switch (face) {
    case 0: *u = r.y / r.x; *v = r.z / r.x; break;
    case 1: *u = -r.x / r.y; *v = r.z / r.y; break;
    case 2: *u = -r.x / r.z; *v = -r.y / r.z; break;
    case 3: *u = r.z / r.x; *v = r.y / r.x; break;
    case 4: *u = r.z / r.y; *v = -r.x / r.y; break;
    default: *u = -r.y / r.z; *v = -r.x / r.z; break;
    }
}
static inline int face_xyz_to_uv(int face, V3 p, double *u, double *v)
{
    switch (face) {
    case 0: if (p.x <= 0) return 0; break;
    case 1: if (p.y <= 0) return 0; break;
    case 2: if (p.z <= 0) return 0; break;
    case 3: if (p.x >= 0) return 0; break;
    case 4: if (p.y >= 0) return 0; break;
    default: if (p.z >= 0) return 0; break;
    }
    valid_face_xyz_to_uv(face, p, u, v);
    return 1;
}
static inline V3 face_uv_to_xyz(int face, double u, double v)
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
/* edge_clipping.go faceXYZtoUVW */
static inline V3 face_xyz_to_uvw(int face, V3 p)
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

/* ----------------------------------------------------------- CellID
 * s2/cellid.go                                                         */
#define LOOKUP_BITS 4
#define SWAP_MASK 1
#define INVERT_MASK 2
static int lookup_pos[1 << (2 * LOOKUP_BITS + 2)];
static int lookup_ij[1 << (2 * LOOKUP_BITS + 2)];
static const int pos_to_ij[4][4] = {{0, 1, 3, 2}, {0, 2, 3, 1}, {3, 2, 0, 1}, {3, 1, 0, 2}};
static const int pos_to_orientation[4] = {SWAP_MASK, 0, 0, INVERT_MASK | SWAP_MASK};
static int lookup_ready = 0;

static void init_lookup_cell(int level, int i, int j, int orig, int pos, int orientation)
{
    if (level == LOOKUP_BITS) {
        int ij = (i << LOOKUP_BITS) + j;
        lookup_pos[(ij << 2) + orig] = (pos << 2) + orientation;
        lookup_ij[(pos << 2) + orig] = (ij << 2) + orientation;
        return;
    }
    level++;
    i <<= 1;
    j <<= 1;
    pos <<= 2;
    const int *r = pos_to_ij[orientation];
    for (int k = 0; k < 4; k++)
        init_lookup_cell(level, i + (r[k] >> 1), j + (r[k] & 1), orig, pos + k, orientation ^ pos_to_orientation[k]);
}
static void ensure_lookup(void)
{
    if (lookup_ready) return;
    init_lookup_cell(0, 0, 0, 0, 0, 0);
    init_lookup_cell(0, 0, 0, SWAP_MASK, 0, SWAP_MASK);
    init_lookup_cell(0, 0, 0, INVERT_MASK, 0, INVERT_MASK);
    init_lookup_cell(0, 0, 0, SWAP_MASK | INVERT_MASK, 0, SWAP_MASK | INVERT_MASK);
    lookup_ready = 1;
}

static uint64_t cellid_from_face_ij(int f, int i, int j)
{
    uint64_t n = (uint64_t)f << 60;
    int bits = f & SWAP_MASK;
    for (int k = 7; k >= 0; k--) {
        int mask = (1 << LOOKUP_BITS) - 1;
        bits += ((i >> (k * LOOKUP_BITS)) & mask) << (LOOKUP_BITS + 2);
        bits += ((j >> (k * LOOKUP_BITS)) & mask) << 2;
        bits = lookup_pos[bits];
        n |= (uint64_t)(bits >> 2) << (k * 2 * LOOKUP_BITS);
        bits &= (SWAP_MASK | INVERT_MASK);
    }
    return n * 2 + 1;
}
static inline int cellid_face(uint64_t id) { return (int)(id >> 61); }
static inline uint64_t cellid_lsb(uint64_t id) { return id & (~id + 1); }
static inline int cellid_level(uint64_t id) { return MAX_LEVEL - (__builtin_ctzll(id) >> 1); }
static inline uint64_t lsb_for_level(int level) { return (uint64_t)1 << (2 * (MAX_LEVEL - level)); }
static inline uint64_t cellid_parent(uint64_t id, int level)
{
    uint64_t lsb = lsb_for_level(level);
    return (id & (~lsb + 1)) | lsb;
}
static inline uint64_t cellid_child_begin(uint64_t id)
{
    uint64_t old = cellid_lsb(id);
    return id - old + (old >> 2);
}
static inline uint64_t cellid_next(uint64_t id) { return id + (cellid_lsb(id) << 1); }
static inline int cellid_is_leaf(uint64_t id) { return (id & 1) != 0; }

static void cellid_face_ij_orientation(uint64_t id, int *fo, int *io, int *jo, int *oo)
{
    int f = cellid_face(id), i = 0, j = 0;
    int orientation = f & SWAP_MASK;
    int nbits = MAX_LEVEL - 7 * LOOKUP_BITS;
    for (int k = 7; k >= 0; k--) {
        orientation += ((int)(id >> (k * 2 * LOOKUP_BITS + 1)) & ((1 << (2 * nbits)) - 1)) << 2;
        orientation = lookup_ij[orientation];
        i += (orientation >> (LOOKUP_BITS + 2)) << (k * LOOKUP_BITS);
        j += ((orientation >> 2) & ((1 << LOOKUP_BITS) - 1)) << (k * LOOKUP_BITS);
        orientation &= (SWAP_MASK | INVERT_MASK);
        nbits = LOOKUP_BITS;
    }
    if (cellid_lsb(id) & 0x1111111111111110ULL) orientation ^= SWAP_MASK;
    *fo = f;
    *io = i;
    *jo = j;
    *oo = orientation;
}

/* cellid.go CellIDFromPoint (used by tests / cap bound) */
static uint64_t cellid_from_point(V3 p)
{
    int f = xyz_face(p);
    double u, v;
    valid_face_xyz_to_uv(f, p, &u, &v);
    return cellid_from_face_ij(f, st_to_ij(uv_to_st(u)), st_to_ij(uv_to_st(v)));
}

/* -------------------------------------------------------------- Cell
 * s2/cell.go                                                           */
typedef struct {
    uint64_t id;
    int face, level;
    double ulo, uhi, vlo, vhi;
} Cell;

static Cell cell_from_id(uint64_t id)
{
    Cell c;
    int f, i, j, o;
    cellid_face_ij_orientation(id, &f, &i, &j, &o);
    c.id = id;
    c.face = f;
    c.level = cellid_level(id);
    int size = 1 << (MAX_LEVEL - c.level); /* sizeIJ */
    int xlo = i & -size, ylo = j & -size;
    c.ulo = st_to_uv(ij_to_st_min(xlo));
    c.uhi = st_to_uv(ij_to_st_min(xlo + size));
    c.vlo = st_to_uv(ij_to_st_min(ylo));
    c.vhi = st_to_uv(ij_to_st_min(ylo + size));
    return c;
}
/* cellid.go faceSiTi + rawPoint; cell.go Center */
static V3 cell_center(const Cell *c)
{
    int f, i, j, o;
    cellid_face_ij_orientation(c->id, &f, &i, &j, &o);
    int delta = 0;
    if (cellid_is_leaf(c->id)) delta = 1;
    else if ((i ^ ((int)(c->id >> 2))) & 1) delta = 2;
    uint32_t si = (uint32_t)(2 * i + delta), ti = (uint32_t)(2 * j + delta);
    const double half = 0.5 / MAX_SIZE;
    V3 raw = face_uv_to_xyz(f, st_to_uv(half * (double)si), st_to_uv(half * (double)ti));
    return v_normalize(raw);
}
/* cell.go Vertex(k): r2.Rect.Vertices order LL, LR, UR, UL */
static V3 cell_vertex(const Cell *c, int k)
{
    double u = (k == 0 || k == 3) ? c->ulo : c->uhi;
    double v = (k < 2) ? c->vlo : c->vhi;
    return v_normalize(face_uv_to_xyz(c->face, u, v));
}
/* cell.go ContainsPoint (uv bound expanded by dblEpsilon) */
static int cell_contains_point(const Cell *c, V3 p)
{
    double u, v;
    if (!face_xyz_to_uv(c->face, p, &u, &v)) return 0;
    double m = ORC_DBL_EPS;
    return (c->ulo - m) <= u && u <= (c->uhi + m) && (c->vlo - m) <= v && v <= (c->vhi + m);
}

/* ------------------------------------------------------ edge clipping
 * s2/edge_clipping.go                                                  */
static int uvw_intersects_face(V3 n)
{
    double u = fabs(n.x), v = fabs(n.y), w = fabs(n.z);
    return (v >= w - u) && (u >= w - v);
}
static int uvw_intersects_opposite_edges(V3 n)
{
    double u = fabs(n.x), v = fabs(n.y), w = fabs(n.z);
    if (fabs(u - v) != w) return fabs(u - v) >= w;
    if (u >= v) return u - w >= v;
    return v - w >= u;
}
static int uvw_exit_axis(V3 n) /* 0 = axisU, 1 = axisV */
{
    if (uvw_intersects_opposite_edges(n)) return fabs(n.x) >= fabs(n.y) ? 1 : 0;
    int x = signbit(n.x) ? 1 : 0, y = signbit(n.y) ? 1 : 0, z = signbit(n.z) ? 1 : 0;
    return ((x ^ y ^ z) == 0) ? 1 : 0;
}
static void uvw_exit_point(V3 n, int axis, double *pu, double *pv)
{
    if (axis == 0) {
        double u = -1.0;
        if (n.y > 0) u = 1.0;
        *pu = u;
        *pv = (-u * n.x - n.z) / n.y;
    } else {
        double v = -1.0;
        if (n.x < 0) v = 1.0;
        *pu = (-v * n.y - n.z) / n.x;
        *pv = v;
    }
}
static int clip_destination(V3 a, V3 b, V3 scaled_n, V3 a_tan, V3 b_tan, double scale_uv, double *ou, double *ov)
{
    const double max_safe = ORC_MAX_SAFE_UV_COORD;
    double u, v;
    if (b.z > 0) {
        u = b.x / b.z;
        v = b.y / b.z;
        if (go_max(fabs(u), fabs(v)) <= max_safe) {
            *ou = u;
            *ov = v;
            return 0;
        }
    }
    uvw_exit_point(scaled_n, uvw_exit_axis(scaled_n), &u, &v);
    u = scale_uv * u;
    v = scale_uv * v;
    V3 p = v3(u, v, 1.0);
    int score = 0;
    if (v_dot(v_sub(p, a), a_tan) < 0) score = 2;
    else if (v_dot(v_sub(p, b), b_tan) < 0) score = 1;
    if (score > 0) {
        if (b.z <= 0) score = 3;
        else { u = b.x / b.z; v = b.y / b.z; }
    }
    *ou = u;
    *ov = v;
    return score;
}
/* edge_clipping.go ClipToPaddedFace */
static int clip_to_padded_face(V3 a, V3 b, int f, double padding, double uv[4])
{
    if (xyz_face(a) == f && xyz_face(b) == f) {
        valid_face_xyz_to_uv(f, a, &uv[0], &uv[1]);
        valid_face_xyz_to_uv(f, b, &uv[2], &uv[3]);
        return 1;
    }
    V3 norm_uvw = face_xyz_to_uvw(f, point_cross(a, b));
    V3 a_uvw = face_xyz_to_uvw(f, a);
    V3 b_uvw = face_xyz_to_uvw(f, b);
    double scale_uv = 1 + padding;
    V3 scaled_n = v3(scale_uv * norm_uvw.x, scale_uv * norm_uvw.y, norm_uvw.z);
    if (!uvw_intersects_face(scaled_n)) return 0;
    norm_uvw = v_normalize(norm_uvw);
    V3 a_tan = v_cross(norm_uvw, a_uvw);
    V3 b_tan = v_cross(b_uvw, norm_uvw);
    int a_score = clip_destination(b_uvw, a_uvw, v_mul(scaled_n, -1), b_tan, a_tan, scale_uv, &uv[0], &uv[1]);
    int b_score = clip_destination(a_uvw, b_uvw, scaled_n, a_tan, b_tan, scale_uv, &uv[2], &uv[3]);
    return a_score + b_score < 3;
}
/* edge_clipping.go edgeIntersectsRect (r = [ulo,uhi]x[vlo,vhi]) */
static int edge_intersects_rect(double au, double av, double bu, double bv, double ulo, double uhi, double vlo, double vhi)
{
    /* r1.Interval.Intersects of rect and RectFromPoints(a,b) */
    double blo_u = au, bhi_u = au, blo_v = av, bhi_v = av;
    if (bu < blo_u) blo_u = bu;
    if (bu > bhi_u) bhi_u = bu;
    if (bv < blo_v) blo_v = bv;
    if (bv > bhi_v) bhi_v = bv;
    int xi = (ulo <= blo_u) ? (blo_u <= uhi && blo_u <= bhi_u) : (ulo <= bhi_u && ulo <= uhi);
    int yi = (vlo <= blo_v) ? (blo_v <= vhi && blo_v <= bhi_v) : (vlo <= bhi_v && vlo <= vhi);
    if (!(xi && yi)) return 0;
    double nx = -(bv - av), ny = bu - au; /* (b-a).Ortho() */
    int i = nx >= 0 ? 1 : 0, j = ny >= 0 ? 1 : 0;
    double vx = i ? uhi : ulo, vy = j ? vhi : vlo;
    double mx = nx * (vx - au) + ny * (vy - av);
    vx = i ? ulo : uhi;
    vy = j ? vlo : vhi;
    double mn = nx * (vx - au) + ny * (vy - av);
    return (mx >= 0) && (mn <= 0);
}

/* ------------------------------------------------------ intervals
 * s1/interval.go, r1/interval.go, s2/rect.go (only what RectBounder needs) */
typedef struct { double lo, hi; } Ival;
static inline Ival s1_empty(void) { Ival i = {ORC_PI, -ORC_PI}; return i; }
static inline Ival s1_full(void) { Ival i = {-ORC_PI, ORC_PI}; return i; }
static inline int s1_is_full(Ival i) { return i.lo == -ORC_PI && i.hi == ORC_PI; }
static inline int s1_is_empty(Ival i) { return i.lo == ORC_PI && i.hi == -ORC_PI; }
static inline int s1_is_inverted(Ival i) { return i.lo > i.hi; }
static double s1_length(Ival i)
{
    double l = i.hi - i.lo;
    if (l >= 0) return l;
    l += 2 * ORC_PI;
    if (l > 0) return l;
    return -1;
}
static int s1_fast_contains(Ival i, double p)
{
    if (s1_is_inverted(i)) return (p >= i.lo || p <= i.hi) && !s1_is_empty(i);
    return p >= i.lo && p <= i.hi;
}
static double positive_distance(double a, double b)
{
    double d = b - a;
    if (d >= 0) return d;
    return (b + ORC_PI) - (a - ORC_PI);
}
static Ival s1_add_point(Ival i, double p)
{
    if (fabs(p) > ORC_PI) return i;
    if (p == -ORC_PI) p = ORC_PI;
    if (s1_fast_contains(i, p)) return i;
    if (s1_is_empty(i)) { Ival r = {p, p}; return r; }
    if (positive_distance(p, i.lo) < positive_distance(i.hi, p)) { Ival r = {p, i.hi}; return r; }
    Ival r = {i.lo, p};
    return r;
}
static int s1_contains_interval(Ival i, Ival oi)
{
    if (s1_is_inverted(i)) {
        if (s1_is_inverted(oi)) return oi.lo >= i.lo && oi.hi <= i.hi;
        return (oi.lo >= i.lo || oi.hi <= i.hi) && !s1_is_empty(i);
    }
    if (s1_is_inverted(oi)) return s1_is_full(i) || s1_is_empty(oi);
    return oi.lo >= i.lo && oi.hi <= i.hi;
}
static Ival s1_union(Ival i, Ival oi)
{
    if (s1_is_empty(oi)) return i;
    if (s1_fast_contains(i, oi.lo)) {
        if (s1_fast_contains(i, oi.hi)) {
            if (s1_contains_interval(i, oi)) return i;
            return s1_full();
        }
        Ival r = {i.lo, oi.hi};
        return r;
    }
    if (s1_fast_contains(i, oi.hi)) { Ival r = {oi.lo, i.hi}; return r; }
    if (s1_is_empty(i) || s1_fast_contains(oi, i.lo)) return oi;
    if (positive_distance(oi.hi, i.lo) < positive_distance(i.hi, oi.lo)) { Ival r = {oi.lo, i.hi}; return r; }
    Ival r = {i.lo, oi.hi};
    return r;
}
static Ival s1_expanded(Ival i, double margin) /* margin >= 0 */
{
    if (s1_is_empty(i)) return i;
    if (s1_length(i) + 2 * margin + 2 * ORC_DBL_EPS >= 2 * ORC_PI) return s1_full();
    Ival r = {remainder(i.lo - margin, 2 * ORC_PI), remainder(i.hi + margin, 2 * ORC_PI)};
    if (r.lo <= -ORC_PI) r.lo = ORC_PI;
    return r;
}
static inline int r1_is_empty(Ival i) { return i.lo > i.hi; }
static inline Ival r1_empty(void) { Ival i = {1, 0}; return i; }
static Ival r1_add_point(Ival i, double p)
{
    if (r1_is_empty(i)) { Ival r = {p, p}; return r; }
    if (p < i.lo) { Ival r = {p, i.hi}; return r; }
    if (p > i.hi) { Ival r = {i.lo, p}; return r; }
    return i;
}
static Ival r1_union(Ival i, Ival o)
{
    if (r1_is_empty(i)) return o;
    if (r1_is_empty(o)) return i;
    Ival r = {go_min(i.lo, o.lo), go_max(i.hi, o.hi)};
    return r;
}
typedef struct { Ival lat, lng; } Rect;
static Rect rect_empty(void) { Rect r = {r1_empty(), s1_empty()}; return r; }
static Rect rect_add_latlng(Rect r, double lat, double lng)
{
    /* LatLng.IsValid: |lat| <= pi/2 && |lng| <= pi */
    if (!(fabs(lat) <= ORC_PI_2 && fabs(lng) <= ORC_PI)) return r;
    r.lat = r1_add_point(r.lat, lat);
    r.lng = s1_add_point(r.lng, lng);
    return r;
}
static Rect rect_union(Rect a, Rect b)
{
    Rect r = {r1_union(a.lat, b.lat), s1_union(a.lng, b.lng)};
    return r;
}

/* latlng.go LatLngFromPoint */
static inline double point_lat(V3 p) { return go_atan2(p.z, sqrt(p.x * p.x + p.y * p.y)); }
static inline double point_lng(V3 p) { return go_atan2(p.y, p.x); }

/* rect_bounder.go */
typedef struct {
    V3 a;
    double alat, alng;
    Rect bound;
} RectBounder;

static void rb_add_point(RectBounder *r, V3 b)
{
    double blat = point_lat(b), blng = point_lng(b);
    if (r1_is_empty(r->bound.lat)) {
        r->a = b;
        r->alat = blat;
        r->alng = blng;
        r->bound = rect_add_latlng(r->bound, blat, blng);
        return;
    }
    V3 n = v_cross(v_sub(r->a, b), v_add(r->a, b));
    double n_norm = v_norm(n);
    if (n_norm < 1.91346e-15) {
        if (v_dot(r->a, b) < 0) {
            Rect full = {{-ORC_PI_2, ORC_PI_2}, s1_full()};
            r->bound = full;
        } else {
            Rect pr = {{r->alat, r->alat}, {r->alng, r->alng}};
            pr = rect_add_latlng(pr, blat, blng);
            r->bound = rect_union(r->bound, pr);
        }
        r->a = b;
        r->alat = blat;
        r->alng = blng;
        return;
    }
    Ival lng_ab = s1_add_point(s1_add_point(s1_empty(), r->alng), blng);
    if (s1_length(lng_ab) >= ORC_PI_MINUS_2EPS) lng_ab = s1_full();
    Ival lat_ab = r1_add_point((Ival){r->alat, r->alat}, blat);
    V3 m = v_cross(n, v3(0, 0, 1));
    double ma = v_dot(m, r->a), mb = v_dot(m, b);
    double m_error = 6.06638e-16 * n_norm + 6.83174e-31;
    if (ma * mb < 0 || fabs(ma) <= m_error || fabs(mb) <= m_error) {
        double max_lat = go_min(go_atan2(sqrt(n.x * n.x + n.y * n.y), fabs(n.z)) + ORC_THREE_EPS, ORC_PI_2);
        double lat_budget = 2 * go_asin(0.5 * v_norm(v_sub(r->a, b)) * go_sin(max_lat));
        double max_delta = 0.5 * (lat_budget - (lat_ab.hi - lat_ab.lo)) + ORC_DBL_EPS;
        if (ma <= m_error && mb >= -m_error) lat_ab.hi = go_min(max_lat, lat_ab.hi + max_delta);
        if (mb <= m_error && ma >= -m_error) lat_ab.lo = go_max(-max_lat, lat_ab.lo - max_delta);
    }
    r->a = b;
    r->alat = blat;
    r->alng = blng;
    Rect e = {lat_ab, lng_ab};
    r->bound = rect_union(r->bound, e);
}
/* RectBound: expanded by (2*dblEpsilon, 0) then PolarClosure */
static Rect rb_rect_bound(const RectBounder *r)
{
    Rect b = r->bound;
    Ival lat = b.lat;
    if (!r1_is_empty(lat)) { lat.lo = lat.lo - ORC_TWO_EPS; lat.hi = lat.hi + ORC_TWO_EPS; }
    Ival lng = s1_expanded(b.lng, 0);
    if (r1_is_empty(lat) || s1_is_empty(lng)) return rect_empty();
    /* Intersection with validRectLatRange [-pi/2, pi/2] */
    lat.lo = go_max(lat.lo, -ORC_PI_2);
    lat.hi = go_min(lat.hi, ORC_PI_2);
    Rect out = {lat, lng};
    if (out.lat.lo == -ORC_PI_2 || out.lat.hi == ORC_PI_2) out.lng = s1_full();
    return out;
}

/* -------------------------------------------------------------- Loop
 * s2/loop.go                                                           */
typedef struct {
    const V3 *v;
    int n;
    int origin_inside;
    Rect bound;
} Loop;

static inline V3 loop_vertex(const Loop *l, int i) { return l->v[i % l->n]; }

static V3 origin_point(void) { return v3(-0.0099994664350250197, 0.0025924542609324121, 0.99994664350250195); }

static int loop_brute_contains(const Loop *l, V3 p)
{
    if (l->n < 3) return l->origin_inside;
    EdgeCrosser e;
    ec_init(&e, origin_point(), p);
    ec_restart(&e, loop_vertex(l, 0));
    int inside = l->origin_inside;
    for (int i = 1; i <= l->n; i++) inside = inside != ec_edge_or_vertex_chain_crossing(&e, loop_vertex(l, i));
    return inside;
}
static void loop_init(Loop *l, const V3 *v, int n)
{
    l->v = v;
    l->n = n;
    /* initOriginAndBound (n >= 3 on every DSS path) */
    int v1_inside = !v_eq(v[0], v[1]) && !v_eq(v[2], v[1]) && angle_contains_vertex(v[0], v[1], v[2]);
    l->origin_inside = 0;
    if (v1_inside != loop_brute_contains(l, v[1])) l->origin_inside = 1;
    /* initBound */
    RectBounder rb;
    rb.bound = rect_empty();
    rb.alat = rb.alng = 0;
    rb.a = v3(0, 0, 0);
    for (int i = 0; i <= n; i++) rb_add_point(&rb, loop_vertex(l, i));
    Rect b = rb_rect_bound(&rb);
    if (loop_brute_contains(l, v3(0, 0, 1))) {
        b.lat.hi = ORC_PI_2;
        b.lng = s1_full();
    }
    if (s1_is_full(b.lng) && loop_brute_contains(l, v3(0, 0, -1))) b.lat.lo = -ORC_PI_2;
    l->bound = b;
}

/* point_measures.go GirardArea / PointArea, SignedArea */
static double girard_area(V3 a, V3 b, V3 c)
{
    V3 ab = point_cross(a, b), bc = point_cross(b, c), ac = point_cross(a, c);
    double area = v_angle(ab, ac) - v_angle(ab, bc) + v_angle(bc, ac);
    if (area < 0) area = 0;
    return area;
}
static double point_area(V3 a, V3 b, V3 c)
{
    double sa = v_angle(b, c), sb = v_angle(c, a), sc = v_angle(a, b);
    double s = 0.5 * (sa + sb + sc);
    if (s >= 3e-4) {
        double dmin = s - go_max(sa, go_max(sb, sc));
        if (dmin < 1e-2 * s * s * s * s * s) {
            double area = girard_area(a, b, c);
            if (dmin < s * 0.1 * area) return area;
        }
    }
    return 4 * go_atan(sqrt(go_max(0.0, go_tan(0.5 * s) * go_tan(0.5 * (s - sa)) * go_tan(0.5 * (s - sb)) * go_tan(0.5 * (s - sc)))));
}
static double signed_area(V3 a, V3 b, V3 c) { return (double)robust_sign(a, b, c) * point_area(a, b, c); }

static double loop_surface_integral_signed_area(const Loop *l)
{
    const double max_length = ORC_SURFACE_MAX_LENGTH;
    double sum = 0;
    V3 origin = loop_vertex(l, 0);
    for (int i = 1; i + 1 < l->n; i++) {
        if (v_angle(loop_vertex(l, i + 1), origin) > max_length) {
            V3 old_origin = origin;
            if (v_eq(origin, loop_vertex(l, 0))) {
                origin = v_normalize(point_cross(loop_vertex(l, 0), loop_vertex(l, i)));
            } else if (v_angle(loop_vertex(l, i), loop_vertex(l, 0)) < max_length) {
                origin = loop_vertex(l, 0);
            } else {
                origin = v_cross(loop_vertex(l, 0), old_origin);
                sum += signed_area(loop_vertex(l, 0), old_origin, origin);
            }
            sum += signed_area(old_origin, loop_vertex(l, i), origin);
        }
        sum += signed_area(origin, loop_vertex(l, i), loop_vertex(l, i + 1));
    }
    if (!v_eq(origin, loop_vertex(l, 0))) sum += signed_area(origin, loop_vertex(l, l->n - 1), loop_vertex(l, 0));
    return sum;
}
static double turn_angle(V3 a, V3 b, V3 c)
{
    double angle = v_angle(point_cross(a, b), point_cross(b, c));
    if (robust_sign(a, b, c) == COUNTERCLOCKWISE) return angle;
    return -angle;
}
static double loop_turning_angle(const Loop *l)
{
    int n = l->n;
    if (n < 3) return 0;
    /* canonicalFirstVertex */
    int first = 0, dir;
    for (int i = 1; i < n; i++)
        if (v_cmp(loop_vertex(l, i), loop_vertex(l, first)) == -1) first = i;
    if (v_cmp(loop_vertex(l, first + 1), loop_vertex(l, first + n - 1)) == -1) dir = 1;
    else { first += n; dir = -1; }
    int i = first;
    double sum = turn_angle(loop_vertex(l, (i + n - dir) % n), loop_vertex(l, i), loop_vertex(l, (i + dir) % n));
    double comp = 0;
    int cnt = n;
    while (cnt - 1 > 0) {
        i += dir;
        double angle = turn_angle(loop_vertex(l, i - dir), loop_vertex(l, i), loop_vertex(l, i + dir));
        double old_sum = sum;
        angle += comp;
        sum += angle;
        comp = (old_sum - sum) + angle;
        cnt--;
    }
    return (double)dir * (sum + comp);
}
static double loop_turning_angle_max_error(const Loop *l) { return ORC_TURN_ANGLE_ERR_PER_VERTEX * (double)l->n; }
static int loop_is_normalized(const Loop *l)
{
    if (s1_length(l->bound.lng) < ORC_PI) return 1;
    return loop_turning_angle(l) >= -loop_turning_angle_max_error(l);
}
static double loop_area(const Loop *l)
{
    double area = loop_surface_integral_signed_area(l);
    double max_error = loop_turning_angle_max_error(l);
    if (area < 0) area += 4 * ORC_PI;
    if (area > 4 * ORC_PI) area = 4 * ORC_PI;
    if (area < 0) area = 0;
    if (area < max_error && !loop_is_normalized(l)) return 4 * ORC_PI;
    else if (area > (4 * ORC_PI - max_error) && loop_is_normalized(l)) return 0;
    return area;
}

/* Loop.IntersectsCell, restated without the ShapeIndex shortcuts (see header). */
typedef struct {
    const Loop *l;
    /* per-face clipped edges cache: 6 faces x n edges x (ok, u0, v0, u1, v1) */
    double *clip;
    signed char *clip_ok;
    unsigned char face_done[6];
} LoopRegion;

static void loop_region_face(LoopRegion *r, int face)
{
    if (r->face_done[face]) return;
    const Loop *l = r->l;
    for (int i = 0; i < l->n; i++) {
        double *uv = r->clip + ((size_t)face * l->n + i) * 4;
        r->clip_ok[(size_t)face * l->n + i] =
            (signed char)clip_to_padded_face(loop_vertex(l, i), loop_vertex(l, i + 1), face, ORC_FACE_CLIP_PLUS_RECT_ERR, uv);
    }
    r->face_done[face] = 1;
}
static int loop_intersects_cell(LoopRegion *r, const Cell *c)
{
    const Loop *l = r->l;
    loop_region_face(r, c->face);
    const double m = ORC_FACE_CLIP_PLUS_RECT_ERR;
    double ulo = c->ulo - m, uhi = c->uhi + m, vlo = c->vlo - m, vhi = c->vhi + m;
    for (int i = 0; i < l->n; i++) {
        size_t k = (size_t)c->face * l->n + i;
        if (!r->clip_ok[k]) continue;
        const double *uv = r->clip + k * 4;
        if (edge_intersects_rect(uv[0], uv[1], uv[2], uv[3], ulo, uhi, vlo, vhi)) return 1;
    }
    return loop_brute_contains(l, cell_center(c));
}

/* polyline.go IntersectsCell */
static int polyline_intersects_cell(const V3 *p, int n, const Cell *c)
{
    if (n == 0) return 0;
    for (int i = 0; i < n; i++)
        if (cell_contains_point(c, p[i])) return 1;
    V3 cv[4];
    for (int k = 0; k < 4; k++) cv[k] = cell_vertex(c, k);
    for (int j = 0; j < 4; j++) {
        EdgeCrosser e;
        ec_init(&e, cv[j], cv[(j + 1) & 3]);
        ec_restart(&e, p[0]);
        for (int i = 1; i < n; i++)
            if (ec_chain_crossing_sign(&e, p[i]) != DO_NOT_CROSS) return 1;
    }
    return 0;
}

/* ---------------------------------------------------------- coverer
 * s2/regioncoverer.go with MinLevel = MaxLevel = 13, LevelMod = 1,
 * MaxCells = 0 (pkg/geo/s2.go:30-35).  Level < 13 candidates always expand,
 * level-13 candidates are terminal (ContainsCell is never consulted), so the
 * result is the sorted set of level-13 cells reached by descending through
 * cells for which IntersectsCell holds.  Descent starts at the six face
 * cells; the initial candidates only bound the search.                 */
typedef struct {
    uint64_t *v;
    size_t n, cap;
} U64Vec;
static int u64_push(U64Vec *a, uint64_t x)
{
    if (a->n == a->cap) {
        size_t nc = a->cap ? a->cap * 2 : 64;
        uint64_t *nv = (uint64_t *)realloc(a->v, nc * sizeof(uint64_t));
        if (!nv) return -1;
        a->v = nv;
        a->cap = nc;
    }
    a->v[a->n++] = x;
    return 0;
}
static int cmp_u64(const void *a, const void *b)
{
    uint64_t x = *(const uint64_t *)a, y = *(const uint64_t *)b;
    return x < y ? -1 : x > y;
}

typedef int (*IntersectsFn)(void *ctx, const Cell *c);

static int cover_descend(void *ctx, IntersectsFn fn, uint64_t id, int level, U64Vec *out)
{
    Cell c = cell_from_id(id);
    if (!fn(ctx, &c)) return 0;
    if (level == ORC_COVER_LEVEL) {
        /* safety valve for invalid (self-intersecting) loops whose parity
         * interior is most of the sphere: the reference would try to emit
         * ~4e8 cells; the oracle reports it instead. */
        if (out->n >= ORC_MAX_CELLS) return -1;
        return u64_push(out, id);
    }
    uint64_t ch = cellid_child_begin(id);
    for (int k = 0; k < 4; k++, ch = cellid_next(ch))
        if (cover_descend(ctx, fn, ch, level + 1, out)) return -1;
    return 0;
}
static int cover_region(void *ctx, IntersectsFn fn, U64Vec *out)
{
    for (int f = 0; f < 6; f++) {
        uint64_t id = ((uint64_t)f << 61) | ((uint64_t)1 << 60);
        if (cover_descend(ctx, fn, id, 0, out)) return -1;
    }
    qsort(out->v, out->n, sizeof(uint64_t), cmp_u64);
    size_t m = 0;
    for (size_t i = 0; i < out->n; i++)
        if (m == 0 || out->v[m - 1] != out->v[i]) out->v[m++] = out->v[i];
    out->n = m;
    return 0;
}
static int loop_fn(void *ctx, const Cell *c) { return loop_intersects_cell((LoopRegion *)ctx, c); }
typedef struct { const V3 *p; int n; } PolyRegion;
static int poly_fn(void *ctx, const Cell *c)
{
    PolyRegion *pr = (PolyRegion *)ctx;
    return polyline_intersects_cell(pr->p, pr->n, c);
}

static int cover_loop(const Loop *l, U64Vec *out)
{
    LoopRegion r;
    memset(&r, 0, sizeof(r));
    r.l = l;
    r.clip = (double *)malloc(sizeof(double) * 4 * 6 * (size_t)l->n);
    r.clip_ok = (signed char *)malloc(6 * (size_t)l->n);
    if (!r.clip || !r.clip_ok) { free(r.clip); free(r.clip_ok); return -1; }
    int rc = cover_region(&r, loop_fn, out);
    free(r.clip);
    free(r.clip_ok);
    return rc;
}

/* ------------------------------------------------------- public API */

/* s2.PointFromLatLng(s2.LatLngFromDegrees(lat, lng)) (latlng.go, s1/angle.go) */
static V3 point_from_degrees(double lat_deg, double lng_deg)
{
    double phi = lat_deg * ORC_DEGREE, theta = lng_deg * ORC_DEGREE;
    double cosphi = go_cos(phi);
    return v3(go_cos(theta) * cosphi, go_sin(theta) * cosphi, go_sin(phi));
}

void orc_point_from_degrees(double lat, double lng, double out[3])
{
    V3 p = point_from_degrees(lat, lng);
    out[0] = p.x;
    out[1] = p.y;
    out[2] = p.z;
}

uint64_t orc_cellid_from_degrees(double lat, double lng, int level)
{
    ensure_lookup();
    uint64_t id = cellid_from_point(point_from_degrees(lat, lng));
    return cellid_parent(id, level);
}

static int emit(const U64Vec *cells, uint64_t *out, size_t cap, size_t *needed)
{
    *needed = cells->n;
    if (out && cells->n <= cap) memcpy(out, cells->v, cells->n * sizeof(uint64_t));
    return 0;
}

/* pkg/geo/s2.go:89-95 loopAreaKm2 (Q1: multiplies by pi instead of dividing) */
static double loop_area_km2(const Loop *l) { return (loop_area(l) * ORC_EARTH_AREA_KM2) / 4.0 * ORC_PI; }

double orc_loop_area(const double *xyz, int n)
{
    ensure_lookup();
    Loop l;
    loop_init(&l, (const V3 *)xyz, n);
    return loop_area(&l);
}

/* pkg/geo/s2.go:99-122 Covering, on points already converted to S2 (xyz).
 * `xyz` is reversed in place when the area test triggers (Q4). */
int orc_covering_xyz(double *xyz, int n, uint64_t *out, size_t cap, size_t *needed, double *area_km2)
{
    ensure_lookup();
    V3 *pts = (V3 *)xyz;
    Loop l;
    loop_init(&l, pts, n);
    double area = loop_area_km2(&l);
    if (area > ORC_MAX_AREA_KM2) {
        for (int i = 0, j = n - 1; i < j; i++, j--) {
            V3 t = pts[i];
            pts[i] = pts[j];
            pts[j] = t;
        }
        loop_init(&l, pts, n);
    }
    area = loop_area_km2(&l);
    if (area_km2) *area_km2 = area;
    *needed = 0;
    if (area > ORC_MAX_AREA_KM2) return ORC_ERR_AREA_TOO_LARGE;
    U64Vec cells = {0, 0, 0};
    int rc;
    if (area <= 0) {
        PolyRegion pr = {pts, n};
        rc = cover_region(&pr, poly_fn, &cells);
    } else {
        rc = cover_loop(&l, &cells);
    }
    if (rc) { free(cells.v); return ORC_ERR_NOMEM; }
    emit(&cells, out, cap, needed);
    free(cells.v);
    return ORC_OK;
}

/* pkg/models/geo.go:252-268 GeoPolygon.CalculateCovering */
int orc_polygon_covering(const double *lat, const double *lng, int n, uint64_t *out, size_t cap, size_t *needed,
                         double *area_km2)
{
    *needed = 0;
    if (area_km2) *area_km2 = 0;
    for (int i = 0; i < n; i++) /* Q17: coordinates are checked before the count */
        if (lat[i] > 90.0 || lat[i] < -90.0 || lng[i] > 180.0 || lng[i] < -180.0) return ORC_ERR_BAD_COORD_SET;
    if (n < 3) return ORC_ERR_NOT_ENOUGH_POINTS;
    double *xyz = (double *)malloc(sizeof(double) * 3 * (size_t)n);
    if (!xyz) return ORC_ERR_NOMEM;
    for (int i = 0; i < n; i++) orc_point_from_degrees(lat[i], lng[i], xyz + 3 * i);
    int rc = orc_covering_xyz(xyz, n, out, cap, needed, area_km2);
    free(xyz);
    return rc;
}

/* regular_loop.go getFrame / regularPointsForFrame */
static void regular_loop_points(V3 center, double radius, int num, V3 *out)
{
    /* frame columns: col2 = z = center, col1 = Ortho(center), col0 = col1 x center */
    V3 c2 = center, c1 = v_ortho(center), c0 = v_cross(c1, center);
    double m[3][3] = {{c0.x, c1.x, c2.x}, {c0.y, c1.y, c2.y}, {c0.z, c1.z, c2.z}};
    double z = go_cos(radius), r = go_sin(radius);
    double radian_step = 2 * ORC_PI / (double)num;
    for (int i = 0; i < num; i++) {
        double angle = (double)i * radian_step;
        V3 p = v3(r * go_cos(angle), r * go_sin(angle), z);
        V3 q = v3(m[0][0] * p.x + m[0][1] * p.y + m[0][2] * p.z, m[1][0] * p.x + m[1][1] * p.y + m[1][2] * p.z,
                  m[2][0] * p.x + m[2][1] * p.y + m[2][2] * p.z);
        out[i] = v_normalize(q);
    }
}

void orc_regular_loop(double lat, double lng, float radius_m, int num, double *xyz_out)
{
    V3 c = point_from_degrees(lat, lng);
    double angle = (double)radius_m / ORC_RADIUS_EARTH_M; /* geo.DistanceMetersToAngle */
    regular_loop_points(c, angle, num, (V3 *)xyz_out);
}

/* pkg/models/geo.go:224-239 GeoCircle.CalculateCovering (Q2: inscribed 20-gon, no area cap) */
int orc_circle_covering(double lat, double lng, float radius_m, uint64_t *out, size_t cap, size_t *needed)
{
    ensure_lookup();
    *needed = 0;
    if (lat > 90.0 || lat < -90.0 || lng > 180.0 || lng < -180.0) return ORC_ERR_BAD_COORD_SET;
    if (!(radius_m > 0)) return ORC_ERR_RADIUS;
    V3 pts[20];
    orc_regular_loop(lat, lng, radius_m, 20, (double *)pts);
    Loop l;
    loop_init(&l, pts, 20);
    U64Vec cells = {0, 0, 0};
    if (cover_loop(&l, &cells)) { free(cells.v); return ORC_ERR_NOMEM; }
    emit(&cells, out, cap, needed);
    free(cells.v);
    return ORC_OK;
}

/* Test hooks for individual predicates / primitives. */
int orc_robust_sign(const double *a, const double *b, const double *c)
{
    return robust_sign(*(const V3 *)a, *(const V3 *)b, *(const V3 *)c);
}
int orc_loop_contains(const double *xyz, int n, const double *p)
{
    ensure_lookup();
    Loop l;
    loop_init(&l, (const V3 *)xyz, n);
    return loop_brute_contains(&l, *(const V3 *)p);
}
void orc_cell_uv_bound(uint64_t id, double out[4])
{
    ensure_lookup();
    Cell c = cell_from_id(id);
    out[0] = c.ulo;
    out[1] = c.uhi;
    out[2] = c.vlo;
    out[3] = c.vhi;
}
void orc_cell_center(uint64_t id, double out[3])
{
    ensure_lookup();
    Cell c = cell_from_id(id);
    V3 p = cell_center(&c);
    out[0] = p.x;
    out[1] = p.y;
    out[2] = p.z;
}
uint64_t orc_cellid_from_face_ij_level(int face, int i, int j, int level, int *orientation)
{
    ensure_lookup();
    uint64_t id = cellid_parent(cellid_from_face_ij(face, i, j), level);
    int f, ii, jj;
    cellid_face_ij_orientation(id, &f, &ii, &jj, orientation);
    return id;
}
double orc_go_sin(double x) { return go_sin(x); }
double orc_go_cos(double x) { return go_cos(x); }
double orc_go_tan(double x) { return go_tan(x); }
double orc_go_atan(double x) { return go_atan(x); }
double orc_go_atan2(double y, double x) { return go_atan2(y, x); }
double orc_go_asin(double x) { return go_asin(x); }
