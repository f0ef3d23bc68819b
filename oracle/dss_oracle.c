/* ORACLE / TEST INFRASTRUCTURE ONLY -- never linked into the product path.
 *
 * Batch driver for the covering restatement (s2_oracle.c) and an in-memory
 * restatement of the store-side overlap search that the reference pushes into
 * CockroachDB v20.1.1 as SQL:
 *   - SCD searchOperations  pkg/scd/store/cockroach/operations.go:374-435
 *       op.id IN (SELECT DISTINCT operation_id FROM scd_cells_operations
 *                 WHERE cell_id = ANY($1))
 *       AND COALESCE(op.altitude_upper >= $2, true)
 *       AND COALESCE(op.altitude_lower <= $3, true)
 *       AND COALESCE(op.ends_at >= $4, true)
 *       AND COALESCE(op.starts_at <= $5, true)
 *       AND op.ends_at >= $6 (now)
 *   - RID SearchISAs         pkg/rid/cockroach/identification_service_area.go:166-197
 *       ends_at >= $1 AND COALESCE(starts_at <= $2, true) AND cells && $3
 *   - RID SearchSubscriptions[ByOwner] pkg/rid/cockroach/subscriptions.go:222-273
 *       cells && $1 [AND owner = $2] AND ends_at >= now
 * Every form reduces to the generic predicate documented in oracle.h once the
 * COALESCE/NULL cases are mapped to sentinels.  The join is a
 * sorted posting list (cell, entity) probed per query cell by binary search,
 * then per-query sort-unique (the SQL DISTINCT / set semantics, Q13).
 */
#include <math.h>
#include <pthread.h>
#include <stdlib.h>
#include <string.h>

#include "oracle.h"

void orc_free(void *p) { free(p); }

/* ------------------------------------------------------------ covering */
/* pkg/geo/s2.go:145-165: AreaToCellIDs converts without a range check (Q5)
 * and needs >= 3 points, then Covering. */
static int points_covering(const double *lat, const double *lng, int n, uint64_t *out, size_t cap, size_t *needed,
                           double *area)
{
    *needed = 0;
    *area = 0;
    if (n < 3) return ORC_ERR_NOT_ENOUGH_POINTS;
    double *xyz = (double *)malloc(sizeof(double) * 3 * (size_t)n);
    if (!xyz) return ORC_ERR_NOMEM;
    for (int i = 0; i < n; i++) orc_point_from_degrees(lat[i], lng[i], xyz + 3 * i);
    int rc = orc_covering_xyz(xyz, n, out, cap, needed, area);
    free(xyz);
    return rc;
}
typedef struct {
    int64_t n;
    const int32_t *kind;
    const int64_t *voff;
    const double *lat, *lng;
    const float *radius_m;
    int32_t *status;
    double *area;
    uint64_t **cells;
    int64_t *counts;
    int64_t next;
    pthread_mutex_t mu;
} CoverJob;

static void *cover_worker(void *arg)
{
    CoverJob *j = (CoverJob *)arg;
    size_t cap = 4096;
    uint64_t *buf = (uint64_t *)malloc(cap * sizeof(uint64_t));
    for (;;) {
        pthread_mutex_lock(&j->mu);
        int64_t f = j->next;
        j->next += 64;
        pthread_mutex_unlock(&j->mu);
        if (f >= j->n) break;
        int64_t end = f + 64 < j->n ? f + 64 : j->n;
        for (; f < end; f++) {
            size_t needed = 0;
            double area = 0;
            int rc;
            for (;;) {
                int64_t v0 = j->voff[f], nv = j->voff[f + 1] - v0;
                if (j->kind[f] == ORC_KIND_CIRCLE)
                    rc = orc_circle_covering(j->lat[v0], j->lng[v0], j->radius_m[f], buf, cap, &needed);
                else if (j->kind[f] == ORC_KIND_POINTS_XYZ)
                    rc = points_covering(j->lat + v0, j->lng + v0, (int)nv, buf, cap, &needed, &area);
                else
                    rc = orc_polygon_covering(j->lat + v0, j->lng + v0, (int)nv, buf, cap, &needed, &area);
                if (rc == ORC_OK && needed > cap) {
                    cap = needed;
                    buf = (uint64_t *)realloc(buf, cap * sizeof(uint64_t));
                    continue;
                }
                break;
            }
            j->status[f] = rc;
            if (j->area) j->area[f] = area;
            j->counts[f] = rc == ORC_OK ? (int64_t)needed : 0;
            if (rc == ORC_OK && needed) {
                j->cells[f] = (uint64_t *)malloc(needed * sizeof(uint64_t));
                memcpy(j->cells[f], buf, needed * sizeof(uint64_t));
            } else {
                j->cells[f] = NULL;
            }
        }
    }
    free(buf);
    return NULL;
}

int orc_cover_batch(int64_t n, const int32_t *kind, const int64_t *voff, const double *lat, const double *lng,
                    const float *radius_m, int nthreads, int64_t **out_offs, uint64_t **out_cells,
                    int32_t *status, double *area_km2)
{
    /* warm the CellID lookup tables single-threaded */
    (void)orc_cellid_from_degrees(0, 0, 13);
    CoverJob j;
    memset(&j, 0, sizeof(j));
    j.n = n;
    j.kind = kind;
    j.voff = voff;
    j.lat = lat;
    j.lng = lng;
    j.radius_m = radius_m;
    j.status = status;
    j.area = area_km2;
    j.cells = (uint64_t **)calloc((size_t)(n ? n : 1), sizeof(uint64_t *));
    j.counts = (int64_t *)calloc((size_t)(n ? n : 1), sizeof(int64_t));
    pthread_mutex_init(&j.mu, NULL);
    if (nthreads < 1) nthreads = 1;
    pthread_t *th = (pthread_t *)malloc(sizeof(pthread_t) * (size_t)nthreads);
    for (int t = 0; t < nthreads; t++) pthread_create(&th[t], NULL, cover_worker, &j);
    for (int t = 0; t < nthreads; t++) pthread_join(th[t], NULL);
    free(th);
    pthread_mutex_destroy(&j.mu);
    int64_t *offs = (int64_t *)malloc(sizeof(int64_t) * (size_t)(n + 1));
    offs[0] = 0;
    for (int64_t f = 0; f < n; f++) offs[f + 1] = offs[f] + j.counts[f];
    uint64_t *cells = (uint64_t *)malloc(sizeof(uint64_t) * (size_t)(offs[n] ? offs[n] : 1));
    for (int64_t f = 0; f < n; f++) {
        if (j.counts[f]) memcpy(cells + offs[f], j.cells[f], (size_t)j.counts[f] * sizeof(uint64_t));
        free(j.cells[f]);
    }
    free(j.cells);
    free(j.counts);
    *out_offs = offs;
    *out_cells = cells;
    return 0;
}

/* -------------------------------------------------------------- search */
typedef struct {
    uint64_t cell;
    uint32_t e;
} Posting;

static int cmp_posting(const void *a, const void *b)
{
    const Posting *x = (const Posting *)a, *y = (const Posting *)b;
    if (x->cell != y->cell) return x->cell < y->cell ? -1 : 1;
    return (x->e > y->e) - (x->e < y->e);
}
static int cmp_u32(const void *a, const void *b)
{
    uint32_t x = *(const uint32_t *)a, y = *(const uint32_t *)b;
    return (x > y) - (x < y);
}

typedef struct {
    const Posting *post;
    int64_t np;
    const float *e_alt_lo, *e_alt_hi;
    const int64_t *e_t0, *e_t1;
    const int32_t *e_owner;
    const int64_t *q_offs;
    const uint64_t *q_cells;
    const float *q_alt_lo, *q_alt_hi;
    const int64_t *q_tlo, *q_thi;
    const int32_t *q_owner;
    int64_t nq;
    uint32_t **res;
    int64_t *cnt;
    int64_t next;
    pthread_mutex_t mu;
} SearchJob;

static inline int pred(const SearchJob *j, int64_t q, uint32_t e)
{
    if (!(j->e_t1[e] >= j->q_tlo[q])) return 0;
    if (!(j->e_t0[e] <= j->q_thi[q])) return 0;
    if (!(j->e_alt_hi[e] >= j->q_alt_lo[q])) return 0;
    if (!(j->e_alt_lo[e] <= j->q_alt_hi[q])) return 0;
    if (j->q_owner && j->q_owner[q] >= 0 && j->e_owner[e] != j->q_owner[q]) return 0;
    return 1;
}

static void *search_worker(void *arg)
{
    SearchJob *j = (SearchJob *)arg;
    size_t cap = 1024;
    uint32_t *buf = (uint32_t *)malloc(cap * sizeof(uint32_t));
    for (;;) {
        pthread_mutex_lock(&j->mu);
        int64_t q = j->next;
        j->next += 16;
        pthread_mutex_unlock(&j->mu);
        if (q >= j->nq) break;
        int64_t end = q + 16 < j->nq ? q + 16 : j->nq;
        for (; q < end; q++) {
            size_t m = 0;
            for (int64_t k = j->q_offs[q]; k < j->q_offs[q + 1]; k++) {
                uint64_t c = j->q_cells[k];
                /* lower_bound on cell */
                int64_t lo = 0, hi = j->np;
                while (lo < hi) {
                    int64_t mid = (lo + hi) / 2;
                    if (j->post[mid].cell < c) lo = mid + 1;
                    else hi = mid;
                }
                for (int64_t p = lo; p < j->np && j->post[p].cell == c; p++) {
                    uint32_t e = j->post[p].e;
                    if (!pred(j, q, e)) continue;
                    if (m == cap) {
                        cap *= 2;
                        buf = (uint32_t *)realloc(buf, cap * sizeof(uint32_t));
                    }
                    buf[m++] = e;
                }
            }
            qsort(buf, m, sizeof(uint32_t), cmp_u32);
            size_t u = 0;
            for (size_t i = 0; i < m; i++)
                if (u == 0 || buf[u - 1] != buf[i]) buf[u++] = buf[i];
            j->cnt[q] = (int64_t)u;
            if (u) {
                j->res[q] = (uint32_t *)malloc(u * sizeof(uint32_t));
                memcpy(j->res[q], buf, u * sizeof(uint32_t));
            } else {
                j->res[q] = NULL;
            }
        }
    }
    free(buf);
    return NULL;
}

struct orc_index {
    Posting *post;
    int64_t np, ne;
    float *alo, *ahi;
    int64_t *t0, *t1;
    int32_t *owner;
};

orc_index *orc_index_new(int64_t ne, const int64_t *e_offs, const uint64_t *e_cells, const float *e_alt_lo,
                         const float *e_alt_hi, const int64_t *e_t0, const int64_t *e_t1, const int32_t *e_owner)
{
    orc_index *x = (orc_index *)calloc(1, sizeof(orc_index));
    int64_t np = e_offs[ne];
    x->np = np;
    x->ne = ne;
    x->post = (Posting *)malloc(sizeof(Posting) * (size_t)(np ? np : 1));
    for (int64_t e = 0; e < ne; e++)
        for (int64_t k = e_offs[e]; k < e_offs[e + 1]; k++) {
            x->post[k].cell = e_cells[k];
            x->post[k].e = (uint32_t)e;
        }
    qsort(x->post, (size_t)np, sizeof(Posting), cmp_posting);
    size_t n1 = (size_t)(ne ? ne : 1);
    x->alo = (float *)malloc(n1 * sizeof(float));
    x->ahi = (float *)malloc(n1 * sizeof(float));
    x->t0 = (int64_t *)malloc(n1 * sizeof(int64_t));
    x->t1 = (int64_t *)malloc(n1 * sizeof(int64_t));
    x->owner = (int32_t *)calloc(n1, sizeof(int32_t));
    memcpy(x->alo, e_alt_lo, (size_t)ne * sizeof(float));
    memcpy(x->ahi, e_alt_hi, (size_t)ne * sizeof(float));
    memcpy(x->t0, e_t0, (size_t)ne * sizeof(int64_t));
    memcpy(x->t1, e_t1, (size_t)ne * sizeof(int64_t));
    if (e_owner) memcpy(x->owner, e_owner, (size_t)ne * sizeof(int32_t));
    return x;
}

void orc_index_free(orc_index *x)
{
    if (!x) return;
    free(x->post);
    free(x->alo);
    free(x->ahi);
    free(x->t0);
    free(x->t1);
    free(x->owner);
    free(x);
}

int64_t orc_index_search(const orc_index *x, int64_t nq, const int64_t *q_offs, const uint64_t *q_cells,
                         const float *q_alt_lo, const float *q_alt_hi, const int64_t *q_tlo, const int64_t *q_thi,
                         const int32_t *q_owner, int nthreads, uint32_t **out_q, uint32_t **out_e)
{
    SearchJob j;
    memset(&j, 0, sizeof(j));
    j.post = x->post;
    j.np = x->np;
    j.e_alt_lo = x->alo;
    j.e_alt_hi = x->ahi;
    j.e_t0 = x->t0;
    j.e_t1 = x->t1;
    j.e_owner = x->owner;
    j.q_offs = q_offs;
    j.q_cells = q_cells;
    j.q_alt_lo = q_alt_lo;
    j.q_alt_hi = q_alt_hi;
    j.q_tlo = q_tlo;
    j.q_thi = q_thi;
    j.q_owner = q_owner;
    j.nq = nq;
    j.res = (uint32_t **)calloc((size_t)(nq ? nq : 1), sizeof(uint32_t *));
    j.cnt = (int64_t *)calloc((size_t)(nq ? nq : 1), sizeof(int64_t));
    pthread_mutex_init(&j.mu, NULL);
    if (nthreads < 1) nthreads = 1;
    pthread_t *th = (pthread_t *)malloc(sizeof(pthread_t) * (size_t)nthreads);
    for (int t = 0; t < nthreads; t++) pthread_create(&th[t], NULL, search_worker, &j);
    for (int t = 0; t < nthreads; t++) pthread_join(th[t], NULL);
    free(th);
    pthread_mutex_destroy(&j.mu);
    int64_t total = 0;
    for (int64_t q = 0; q < nq; q++) total += j.cnt[q];
    uint32_t *oq = (uint32_t *)malloc(sizeof(uint32_t) * (size_t)(total ? total : 1));
    uint32_t *oe = (uint32_t *)malloc(sizeof(uint32_t) * (size_t)(total ? total : 1));
    int64_t w = 0;
    for (int64_t q = 0; q < nq; q++) {
        for (int64_t i = 0; i < j.cnt[q]; i++) {
            oq[w] = (uint32_t)q;
            oe[w] = j.res[q][i];
            w++;
        }
        free(j.res[q]);
    }
    free(j.res);
    free(j.cnt);
    *out_q = oq;
    *out_e = oe;
    return total;
}

int64_t orc_search(int64_t ne, const int64_t *e_offs, const uint64_t *e_cells, const float *e_alt_lo,
                   const float *e_alt_hi, const int64_t *e_t0, const int64_t *e_t1, const int32_t *e_owner,
                   int64_t nq, const int64_t *q_offs, const uint64_t *q_cells, const float *q_alt_lo,
                   const float *q_alt_hi, const int64_t *q_tlo, const int64_t *q_thi, const int32_t *q_owner,
                   int nthreads, uint32_t **out_q, uint32_t **out_e)
{
    orc_index *x = orc_index_new(ne, e_offs, e_cells, e_alt_lo, e_alt_hi, e_t0, e_t1, e_owner);
    int64_t n = orc_index_search(x, nq, q_offs, q_cells, q_alt_lo, q_alt_hi, q_tlo, q_thi, q_owner, nthreads, out_q,
                                 out_e);
    orc_index_free(x);
    return n;
}
