/* ORACLE / TEST INFRASTRUCTURE ONLY -- never linked into the product path.
 * C restatement of the reference's covering + search semantics, used as the
 * parity checker (tests/, __graft_entry__.smoke) and as the timed CPU baseline
 * (bench.py cpu_baseline, kind "port").  See oracle/s2_oracle.c and
 * oracle/dss_oracle.c for the file:line citations.                        */
#ifndef DSS_ORACLE_H
#define DSS_ORACLE_H
#include <stddef.h>
#include <stdint.h>

#define ORC_COVER_LEVEL 13
#define ORC_MAX_CELLS (1u << 24) /* oracle refuses coverings above this */

/* Status codes: one per Go sentinel error on the path (same numbering as the
 * product ABI, include/dssgpu.h). */
enum {
    ORC_OK = 0,
    ORC_ERR_BAD_COORD_SET = 1,        /* errBadCoordSet            pkg/geo/s2.go:39, pkg/models/geo.go:37 */
    ORC_ERR_NOT_ENOUGH_POINTS = 2,    /* errNotEnoughPointsInPolygon pkg/geo/s2.go:38, pkg/models/geo.go:36 */
    ORC_ERR_ODD_COORDS = 3,           /* errOddNumberOfCoordinatesInAreaString pkg/geo/s2.go:37 */
    ORC_ERR_RADIUS = 4,               /* errRadiusMustBeLargerThan0 pkg/models/geo.go:38 */
    ORC_ERR_AREA_TOO_LARGE = 5,       /* *ErrAreaTooLarge pkg/geo/s2.go:59-66 */
    ORC_ERR_MISSING_CELLS = 6,        /* BadRequest("missing cell IDs for query") */
    ORC_ERR_NOMEM = 100,
};

/* footprint kinds for the batch covering */
enum { ORC_KIND_POLYGON = 0, ORC_KIND_CIRCLE = 1, ORC_KIND_POINTS_XYZ = 2 };

#ifdef __cplusplus
extern "C" {
#endif

void orc_point_from_degrees(double lat, double lng, double out[3]);
uint64_t orc_cellid_from_degrees(double lat, double lng, int level);
double orc_loop_area(const double *xyz, int n);
int orc_covering_xyz(double *xyz, int n, uint64_t *out, size_t cap, size_t *needed, double *area_km2);
int orc_polygon_covering(const double *lat, const double *lng, int n, uint64_t *out, size_t cap, size_t *needed,
                         double *area_km2);
int orc_circle_covering(double lat, double lng, float radius_m, uint64_t *out, size_t cap, size_t *needed);
void orc_regular_loop(double lat, double lng, float radius_m, int num, double *xyz_out);
int orc_robust_sign(const double *a, const double *b, const double *c);
int orc_loop_contains(const double *xyz, int n, const double *p);
void orc_cell_uv_bound(uint64_t id, double out[4]);
void orc_cell_center(uint64_t id, double out[3]);
uint64_t orc_cellid_from_face_ij_level(int face, int i, int j, int level, int *orientation);
double orc_go_sin(double x);
double orc_go_cos(double x);
double orc_go_tan(double x);
double orc_go_atan(double x);
double orc_go_atan2(double y, double x);
double orc_go_asin(double x);

/* Batch covering.  Footprint f: kind[f]; polygons use lat/lng[voff[f]..voff[f+1]);
 * circles use lat/lng[voff[f]] as centre and radius_m[f].
 * Output is malloc'd CSR (*out_offs: n+1, *out_cells), freed with orc_free. */
int orc_cover_batch(int64_t n, const int32_t *kind, const int64_t *voff, const double *lat, const double *lng,
                    const float *radius_m, int nthreads, int64_t **out_offs, uint64_t **out_cells,
                    int32_t *status, double *area_km2);

/* Generic 4D overlap search restating the SQL predicates of
 * pkg/scd/store/cockroach/operations.go:376-402 and
 * pkg/rid/cockroach/identification_service_area.go:170-180,
 * pkg/rid/cockroach/subscriptions.go:222-273:
 *   share >= 1 cell  AND e.t1 >= q.tlo AND e.t0 <= q.thi
 *   AND e.alt_hi >= q.alt_lo AND e.alt_lo <= q.alt_hi
 *   AND (q.owner < 0 OR e.owner == q.owner)
 * NULL conventions: stored NULL start -> INT64_MIN, stored NULL end ->
 * INT64_MIN (row never matches, Q9), query NULL end -> INT64_MAX, stored or
 * query NULL altitudes -> +-INFINITY.  Output pairs sorted by (q, e). */
int64_t orc_search(int64_t ne, const int64_t *e_offs, const uint64_t *e_cells, const float *e_alt_lo,
                   const float *e_alt_hi, const int64_t *e_t0, const int64_t *e_t1, const int32_t *e_owner,
                   int64_t nq, const int64_t *q_offs, const uint64_t *q_cells, const float *q_alt_lo,
                   const float *q_alt_hi, const int64_t *q_tlo, const int64_t *q_thi, const int32_t *q_owner,
                   int nthreads, uint32_t **out_q, uint32_t **out_e);

/* Same search with the posting list built once (CPU-baseline timing). */
typedef struct orc_index orc_index;
orc_index *orc_index_new(int64_t ne, const int64_t *e_offs, const uint64_t *e_cells, const float *e_alt_lo,
                         const float *e_alt_hi, const int64_t *e_t0, const int64_t *e_t1, const int32_t *e_owner);
int64_t orc_index_search(const orc_index *x, int64_t nq, const int64_t *q_offs, const uint64_t *q_cells,
                         const float *q_alt_lo, const float *q_alt_hi, const int64_t *q_tlo, const int64_t *q_thi,
                         const int32_t *q_owner, int nthreads, uint32_t **out_q, uint32_t **out_e);
void orc_index_free(orc_index *x);

void orc_free(void *p);

#ifdef __cplusplus
}
#endif
#endif
