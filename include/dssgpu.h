/* dssgpu.h -- C ABI of the MI355X (gfx950) spatial-discovery / 4D-conflict
 * engine.  Plain C types only (no HIP, no torch): a Go cgo adapter binds it
 * directly.
 *
 * The engine replaces two halves of the reference (InterUSS DSS,
 * /root/reference) hot path:
 *   covering  pkg/geo/s2.go:99-166 (Covering, AreaToCellIDs) and
 *             pkg/models/geo.go:224-268 (GeoCircle / GeoPolygon
 *             .CalculateCovering), computed by golang/geo's RegionCoverer
 *             {MinLevel:13, MaxLevel:13} (pkg/geo/s2.go:30-35);
 *   search    the CockroachDB overlap queries behind
 *             scdstore.OperationStore.SearchOperations (pkg/scd/store/store.go:29,
 *             impl pkg/scd/store/cockroach/operations.go:374-445),
 *             repos.ISA.SearchISAs (pkg/rid/repos/isa.go:27, impl
 *             pkg/rid/cockroach/identification_service_area.go:166-197) and
 *             repos.Subscription.SearchSubscriptions[ByOwner]
 *             (pkg/rid/repos/subscription.go:26-29, impl
 *             pkg/rid/cockroach/subscriptions.go:222-273).
 *
 * Conventions (cgo rule: C keeps no Go pointer after returning):
 *   - cells are uint64 S2 CellIDs (level 13 on every covering output); the
 *     store's INT64 columns are the same bits reinterpreted (quirk Q12);
 *   - times are int64 microseconds since the Unix epoch (CRDB TIMESTAMPTZ
 *     resolution, quirk Q19); the caller converts a finer time the way CRDB
 *     does, rounding to the nearest microsecond, half up (Go:
 *     t.Round(time.Microsecond), as go/pkg/gpu's usOf), for query bounds,
 *     `now` and stored rows alike -- truncation would disagree with SQL for
 *     a sub-microsecond remainder >= 500 ns; altitudes float32 metres (REAL
 *     columns, Q20);
 *   - NULLs: stored/query NULL altitude -> -INFINITY (lower) / +INFINITY
 *     (upper); stored NULL starts_at -> DSSG_TIME_NULL_START; stored NULL
 *     ends_at -> DSSG_TIME_NULL_END (such a row never matches, Q9); query
 *     NULL start -> DSSG_TIME_NULL_START, query NULL end -> DSSG_TIME_NULL_END_Q.
 *   - variable-size outputs use two-call sizing: pass capacity, get `*needed`;
 *     DSSG_ERR_CAPACITY means "call again with capacity >= *needed".
 *   - *_device entry points take device pointers (HBM resident) and a
 *     hipStream_t passed as void*; outputs stay in context-owned device memory
 *     until the next call on the same context.
 * Every function returns 0 on success or a DSSG_ERR_* code; per-item covering
 * errors are reported in a status array using the DSSG_ST_* codes.
 */
#ifndef DSSGPU_H
#define DSSGPU_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* ---- return codes ---------------------------------------------------- */
#define DSSG_OK 0
#define DSSG_ERR_INVALID 1   /* bad argument (null pointer, negative size) */
#define DSSG_ERR_CAPACITY 2  /* output buffer too small; see *needed */
#define DSSG_ERR_DEVICE 3    /* HIP runtime failure */
#define DSSG_ERR_NOMEM 4
#define DSSG_ERR_NO_DEVICE 5 /* no gfx950 device visible */

/* ---- per-footprint covering status: the Go sentinel errors ----------- */
#define DSSG_ST_OK 0
#define DSSG_ST_BAD_COORD_SET 1     /* errBadCoordSet pkg/geo/s2.go:39, pkg/models/geo.go:37 */
#define DSSG_ST_NOT_ENOUGH_POINTS 2 /* errNotEnoughPointsInPolygon pkg/geo/s2.go:38, pkg/models/geo.go:36 */
#define DSSG_ST_ODD_COORDS 3        /* errOddNumberOfCoordinatesInAreaString pkg/geo/s2.go:37 */
#define DSSG_ST_RADIUS 4            /* errRadiusMustBeLargerThan0 pkg/models/geo.go:38 */
#define DSSG_ST_AREA_TOO_LARGE 5    /* *ErrAreaTooLarge pkg/geo/s2.go:59-66; area in area_km2[] */

/* ---- footprint kinds --------------------------------------------------- */
#define DSSG_KIND_POLYGON 0 /* models.GeoPolygon.CalculateCovering  pkg/models/geo.go:252-268 */
#define DSSG_KIND_CIRCLE 1  /* models.GeoCircle.CalculateCovering   pkg/models/geo.go:224-239 */
#define DSSG_KIND_POINTS 2  /* geo.Covering on parsed points (no lat/lng range check, Q5) pkg/geo/s2.go:99 */

/* ---- time sentinels ---------------------------------------------------- */
#define DSSG_TIME_NULL_START INT64_MIN
#define DSSG_TIME_NULL_END INT64_MIN         /* stored ends_at NULL: row excluded */
#define DSSG_TIME_NULL_END_Q INT64_MAX       /* query end NULL: COALESCE(..., true) */

typedef struct dssg_ctx dssg_ctx;
typedef struct dssg_index dssg_index;

/* Device-resident covering result (context-owned, valid until next call). */
typedef struct {
    int64_t n;              /* footprints */
    const int64_t *offs;    /* device, n+1 */
    const uint64_t *cells;  /* device, offs[n] level-13 cells, sorted per footprint */
    const int32_t *status;  /* device, n (DSSG_ST_*) */
    const double *area_km2; /* device, n (loopAreaKm2 after the reversal step; 0 for circles) */
    int64_t total_cells;
} dssg_cells;

/* Device-resident search result: unordered set of (query, entity) pairs,
 * each pair once (SQL DISTINCT, quirk Q13).  n_tagged is informational: the
 * last n_tagged pairs are the "long x long" ones (both footprints spread
 * beyond one 8x8-cell window) that the join deduplicated after the fact.
 * Cell-range shards (dssg_index_build_range) already return those exactly
 * once across shards (a shard past the first drops the ones whose smallest
 * shared cell lies below its range), so a sharded caller needs no dedupe;
 * dssg_sharded_search_device reports n_tagged = 0. */
typedef struct {
    const uint32_t *q; /* device */
    const uint32_t *e; /* device */
    int64_t n;
    int64_t n_tagged;
} dssg_pairs;

/* ---- context ----------------------------------------------------------- */
int dssg_create(int device, dssg_ctx **out);
void dssg_destroy(dssg_ctx *ctx);
const char *dssg_strerror(int code);
const char *dssg_last_error(dssg_ctx *ctx);

/* ---- covering ----------------------------------------------------------
 * Footprint f: kind[f]; polygon/points vertices lat/lng[voff[f] .. voff[f+1]);
 * circle centre lat/lng[voff[f]] with radius_m[f] (float32 metres, as
 * GeoCircle.RadiusMeter).  Replaces geo.Covering / GeoPolygon / GeoCircle
 * .CalculateCovering (pkg/geo/s2.go:99, pkg/models/geo.go:224,252).
 */
int dssg_cover_batch(dssg_ctx *ctx, int64_t n, const int32_t *kind, const int64_t *voff, const double *lat,
                     const double *lng, const float *radius_m, int64_t *out_offs, uint64_t *out_cells,
                     int64_t cells_cap, int64_t *cells_needed, int32_t *status, double *area_km2);
int dssg_cover_batch_device(dssg_ctx *ctx, int64_t n, const int32_t *d_kind, const int64_t *d_voff,
                            const double *d_lat, const double *d_lng, const float *d_radius_m, void *stream,
                            dssg_cells *out);

/* geo.AreaToCellIDs (pkg/geo/s2.go:129-166): parse "lat0,lng0,lat1,lng1,..."
 * then Covering.  Status via *status (DSSG_ST_*). */
int dssg_area_to_cell_ids(dssg_ctx *ctx, const char *area, uint64_t *out_cells, int64_t cap, int64_t *needed,
                          int32_t *status, double *area_km2);

/* ---- batched ingress: models.UnionVolumes4D (pkg/models/geo.go:126-190) --
 * A batch of multi-extent volumes: extents [vol_offs[v], vol_offs[v+1]) form
 * volume v (vol_offs on device for the _device form).  Extent x: footprint as
 * dssg_cover_batch (kind/voff/lat/lng/radius_m) iff has_fp[x] != 0; altitudes
 * NaN = NULL on input; t0 = DSSG_TIME_NULL_START / t1 = DSSG_TIME_NULL_END_Q = NULL.
 * Per volume: the union of the extents' coverings (sorted, unique; the
 * reference's map order is unspecified, Q14), min start / max end / min
 * altitude_lower / max altitude_upper over the extents carrying them (NULL if
 * none, returned as -INFINITY / +INFINITY so a union volume can be passed
 * straight to the index build or a search), has_footprint, and the first covering error in extent order (status
 * DSSG_ST_*, area_km2 for DSSG_ST_AREA_TOO_LARGE), where UnionVolumes4D would
 * return that error. */
typedef struct {
    int64_t n;                 /* volumes */
    const int64_t *offs;       /* device, n+1 */
    const uint64_t *cells;     /* device, union cells per volume, sorted */
    const int32_t *status;     /* device, n */
    const double *area_km2;    /* device, n */
    const float *alt_lo, *alt_hi;  /* device, n (NULL -> -INFINITY / +INFINITY, the search sentinels) */
    const int64_t *t0, *t1;    /* device, n (NULL sentinels as above) */
    const uint8_t *has_footprint;  /* device, n */
    int64_t total_cells;
} dssg_volumes;
int dssg_union_volumes_device(dssg_ctx *ctx, int64_t nvol, const int64_t *d_vol_offs, const int32_t *d_kind,
                              const int64_t *d_voff, const double *d_lat, const double *d_lng, const float *d_radius_m,
                              const uint8_t *d_has_fp, const float *d_alt_lo, const float *d_alt_hi,
                              const int64_t *d_t0, const int64_t *d_t1, void *stream, dssg_volumes *out);

/* ---- entity index (intents / ISAs / subscriptions) ----------------------
 * Replaces the CRDB tables scd_operations + scd_cells_operations
 * (pkg/scd/store/cockroach/store.go:120-147) and the RID INT64[] cells
 * columns with INVERTED INDEX (pkg/rid/cockroach/store.go:122-151).
 * Entity e: cells[cell_offs[e] .. cell_offs[e+1]), altitude [alt_lo, alt_hi],
 * time [t0, t1] (us), owner id (int32, for SearchSubscriptionsByOwner).
 * Postings are kept per (entity, group of cells), each with the mask of the
 * entity's cells in the group, at one of two grains picked per build: quads
 * (level-12 cells, 2 x 2 level-13 cells: when an entity's cells fill them,
 * >= 1.5 per (entity, quad)) or level-13 cells; dssg_set_tuning
 * "index_grain" forces one.  Results do not depend on the grain.
 */
int dssg_index_build(dssg_ctx *ctx, int64_t n, const int64_t *cell_offs, const uint64_t *cells, const float *alt_lo,
                     const float *alt_hi, const int64_t *t0, const int64_t *t1, const int32_t *owner,
                     dssg_index **out);
int dssg_index_build_device(dssg_ctx *ctx, int64_t n, const int64_t *d_cell_offs, const uint64_t *d_cells,
                            const float *d_alt_lo, const float *d_alt_hi, const int64_t *d_t0, const int64_t *d_t1,
                            const int32_t *d_owner, void *stream, dssg_index **out);
/* Cell-range shard of the same index (the postings table
 * scd_cells_operations is range-partitioned by cell_id, store.go:140-147):
 * postings only for cells in [cell_lo, cell_hi] (uint64 order), entity cell
 * lists whole, so a (query, entity) pair is emitted by exactly one shard --
 * the one holding their smallest shared cell.  Searches take the full query
 * batch.  A range holds whole quads: cell_lo is 0 or a multiple of 2^37 and
 * cell_hi is UINT64_MAX or ends in 37 one bits (else DSSG_ERR_INVALID). */
int dssg_index_build_range(dssg_ctx *ctx, int64_t n, const int64_t *cell_offs, const uint64_t *cells,
                           const float *alt_lo, const float *alt_hi, const int64_t *t0, const int64_t *t1,
                           const int32_t *owner, uint64_t cell_lo, uint64_t cell_hi, dssg_index **out);
int dssg_index_build_range_device(dssg_ctx *ctx, int64_t n, const int64_t *d_cell_offs, const uint64_t *d_cells,
                                  const float *d_alt_lo, const float *d_alt_hi, const int64_t *d_t0, const int64_t *d_t1,
                                  const int32_t *d_owner, uint64_t cell_lo, uint64_t cell_hi, void *stream,
                                  dssg_index **out);
void dssg_index_free(dssg_index *idx);
int64_t dssg_index_num_postings(const dssg_index *idx);
int64_t dssg_index_num_cells(const dssg_index *idx);  /* distinct groups (quads or cells) with postings */
int32_t dssg_index_grain(const dssg_index *idx);      /* S2 level of the posting groups: 12 or 13 */

/* ---- search -------------------------------------------------------------
 * Generic 4D overlap join, the predicate every store search reduces to:
 *   cells(q) && cells(e)  AND  e.t1 >= q.tlo  AND  e.t0 <= q.thi
 *   AND e.alt_hi >= q.alt_lo AND e.alt_lo <= q.alt_hi
 *   AND (q.owner < 0 OR e.owner == q.owner)
 * q.tlo must be > INT64_MIN (it always carries `now` or `earliest`).
 * Limits per call: nq < 2^25 queries (a join record keeps the query id below
 * its flag bits) and < 2^32 - 1 query cells; beyond either, DSSG_ERR_INVALID
 * / DSSG_ERR_CAPACITY -- split the batch.
 */
int dssg_search_device(dssg_ctx *ctx, const dssg_index *idx, int64_t nq, const int64_t *d_q_offs,
                       const uint64_t *d_q_cells, const float *d_q_alt_lo, const float *d_q_alt_hi,
                       const int64_t *d_q_tlo, const int64_t *d_q_thi, const int32_t *d_q_owner, void *stream,
                       dssg_pairs *out);
int dssg_search(dssg_ctx *ctx, const dssg_index *idx, int64_t nq, const int64_t *q_offs, const uint64_t *q_cells,
                const float *q_alt_lo, const float *q_alt_hi, const int64_t *q_tlo, const int64_t *q_thi,
                const int32_t *q_owner, uint32_t *out_q, uint32_t *out_e, int64_t cap, int64_t *needed);

/* scdstore SearchOperations semantics (operations.go:374-435) for a batch of
 * already-covered query volumes: q_start/q_end may be DSSG_TIME_NULL_START /
 * DSSG_TIME_NULL_END_Q; altitudes NULL -> -/+INFINITY (SCD protos always set
 * them, quirk Q8); `now_us` is the store clock.  Owner is ignored (Q6). */
int dssg_search_operations(dssg_ctx *ctx, const dssg_index *idx, int64_t nq, const int64_t *q_offs,
                           const uint64_t *q_cells, const float *q_alt_lo, const float *q_alt_hi,
                           const int64_t *q_start, const int64_t *q_end, int64_t now_us, uint32_t *out_q,
                           uint32_t *out_e, int64_t cap, int64_t *needed);
/* repos.ISA.SearchISAs (identification_service_area.go:166-197): earliest
 * required (the app layer clamps it to now, pkg/rid/application/isa.go:38-45),
 * latest may be DSSG_TIME_NULL_END_Q.  No altitude filter. */
int dssg_search_isas(dssg_ctx *ctx, const dssg_index *idx, int64_t nq, const int64_t *q_offs,
                     const uint64_t *q_cells, const int64_t *earliest, const int64_t *latest, uint32_t *out_q,
                     uint32_t *out_e, int64_t cap, int64_t *needed);
/* repos.Subscription.SearchSubscriptions / SearchSubscriptionsByOwner
 * (subscriptions.go:222-273): owner < 0 means "any owner". */
int dssg_search_subscriptions(dssg_ctx *ctx, const dssg_index *idx, int64_t nq, const int64_t *q_offs,
                              const uint64_t *q_cells, const int32_t *owner, int64_t now_us, uint32_t *out_q,
                              uint32_t *out_e, int64_t cap, int64_t *needed);

/* ---- write path: a mutable store over the index --
 * Replaces the row + posting rewrites of UpsertOperation / pushOperation /
 * DeleteOperation (pkg/scd/store/cockroach/operations.go:119-193, 239-372)
 * and RID InsertISA / DeleteISA (pkg/rid/cockroach/
 * identification_service_area.go:97-160): entities are keyed by a caller id
 * (uint32, the Go side's row handle; 0xffffffff reserved).  Upsert replaces an
 * id's cells and attributes (or inserts it); delete removes it (found[i] = 0
 * if it was not live).  Every later search sees every earlier write.  Inside:
 * an immutable base index, a delta index over the entities written since the
 * base was built (rebuilt per write batch), and a tombstone bitmap that masks
 * the base copies of rewritten/deleted ids in the join; the delta is folded
 * into a new base once it exceeds max(4096, base / 16) entities, or on
 * dssg_store_compact.  Writes must be serialised by the caller (the Go
 * store's transaction); dssg_store_search returns (query, id) pairs sorted.
 * The SCD OVN conflict check of UpsertOperation (operations.go:333-360) is
 * this search with the operation's own volume, minus the ids whose OVN the
 * caller's key holds (dss_amd.store.MutableOperationStore). */
typedef struct dssg_store dssg_store;
int dssg_store_create(dssg_ctx *ctx, int32_t with_owner, dssg_store **out);
void dssg_store_free(dssg_store *st);
int dssg_store_upsert(dssg_ctx *ctx, dssg_store *st, int64_t n, const uint32_t *ids, const int64_t *cell_offs,
                      const uint64_t *cells, const float *alt_lo, const float *alt_hi, const int64_t *t0,
                      const int64_t *t1, const int32_t *owner);
int dssg_store_delete(dssg_ctx *ctx, dssg_store *st, int64_t n, const uint32_t *ids, int32_t *found);
int dssg_store_compact(dssg_ctx *ctx, dssg_store *st);
int dssg_store_stats(const dssg_store *st, int64_t *live, int64_t *base, int64_t *delta, int64_t *compactions);
int dssg_store_search(dssg_ctx *ctx, dssg_store *st, int64_t nq, const int64_t *q_offs, const uint64_t *q_cells,
                      const float *q_alt_lo, const float *q_alt_hi, const int64_t *q_tlo, const int64_t *q_thi,
                      const int32_t *q_owner, uint32_t *out_q, uint32_t *out_id, int64_t cap, int64_t *needed);
/* RID MaxSubscriptionCountInCellsByOwner (pkg/rid/cockroach/
 * subscriptions.go:83-116) over a store's live rows (base + delta, the GPU
 * mirror the Go binding keeps): out_count[q] = max over q's cells of the
 * owner[q] rows with ends_at >= now posted in the cell, repeats of the cell
 * in a row counted (`unnest(cells)`), 0 if none (IFNULL(MAX(..), 0)).  The
 * store must be created with owners. */
int dssg_store_max_subscription_count(dssg_ctx *ctx, dssg_store *st, int64_t nq, const int64_t *q_offs,
                                      const uint64_t *q_cells, const int32_t *owner, int64_t now_us,
                                      int64_t *out_count);

/* ---- subscription-store queries -----------------------------------------
 * Notification fan-out: RID UpdateNotificationIdxsInCells
 * (pkg/rid/cockroach/subscriptions.go:204-219) and SCD
 * fetchSubscriptionsForNotification (pkg/scd/store/cockroach/
 * subscriptions.go:128-173).  For each query q (processed in batch order),
 * every entity sharing a cell with it and with ends_at >= now has its
 * notification_index incremented; pair k returns the value after its own
 * increment (UPDATE ... RETURNING).  Pairs come back sorted by (entity,
 * query).  On DSSG_ERR_CAPACITY no counter moves.  The counters live in the
 * index (0 after a build; set/get copy n host int64 values). */
int dssg_index_set_notification_index(dssg_ctx *ctx, dssg_index *idx, const int64_t *values);
int dssg_index_get_notification_index(dssg_ctx *ctx, const dssg_index *idx, int64_t *values);
int dssg_notify_subscriptions(dssg_ctx *ctx, dssg_index *idx, int64_t nq, const int64_t *q_offs, const uint64_t *q_cells,
                              int64_t now_us, uint32_t *out_q, uint32_t *out_e, int64_t *out_index, int64_t cap,
                              int64_t *needed);
/* SCD SubscriptionStore.SearchSubscriptions (pkg/scd/store/cockroach/
 * subscriptions.go:497-545): its LEFT JOIN keeps every row, so the answer is
 * every entity of owner[q] with ends_at >= now and the cells do not filter
 * (quirk Q7; the caller still rejects an empty covering with BadRequest("no
 * location provided")).  Needs an index built with owners.  Pairs sorted by
 * (query, entity). */
int dssg_owner_subscriptions(dssg_ctx *ctx, const dssg_index *idx, int64_t nq, const int32_t *owner, int64_t now_us,
                             uint32_t *out_q, uint32_t *out_e, int64_t cap, int64_t *needed);
/* RID MaxSubscriptionCountInCellsByOwner (pkg/rid/cockroach/
 * subscriptions.go:83-116) and SCD fetchMaxSubscriptionCountByCellAndOwner
 * (pkg/scd/store/cockroach/subscriptions.go:255-283): out_count[q] = max over
 * the query's cells c of the number of owner[q]'s entities with
 * ends_at >= now that hold c (a cell repeated in a stored array counts each
 * time, as RID's unnest(cells) does), 0 if none (IFNULL).  Query cells may be
 * unsorted or repeated.  Needs an index built with owners. */
int dssg_max_subscription_count(dssg_ctx *ctx, const dssg_index *idx, int64_t nq, const int64_t *q_offs,
                                const uint64_t *q_cells, const int32_t *owner, int64_t now_us, int64_t *out_count);

/* ---- multi-GPU routing (cell-range shards) --------------
 * The reference range-partitions scd_cells_operations by cell_id inside
 * CockroachDB (pkg/scd/store/cockroach/store.go:140-147) and the SQL layer
 * fans `cell_id = ANY($cells)` (operations.go:384-390) out to the ranges.
 * Here, one process per GPU:
 *  1. dssg_route_plan_device + dssg_route_fill_device: the home rank's
 *     covered batch -> ONE send buffer (caller-owned device memory) of
 *     part-major segments.  Part d's segment holds, per query with >= 1 cell
 *     in part d, one DSSG_ROUTE_ROW_BYTES row {i64 tlo, i64 thi, f32 alo,
 *     f32 ahi, u32 qid, u32 ncells}, then those queries' whole cell lists (in
 *     the order of the rows), padded to 32 bytes: seg_bytes[d] =
 *     32 * row_counts[d] + 32 * ceil(cell_counts[d] / 4).  Part d owns cells
 *     c with part_hi[d-1] < c <= part_hi[d] (uint64 order, part_hi[nparts-1]
 *     = UINT64_MAX; d_part_hi is a device array).  The plan returns the
 *     per-part row and cell counts and segment sizes (host arrays of nparts).
 *  2. the caller all-to-alls the segments (one exchange: RCCL over xGMI);
 *  3. dssg_unpack_queries_device: the received segments (source-part-major,
 *     src_rows[s] rows and src_cells[s] cells from part s, each segment laid
 *     out as above) -> a query batch for dssg_search_device against the
 *     part's dssg_index_build_range index (context-owned until the next unpack);
 *  4. dssg_route_pairs_plan_device + dssg_route_pairs_fill_device: that
 *     search's pairs by home part: the pairs of self_part's own queries go
 *     straight to (d_self_q, d_self_e) as (home-local qid, entity) -- no
 *     exchange, no unpacking -- the others part-major into d_send, packed
 *     (home-local qid << 32 | entity), the self part taking no space there;
 *     the caller all-to-alls them back and dssg_unpack_pairs_device splits
 *     the received ones into (qid, entity) arrays.
 * A part sees a query's whole cell list and every entity's whole cell list, so
 * each (query, entity) pair is emitted by exactly one part (the one owning
 * their smallest shared cell; long x long pairs, met on every shard they
 * share a cell with, are dropped by the shards past the smallest): no
 * cross-shard dedupe. */
#define DSSG_MAX_PARTS 64
#define DSSG_ROUTE_ROW_BYTES 32
typedef struct {
    int64_t n;                   /* rows = queries of the batch */
    const int64_t *offs;         /* device, n+1 */
    const uint64_t *cells;       /* device (the caller's received cells) */
    const float *alt_lo, *alt_hi;
    const int64_t *tlo, *thi;
    const uint32_t *home;        /* source part of each row */
    const uint32_t *qid;         /* query index in its home batch */
} dssg_batch;
int dssg_route_plan_device(dssg_ctx *ctx, int64_t nq, const int64_t *d_q_offs, const uint64_t *d_q_cells,
                           int32_t nparts, const uint64_t *d_part_hi, void *stream, int64_t *row_counts,
                           int64_t *cell_counts, int64_t *seg_bytes);
int dssg_route_fill_device(dssg_ctx *ctx, int64_t nq, const int64_t *d_q_offs, const uint64_t *d_q_cells,
                           const float *d_q_alt_lo, const float *d_q_alt_hi, const int64_t *d_q_tlo,
                           const int64_t *d_q_thi, void *stream, void *d_send);
int dssg_unpack_queries_device(dssg_ctx *ctx, const void *d_recv, int32_t nparts, const int64_t *src_rows,
                               const int64_t *src_cells, void *stream, dssg_batch *out);
int dssg_route_pairs_plan_device(dssg_ctx *ctx, const dssg_batch *batch, const dssg_pairs *pairs, int32_t nparts,
                                 int32_t self_part, void *stream, int64_t *counts);
int dssg_route_pairs_fill_device(dssg_ctx *ctx, const dssg_batch *batch, const dssg_pairs *pairs, void *stream,
                                 uint64_t *d_send, uint32_t *d_self_q, uint32_t *d_self_e);
int dssg_unpack_pairs_device(dssg_ctx *ctx, int64_t n, const uint64_t *d_in, uint32_t *d_q, uint32_t *d_e,
                             void *stream);

/* ---- native exchange over RCCL (xGMI) -----------------------------------
 * The sharded step without any framework: one process per GPU, one
 * communicator per process.  Rank 0 makes an id (dssg_comm_unique_id), the
 * processes share it out of band (the Go binding: over its own transport),
 * each calls dssg_comm_init.  RCCL is opened on first use (dlopen, local
 * symbols); without it these calls return DSSG_ERR_DEVICE.
 * dssg_sharded_search_device runs steps 1-4 of the routing protocol above:
 * route the rank's covered batch, all-to-all the fused query segments (one
 * count allgather, one grouped ncclSend/ncclRecv exchange; the rank's own
 * segment is copied locally), join them against this rank's
 * dssg_index_build_range shard, write its own queries' pairs to the output
 * and all-to-all the others' home (one more count allgather + exchange).
 * With one rank the routing is the identity and the batch is joined as
 * given (dssg_set_tuning "route_identity" = 0 forces the general path).
 * Output: this rank's pairs (query index in its own batch, entity), each
 * exactly once, in device memory owned by the communicator or the context
 * until the next call on either.  Collective: every rank calls it, in the
 * same order.  Collectives of different communicators issued by different
 * host threads are NOT supported: RCCL kernels wait for their peers, so two
 * ranks that interleave two communicators' calls differently can deadlock
 * when those kernels share a hardware queue.  One host thread issues every
 * collective of a rank (other threads may cover ahead: no collectives).
 *
 * dssg_sharded_search_async_device: the same step with the pairs' trip home
 * on a second communicator and stream (xcomm, xstream; both distinct from
 * comm, stream): the query exchange and the join run on `stream`, the pair
 * counts, the pair all-to-all and the split on `xstream`, so step k's pairs
 * travel while step k+1 routes and joins.  The output is complete once the
 * work queued on xstream has run; it lives in one of two buffer sets of
 * xcomm, used alternately, so it stays valid until the second next call on
 * xcomm.  Both communicators must span the same ranks in the same order.
 *
 * dssg_sharded_stats: the most recent sharded step on this context --
 * ms[5] = route, query exchange (+ unpack), join, pair packing, pair
 * exchange (+ split), by HIP events when timing is on (dssg_set_timing;
 * the call then waits for both streams), else 0; counts[8] = query bytes
 * sent to / received from other ranks, pair bytes sent / received, routed
 * rows joined here, pairs this shard produced, routed query cells joined
 * here, postings of their distinct cells (timing on, else 0).  Either
 * pointer may be NULL. */
#define DSSG_COMM_ID_BYTES 128
typedef struct dssg_comm dssg_comm;
int dssg_comm_unique_id(uint8_t *id);
int dssg_comm_init(dssg_ctx *ctx, int32_t nranks, int32_t rank, const uint8_t *id, dssg_comm **out);
void dssg_comm_free(dssg_comm *comm);
/* Byte blocks, part-major: send_bytes[d] to rank d, recv_bytes[s] from rank s
 * (the own block, send_bytes[rank] == recv_bytes[rank], is copied locally). */
int dssg_comm_alltoallv_device(dssg_ctx *ctx, dssg_comm *comm, const void *d_send, const int64_t *send_bytes,
                               void *d_recv, const int64_t *recv_bytes, void *stream);
/* A sharded step joins on each shard the rows routed to it from every rank:
 * up to nranks * nq rows, which must stay below the search's 2^25 queries
 * per call (checked: DSSG_ERR_INVALID; the caller splits its batch). */
int dssg_sharded_search_device(dssg_ctx *ctx, dssg_comm *comm, const dssg_index *shard, const uint64_t *d_part_hi,
                               int64_t nq, const int64_t *d_q_offs, const uint64_t *d_q_cells,
                               const float *d_q_alt_lo, const float *d_q_alt_hi, const int64_t *d_q_tlo,
                               const int64_t *d_q_thi, void *stream, dssg_pairs *out);
int dssg_sharded_search_async_device(dssg_ctx *ctx, dssg_comm *comm, dssg_comm *xcomm, const dssg_index *shard,
                                     const uint64_t *d_part_hi, int64_t nq, const int64_t *d_q_offs,
                                     const uint64_t *d_q_cells, const float *d_q_alt_lo, const float *d_q_alt_hi,
                                     const int64_t *d_q_tlo, const int64_t *d_q_thi, void *stream, void *xstream,
                                     dssg_pairs *out);
int dssg_sharded_stats(dssg_ctx *ctx, double *ms, int64_t *counts);

/* ---- per-request path: micro-batcher -------------------------------------
 * The reference covers and searches once per RPC (pkg/scd/operations_handler
 * .go:118-168).  A batcher owns a context and a worker thread; concurrent
 * callers each submit one SCD searchOperations request (an uncovered
 * footprint as dssg_cover_batch takes it, altitudes, start/end, now) and
 * block until the worker has run the batch it joined -- up to max_batch
 * requests, waiting at most max_wait_us after the first -- as one cover
 * launch and one join.  Result: the entity ids (sorted), the covering status
 * (DSSG_ST_*; the caller maps an error or an empty covering to its
 * BadRequest as searchOperations does), area_km2.  The index must outlive
 * the batcher; it is read concurrently, never written. */
typedef struct dssg_batcher dssg_batcher;
int dssg_batcher_create(int device, const dssg_index *idx, int32_t max_batch, int32_t max_wait_us, dssg_batcher **out);
void dssg_batcher_free(dssg_batcher *b);
int dssg_batcher_search_operations(dssg_batcher *b, int32_t kind, int64_t nv, const double *lat, const double *lng,
                                   float radius_m, float alt_lo, float alt_hi, int64_t start, int64_t end,
                                   int64_t now_us, uint32_t *out_e, int64_t cap, int64_t *needed, int32_t *status,
                                   double *area_km2);
int dssg_batcher_stats(dssg_batcher *b, int64_t *requests, int64_t *batches);

/* ---- diagnostics --------------------------------------------------------
 * Average device time (ms) of the most recent launches of the named kernel
 * phase, measured with HIP events on the launching stream (bench.py). */
int dssg_phase_times(dssg_ctx *ctx, double *cover_ms, double *join_ms, double *join_kernel_ms);
void dssg_set_timing(dssg_ctx *ctx, int enabled);
/* Tuning knobs of this context's engines (defaults suit every BASELINE
 * config):  "tag_bucket_avg" = average long x long pairs per deduplication
 * bucket (default 2048; <= 0 selects the full-sort path); "lazy_sig_recs" =
 * join units with at most this many query records load the postings'
 * near-prefix signatures only for the lanes that need them (default 0:
 * always prefetched); "join_shape" = the join's occupancy / pair-stage shape
 * (0: picked per batch from the previous batch's pass density, the default;
 * 1: 7 workgroups per CU with 640-pair stages; 2: 6 with 1024);
 * "index_grain" = the posting grain of the indexes this context builds (0:
 * picked per build, the default; 1: level-13 cells; 2: quads);
 * "index_bands" = altitude bands of the dense posting groups of later builds
 * (1: none, 2..8; default 4: a group's regular postings in alt_lo-quantile
 * runs, so a join tile's altitude hull skips records); "band_dense" = the
 * group size (postings, >= 64) from which the bands apply (default 4096);
 * "record_order" = where the join reads its query records (0: picked per
 * index, the default -- key order when some group holds >= 8192 postings;
 * 1: query order through the sorted keys; 2: key order, permuted after the
 * key sort); "small_search" = the largest batch (queries) the one-launch
 * small join takes (default 4096; 0: never); "route_identity" (below);
 * "cover_wave" = the largest batch (footprints) the covering's
 * wave-per-footprint path takes (default 16384; 0: never);
 * "cover_slot_order" = the general covering's vertex slots polygons first
 * (1, the default) or in footprint order (0); "cover_exact_setup" = 1 sends
 * every general-path footprint through the exact setup (tests; default 0).
 * Results do not depend on any of them.  Unknown key or value:
 * DSSG_ERR_INVALID. */
int dssg_set_tuning(dssg_ctx *ctx, const char *key, int64_t value);
/* Work counters of the most recent search: query-cell keys (cells of the
 * batch whose cell holds postings), join units (<= 64 records x a posting
 * range), (cell, query class) runs, posting broadcasts (wave iterations) and
 * record x posting lane tests.  Any pointer may be NULL. */
int dssg_search_counters(dssg_ctx *ctx, int64_t *keys, int64_t *units, int64_t *runs, int64_t *iters,
                         int64_t *tests);
/* Join events of the most recent search: output flushes (one atomic each)
 * and exact cell-list merges where the prefix signatures were inconclusive
 * (wave events, lanes) -- these three only in a DSS_JOIN_DIAG build, with
 * timing on -- and the long x long pair occurrences that were deduplicated
 * after the join (always).  Any pointer may be NULL. */
int dssg_join_events(dssg_ctx *ctx, int64_t *flushes, int64_t *merges, int64_t *merge_lanes, int64_t *tagged);
/* Long footprints of the most recent search (cells outside one 8x8 level-13
 * window): queries of the batch and bucketed postings of the index.  Only
 * when both are non-zero can a long x long pair exist, and only then does
 * the join run its tagging variant.  Any pointer may be NULL. */
int dssg_join_longs(dssg_ctx *ctx, int64_t *long_queries, int64_t *long_postings);
/* Per-predicate outcome counts of the join's lane tests (which predicate --
 * time, altitude, owner, quad mask -- rejects each test, how many reach the
 * smallest-shared-cell check and how many it drops, staging and emission
 * shapes), summed over every join launch since the last call and cleared by
 * it.  Only a counting build of the library (-DDSS_JOIN_PROFILE) counts:
 * the shipped library sets *written = 0.  Names by dssg_join_profile_name
 * (NULL past the last counter). */
int dssg_join_profile(dssg_ctx *ctx, int64_t *out, int n, int *written);
const char *dssg_join_profile_name(int i);
/* Roofline accounting for a device query batch: total postings the join
 * scans (sum of M_q) and distinct candidate entities before the
 * altitude/time filter (sum of D_q), SURVEY.md s8(d). */
int dssg_search_stats_device(dssg_ctx *ctx, const dssg_index *idx, int64_t nq, const int64_t *d_q_offs,
                             const uint64_t *d_q_cells, void *stream, int64_t *matched, int64_t *distinct);
/* Postings of the distinct cells a device query batch touches, each counted
 * once (the 28 B/posting term of the join's algorithmic byte model, DESIGN.md
 * s5). */
int dssg_search_touched_device(dssg_ctx *ctx, const dssg_index *idx, int64_t nq, const int64_t *d_q_offs,
                               const uint64_t *d_q_cells, void *stream, int64_t *touched);
/* Index shape: postings held, distinct cells, postings of long-duration
 * entities (scanned by every record of their cell) and of long footprints,
 * the largest cell, and dcap (the longest regular duration, us).  Any output
 * pointer may be NULL. */
int dssg_index_info(const dssg_index *idx, int64_t *postings, int64_t *cells, int64_t *long_duration,
                    int64_t *long_footprint, int64_t *max_cell_postings, int64_t *dcap_us);
/* Device-to-device copy on `stream` (e.g. an engine-owned dssg_cells buffer
 * into caller memory before the next call reuses it). */
int dssg_copy_device(dssg_ctx *ctx, void *dst, const void *src, size_t bytes, void *stream);
/* Copy `bytes` from an engine-owned device buffer (dssg_cells / dssg_pairs)
 * to host memory, on the context's device. */
int dssg_copy_to_host(dssg_ctx *ctx, void *dst, const void *src, size_t bytes);
/* Stable LSD radix sort of n device-resident unsigned keys on their low
 * `bits` bits (key_bytes 4 or 8), values (u32, or NULL for keys only)
 * carried along -- the hand-written sort of the index build and the
 * per-batch key grouping (radix.hip), exported for parity tests and the
 * sort-phase roofline.  In and out buffers are distinct.  With ms != NULL
 * the call waits and reports the sort's duration (HIP events on `stream`). */
int dssg_radix_sort_device(dssg_ctx *ctx, int key_bytes, int64_t n, int bits, const void *d_keys_in, void *d_keys_out,
                           const uint32_t *d_vals_in, uint32_t *d_vals_out, void *stream, double *ms);
/* Exclusive prefix sum of n host int64 values through the device scan the
 * covering and search use (scan.hip), the input placed `shift` elements
 * into its device buffer (0..64; odd = 8- but not 16-byte aligned);
 * out[0] = 0, out[k + 1] = in[0] + ... + in[k] -- for parity tests. */
int dssg_selftest_scan(dssg_ctx *ctx, int64_t n, int shift, const int64_t *in, int64_t *out);
/* Evaluate the device restatement of a Go math routine on n inputs
 * (op: 0 sin, 1 cos, 2 tan, 3 atan, 4 atan2(x, y), 5 asin, 6 sqrt, 7 x/y,
 * 8 stToUV, 9 uvToST, 10 PointFromLatLng(x, y).X) -- for bit-exact tests. */
int dssg_selftest_math(dssg_ctx *ctx, int op, int64_t n, const double *x, const double *y, double *out);

#ifdef __cplusplus
}
#endif
#endif
