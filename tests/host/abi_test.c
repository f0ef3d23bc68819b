/* The C ABI exercised the way the cgo binding (go/pkg/gpu) calls it: plain
 * C99, gcc-compiled, host buffers, no ctypes.  Built by __graft_entry__.build()
 * into tests/host/abi_test; run on the GPU by tests/test_gpu_host_abi.py.
 *
 * Known answers: the reference's covering KAT (pkg/models/geo_test.go:10-55),
 * the covering error statuses of pkg/geo/s2.go:129-166 and
 * pkg/models/geo.go:224-268, and hand-checked searchOperations /
 * SearchISAs / SearchSubscriptionsByOwner answers (operations.go:374-435,
 * identification_service_area.go:166-197, subscriptions.go:247-273) over a
 * three-entity index and the mutable store. */
#include <math.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "dssgpu.h"

static int failures = 0;
#define CHECK(cond, ...)                          \
    do {                                          \
        if (!(cond)) {                            \
            fprintf(stderr, "FAIL %s:%d: ", __FILE__, __LINE__); \
            fprintf(stderr, __VA_ARGS__);         \
            fprintf(stderr, "\n");                \
            failures++;                           \
        }                                         \
    } while (0)

/* Nanoseconds since the epoch -> the microseconds CockroachDB keeps (round
 * half up, as go/pkg/gpu's usOf does with time.Round(time.Microsecond)). */
static int64_t us_round(int64_t ns)
{
    const int64_t q = ns / 1000, r = ns % 1000;
    if (r >= 500) return q + 1;
    if (r < -500) return q - 1;
    return q;
}

static uint64_t token_id(const char *tok)
{
    return (uint64_t)strtoull(tok, NULL, 16) << (64 - 4 * strlen(tok));
}

static const char *kat_tokens[20] = {"808fb0ac", "808fb744", "808fb754", "808fb75c", "808fb9fc", "808fba04", "808fba0c",
                                     "808fba14", "808fba1c", "808fba5c", "808fba64", "808fba6c", "808fba74", "808fba8c",
                                     "808fbad4", "808fbadc", "808fbae4", "808fbaec", "808fbaf4", "808fbb2c"};
static const double kat_lat[3] = {37.427636, 37.408799, 37.421265};
static const double kat_lng[3] = {-122.170502, -122.064069, -122.086504};

static int cover_one(dssg_ctx *ctx, int32_t kind, const double *lat, const double *lng, int64_t nv, float radius,
                     uint64_t *cells, int64_t cap, int64_t *ncells, int32_t *status)
{
    const int64_t voff[2] = {0, nv};
    int64_t offs[2] = {0, 0}, needed = 0;
    double area = 0;
    const int rc = dssg_cover_batch(ctx, 1, &kind, voff, lat, lng, &radius, offs, cells, cap, &needed, status, &area);
    *ncells = offs[1];
    return rc;
}

int main(void)
{
    dssg_ctx *ctx = NULL;
    int rc = dssg_create(0, &ctx);
    if (rc != DSSG_OK) {
        fprintf(stderr, "dssg_create: %s\n", dssg_strerror(rc));
        return rc == DSSG_ERR_NO_DEVICE ? 2 : 1;
    }

    /* ---- covering KAT ---------------------------------------------------- */
    uint64_t kat[20], cells[4096];
    for (int i = 0; i < 20; i++) kat[i] = token_id(kat_tokens[i]);
    int64_t n = 0;
    int32_t st = -1;
    rc = cover_one(ctx, DSSG_KIND_POLYGON, kat_lat, kat_lng, 3, 0.f, cells, 4096, &n, &st);
    CHECK(rc == DSSG_OK && st == DSSG_ST_OK && n == 20, "polygon KAT rc=%d st=%d n=%lld", rc, st, (long long)n);
    CHECK(memcmp(cells, kat, sizeof(kat)) == 0, "polygon KAT cells differ");

    /* the same points through geo.AreaToCellIDs */
    int64_t needed = 0;
    double km2 = 0;
    rc = dssg_area_to_cell_ids(ctx, "37.427636,-122.170502,37.408799,-122.064069,37.421265,-122.086504", cells, 4096,
                               &needed, &st, &km2);
    CHECK(rc == DSSG_OK && st == DSSG_ST_OK && needed == 20 && memcmp(cells, kat, sizeof(kat)) == 0,
          "area string KAT rc=%d st=%d n=%lld", rc, st, (long long)needed);
    /* capacity protocol: too small a buffer reports the size */
    rc = dssg_area_to_cell_ids(ctx, "37.427636,-122.170502,37.408799,-122.064069,37.421265,-122.086504", cells, 4,
                               &needed, &st, &km2);
    CHECK(rc == DSSG_ERR_CAPACITY && needed == 20, "capacity rc=%d needed=%lld", rc, (long long)needed);

    /* error statuses (pkg/geo/s2.go:129-166) */
    rc = dssg_area_to_cell_ids(ctx, "1,2,3", cells, 4096, &needed, &st, &km2);
    CHECK(rc == DSSG_OK && st == DSSG_ST_ODD_COORDS, "odd st=%d", st);
    rc = dssg_area_to_cell_ids(ctx, "1,2,3,4", cells, 4096, &needed, &st, &km2);
    CHECK(rc == DSSG_OK && st == DSSG_ST_NOT_ENOUGH_POINTS, "few st=%d", st);
    rc = dssg_area_to_cell_ids(ctx, "1,2,x,4,5,6", cells, 4096, &needed, &st, &km2);
    CHECK(rc == DSSG_OK && st == DSSG_ST_BAD_COORD_SET, "bad st=%d", st);
    rc = dssg_area_to_cell_ids(ctx, "10,10,10,20,20,20,20,10", cells, 4096, &needed, &st, &km2);
    CHECK(rc == DSSG_OK && st == DSSG_ST_AREA_TOO_LARGE && km2 > 2500.0, "large st=%d km2=%f", st, km2);

    /* GeoPolygon / GeoCircle checks (pkg/models/geo.go:224-268) */
    const double bad_lat[3] = {91.0, 37.4, 37.5}, bad_lng[3] = {-122.1, -122.2, -122.1};
    rc = cover_one(ctx, DSSG_KIND_POLYGON, bad_lat, bad_lng, 3, 0.f, cells, 4096, &n, &st);
    CHECK(rc == DSSG_OK && st == DSSG_ST_BAD_COORD_SET, "lat 91 st=%d", st);
    rc = cover_one(ctx, DSSG_KIND_POLYGON, kat_lat, kat_lng, 2, 0.f, cells, 4096, &n, &st);
    CHECK(rc == DSSG_OK && st == DSSG_ST_NOT_ENOUGH_POINTS, "2 vertices st=%d", st);
    rc = cover_one(ctx, DSSG_KIND_CIRCLE, kat_lat, kat_lng, 1, 0.f, cells, 4096, &n, &st);
    CHECK(rc == DSSG_OK && st == DSSG_ST_RADIUS, "radius 0 st=%d", st);
    uint64_t circle[4096];
    int64_t ncircle = 0;
    rc = cover_one(ctx, DSSG_KIND_CIRCLE, kat_lat, kat_lng, 1, 300.f, circle, 4096, &ncircle, &st);
    CHECK(rc == DSSG_OK && st == DSSG_ST_OK && ncircle > 0, "circle rc=%d st=%d n=%lld", rc, st, (long long)ncircle);
    const double far_lat[1] = {40.7}, far_lng[1] = {-74.0};
    uint64_t far[4096];
    int64_t nfar = 0;
    rc = cover_one(ctx, DSSG_KIND_CIRCLE, far_lat, far_lng, 1, 500.f, far, 4096, &nfar, &st);
    CHECK(rc == DSSG_OK && st == DSSG_ST_OK && nfar > 0, "far circle");

    /* ---- index + searches ------------------------------------------------ */
    /* e0: KAT cells, alt [0, 100], t [1000, 2000]; e1: KAT cells, alt [200, 300],
     * t [1000, 2000]; e2: far cells.  Owners 7, 8, 7. */
    const int64_t ne = 3;
    int64_t eoffs[4] = {0, 20, 40, 40 + nfar};
    uint64_t *ecells = malloc(sizeof(uint64_t) * (size_t)(40 + nfar));
    memcpy(ecells, kat, sizeof(kat));
    memcpy(ecells + 20, kat, sizeof(kat));
    memcpy(ecells + 40, far, sizeof(uint64_t) * (size_t)nfar);
    const float alo[3] = {0.f, 200.f, 0.f}, ahi[3] = {100.f, 300.f, 100.f};
    const int64_t t0[3] = {1000, 1000, 1000}, t1[3] = {2000, 2000, 2000};
    const int32_t owner[3] = {7, 8, 7};
    dssg_index *idx = NULL;
    rc = dssg_index_build(ctx, ne, eoffs, ecells, alo, ahi, t0, t1, owner, &idx);
    CHECK(rc == DSSG_OK && idx, "index build rc=%d %s", rc, dssg_last_error(ctx));
    if (idx) {
        uint32_t oq[16], oe[16];
        /* SCD: the circle around Stanford, alt [50, 150], [1500, 1600], now 0 -> e0 */
        int64_t qoffs[2] = {0, ncircle};
        float qlo = 50.f, qhi = 150.f;
        int64_t qs = 1500, qe = 1600;
        rc = dssg_search_operations(ctx, idx, 1, qoffs, circle, &qlo, &qhi, &qs, &qe, 0, oq, oe, 16, &needed);
        CHECK(rc == DSSG_OK && needed == 1 && oe[0] == 0, "search_operations rc=%d n=%lld e=%u", rc,
              (long long)needed, needed ? oe[0] : 0u);
        /* NULL altitudes -> e0, e1 */
        qlo = -INFINITY;
        qhi = INFINITY;
        rc = dssg_search_operations(ctx, idx, 1, qoffs, circle, &qlo, &qhi, &qs, &qe, 0, oq, oe, 16, &needed);
        CHECK(rc == DSSG_OK && needed == 2 && oe[0] + oe[1] == 1 && oe[0] <= 1 && oe[1] <= 1, "null altitudes n=%lld",
              (long long)needed);
        /* now past every ends_at -> none */
        rc = dssg_search_operations(ctx, idx, 1, qoffs, circle, &qlo, &qhi, &qs, &qe, 2001, oq, oe, 16, &needed);
        CHECK(rc == DSSG_OK && needed == 0, "expired n=%lld", (long long)needed);
        /* the caller's time rule (dssgpu.h "Times"): CockroachDB stores and
         * compares TIMESTAMPTZ rounded to the microsecond, half up (Go's
         * time.Round), so `now` = 2000 us + 500 ns is 2001 us and no row whose
         * ends_at is 2000 us matches, while 2000 us + 499 ns is 2000 us and both
         * match (truncating the nanoseconds would return them for +500 too). */
        {
            const int64_t now_ns[2] = {2000 * 1000 + 500, 2000 * 1000 + 499};
            const int64_t want[2] = {0, 2};
            for (int k = 0; k < 2; k++) {
                const int64_t now_us = us_round(now_ns[k]);
                rc = dssg_search_operations(ctx, idx, 1, qoffs, circle, &qlo, &qhi, &qs, &qe, now_us, oq, oe, 16,
                                            &needed);
                CHECK(rc == DSSG_OK && needed == want[k], "now %lld ns (%lld us): n=%lld want %lld",
                      (long long)now_ns[k], (long long)now_us, (long long)needed, (long long)want[k]);
            }
        }
        /* RID SearchISAs: earliest 1999, latest NULL -> e0, e1 */
        int64_t earliest = 1999, latest = DSSG_TIME_NULL_END_Q;
        rc = dssg_search_isas(ctx, idx, 1, qoffs, circle, &earliest, &latest, oq, oe, 16, &needed);
        CHECK(rc == DSSG_OK && needed == 2, "search_isas n=%lld", (long long)needed);
        /* RID SearchSubscriptionsByOwner: owner 8 -> e1; any owner over the far cells -> e2 */
        int32_t qown = 8;
        rc = dssg_search_subscriptions(ctx, idx, 1, qoffs, circle, &qown, 0, oq, oe, 16, &needed);
        CHECK(rc == DSSG_OK && needed == 1 && oe[0] == 1, "subscriptions by owner n=%lld", (long long)needed);
        int64_t foffs[2] = {0, nfar};
        qown = -1;
        rc = dssg_search_subscriptions(ctx, idx, 1, foffs, far, &qown, 0, oq, oe, 16, &needed);
        CHECK(rc == DSSG_OK && needed == 1 && oe[0] == 2, "subscriptions far n=%lld", (long long)needed);
        dssg_index_free(idx);
    }

    /* ---- the mutable store (write path) ------------------------------------ */
    dssg_store *store = NULL;
    rc = dssg_store_create(ctx, 0, &store);
    CHECK(rc == DSSG_OK && store, "store create rc=%d", rc);
    if (store) {
        const uint32_t ids[3] = {10, 11, 12};
        rc = dssg_store_upsert(ctx, store, 3, ids, eoffs, ecells, alo, ahi, t0, t1, NULL);
        CHECK(rc == DSSG_OK, "upsert rc=%d %s", rc, dssg_last_error(ctx));
        uint32_t oq[16], oid[16];
        int64_t qoffs[2] = {0, 20};
        float qlo = -INFINITY, qhi = INFINITY;
        int64_t tlo = 1500, thi = DSSG_TIME_NULL_END_Q;
        rc = dssg_store_search(ctx, store, 1, qoffs, kat, &qlo, &qhi, &tlo, &thi, NULL, oq, oid, 16, &needed);
        CHECK(rc == DSSG_OK && needed == 2 && oid[0] == 10 && oid[1] == 11, "store search n=%lld", (long long)needed);
        int32_t found = 0;
        const uint32_t del = 10;
        rc = dssg_store_delete(ctx, store, 1, &del, &found);
        CHECK(rc == DSSG_OK && found == 1, "delete rc=%d found=%d", rc, found);
        rc = dssg_store_search(ctx, store, 1, qoffs, kat, &qlo, &qhi, &tlo, &thi, NULL, oq, oid, 16, &needed);
        CHECK(rc == DSSG_OK && needed == 1 && oid[0] == 11, "after delete n=%lld", (long long)needed);
        /* move id 11 to the far cells: the KAT query no longer sees it */
        const int64_t moffs[2] = {0, nfar};
        rc = dssg_store_upsert(ctx, store, 1, &ids[1], moffs, far, &alo[1], &ahi[1], &t0[1], &t1[1], NULL);
        CHECK(rc == DSSG_OK, "re-upsert rc=%d", rc);
        rc = dssg_store_search(ctx, store, 1, qoffs, kat, &qlo, &qhi, &tlo, &thi, NULL, oq, oid, 16, &needed);
        CHECK(rc == DSSG_OK && needed == 0, "after move n=%lld", (long long)needed);
        dssg_store_free(store);
    }
    /* ---- UpsertOperation replayed as go/pkg/gpu runs it --------------------
     * (operations.go:304-372 through the ConflictSearch hook of patch 0002): the
     * conflict search on the store with the transaction's pending writes
     * overlaid on the host (Row.Matches), the OVN set difference, the write at
     * commit, the re-search. */
    {
        dssg_store *ms = NULL;
        rc = dssg_store_create(ctx, 0, &ms);
        CHECK(rc == DSSG_OK && ms, "mirror create rc=%d", rc);
        const int64_t now = 1000;
        /* committed: op A (id 1) over the KAT cells, [1000, 5000], alt [0, 100]; OVN "A" */
        const uint32_t idA = 1;
        const int64_t offsA[2] = {0, 20}, t0A = 1000, t1A = 5000;
        const float loA = 0.f, hiA = 100.f;
        rc = dssg_store_upsert(ctx, ms, 1, &idA, offsA, kat, &loA, &hiA, &t0A, &t1A, NULL);
        CHECK(rc == DSSG_OK, "mirror upsert A rc=%d", rc);
        /* the transaction writes op B (id 2): same cells, [2000, 3000], alt [50, 150] */
        const float loB = 50.f, hiB = 150.f;
        const int64_t t0B = 2000, t1B = 3000;
        uint32_t oq[8], oid[8];
        const int64_t qoffs[2] = {0, 20};
        int64_t tlo = t0B > now ? t0B : now, thi = t1B;
        /* conflict search of B's volume, key = {} -> A is missing (409) */
        rc = dssg_store_search(ctx, ms, 1, qoffs, kat, &loB, &hiB, &tlo, &thi, NULL, oq, oid, 8, &needed);
        CHECK(rc == DSSG_OK && needed == 1 && oid[0] == idA, "conflict search n=%lld", (long long)needed);
        /* key = {A's OVN}: nothing missing, B is written in the transaction (pending, not in the mirror) */
        /* re-search inside the transaction (read-your-writes): the mirror's {A} plus pending B if it matches */
        const float qlo = 0.f, qhi = 500.f;
        int64_t qtlo = 2500, qthi = 2600;
        rc = dssg_store_search(ctx, ms, 1, qoffs, kat, &qlo, &qhi, &qtlo, &qthi, NULL, oq, oid, 8, &needed);
        const int b_matches = t1B >= qtlo && t0B <= qthi && hiB >= qlo && loB <= qhi; /* Row.Matches, cells shared */
        CHECK(rc == DSSG_OK && needed == 1 && oid[0] == idA && b_matches, "read-your-writes n=%lld", (long long)needed);
        /* commit: B reaches the mirror */
        const uint32_t idB = 2;
        rc = dssg_store_upsert(ctx, ms, 1, &idB, qoffs, kat, &loB, &hiB, &t0B, &t1B, NULL);
        CHECK(rc == DSSG_OK, "mirror upsert B rc=%d", rc);
        rc = dssg_store_search(ctx, ms, 1, qoffs, kat, &qlo, &qhi, &qtlo, &qthi, NULL, oq, oid, 8, &needed);
        CHECK(rc == DSSG_OK && needed == 2 && oid[0] == idA && oid[1] == idB, "after commit n=%lld", (long long)needed);
        /* op C over both with key = {A}: B is missing */
        int64_t ctlo = 2000, cthi = 4000;
        rc = dssg_store_search(ctx, ms, 1, qoffs, kat, &qlo, &qhi, &ctlo, &cthi, NULL, oq, oid, 8, &needed);
        int missing = 0;
        for (int64_t k = 0; k < needed; k++) missing += oid[k] != idA;
        CHECK(rc == DSSG_OK && needed == 2 && missing == 1, "C conflicts n=%lld missing=%d", (long long)needed, missing);
        /* B's end before C's start: no conflict with B (COALESCE(ends_at >= start)) */
        ctlo = 3001;
        rc = dssg_store_search(ctx, ms, 1, qoffs, kat, &qlo, &qhi, &ctlo, &cthi, NULL, oq, oid, 8, &needed);
        CHECK(rc == DSSG_OK && needed == 1 && oid[0] == idA, "time-disjoint n=%lld", (long long)needed);
        /* DeleteOperation of A, committed: only B remains */
        int32_t found = 0;
        rc = dssg_store_delete(ctx, ms, 1, &idA, &found);
        CHECK(rc == DSSG_OK && found == 1, "mirror delete rc=%d", rc);
        ctlo = 2000;
        rc = dssg_store_search(ctx, ms, 1, qoffs, kat, &qlo, &qhi, &ctlo, &cthi, NULL, oq, oid, 8, &needed);
        CHECK(rc == DSSG_OK && needed == 1 && oid[0] == idB, "after delete A n=%lld", (long long)needed);
        dssg_store_free(ms);
    }
    /* ---- RID subscription mirror, as go/pkg/gpu/rid.go calls it -------------
     * UpdateNotificationIdxsInCells (subscriptions.go:204-219): the mirror
     * finds the subscriptions sharing a cell with the ISA and unexpired
     * (cells && $1 AND ends_at >= now); CRDB only runs the UPDATE ... WHERE
     * id = ANY($ids) ... RETURNING (the counters here stand in for that
     * column).  The reference's fan-out KAT (isa_test.go:266-324: 42 -> 43
     * on the ISA insert -> 44 on its delete) and the max-count KAT
     * (subscriptions_test.go:275-287: 2 of "myself"'s subscriptions share
     * cell 12494535935418957824) over the subscriptions pool of
     * subscriptions_test.go:19-64. */
    {
        const uint64_t pool = 12494535935418957824ull, overflow = 17106221850767130624ull;
        const uint64_t cells[4] = {overflow, pool, pool, pool};
        const int64_t soffs[4] = {0, 2, 3, 4};
        const uint32_t sid[3] = {0, 1, 2};
        const int32_t sowner[3] = {0, 0, 1}; /* "myself", "myself", "me" */
        const int64_t now = 1600000000000000ll, day = 86400000000ll;
        const int64_t st0[3] = {now, now, now}, st1[3] = {now + day, now + day, now + day};
        const float slo[3] = {-INFINITY, -INFINITY, -INFINITY}, shi[3] = {INFINITY, INFINITY, INFINITY};
        int64_t counter[3] = {42, 42, 42}; /* notification_index in CRDB */
        dssg_store *subs = NULL;
        rc = dssg_store_create(ctx, 1, &subs);
        CHECK(rc == DSSG_OK && subs, "subscription mirror create rc=%d", rc);
        rc = dssg_store_upsert(ctx, subs, 3, sid, soffs, cells, slo, shi, st0, st1, sowner);
        CHECK(rc == DSSG_OK, "subscription mirror upsert rc=%d", rc);
        const int64_t qoffs[2] = {0, 1};
        const float qlo = -INFINITY, qhi = INFINITY;
        for (int round = 0; round < 2; round++) { /* the ISA insert, then its delete */
            int64_t qtlo = now, qthi = DSSG_TIME_NULL_END_Q;
            uint32_t oq[8], oid[8];
            rc = dssg_store_search(ctx, subs, 1, qoffs, &pool, &qlo, &qhi, &qtlo, &qthi, NULL, oq, oid, 8, &needed);
            CHECK(rc == DSSG_OK && needed == 3, "fan-out search n=%lld", (long long)needed);
            for (int64_t k = 0; k < needed; k++)
                if (oid[k] < 3 && st1[oid[k]] >= now) counter[oid[k]]++; /* UPDATE ... WHERE id = ANY($ids) */
            CHECK(counter[0] == 43 + round && counter[1] == 43 + round && counter[2] == 43 + round,
                  "notification index after round %d: %lld %lld %lld", round, (long long)counter[0],
                  (long long)counter[1], (long long)counter[2]);
        }
        /* expired subscriptions are not notified (ends_at >= now) */
        {
            int64_t qtlo = now + 2 * day, qthi = DSSG_TIME_NULL_END_Q;
            uint32_t oq[8], oid[8];
            rc = dssg_store_search(ctx, subs, 1, qoffs, &pool, &qlo, &qhi, &qtlo, &qthi, NULL, oq, oid, 8, &needed);
            CHECK(rc == DSSG_OK && needed == 0, "expired fan-out n=%lld", (long long)needed);
        }
        int64_t count = -1;
        const int32_t myself = 0, me = 1;
        rc = dssg_store_max_subscription_count(ctx, subs, 1, qoffs, &pool, &myself, now, &count);
        CHECK(rc == DSSG_OK && count == 2, "max count KAT rc=%d count=%lld", rc, (long long)count);
        rc = dssg_store_max_subscription_count(ctx, subs, 1, qoffs, &overflow, &me, now, &count);
        CHECK(rc == DSSG_OK && count == 0, "max count (none) count=%lld", (long long)count);
        int32_t found = 0;
        rc = dssg_store_delete(ctx, subs, 1, &sid[1], &found);
        rc = dssg_store_max_subscription_count(ctx, subs, 1, qoffs, &pool, &myself, now, &count);
        CHECK(rc == DSSG_OK && found == 1 && count == 1, "max count after delete count=%lld", (long long)count);
        dssg_store_free(subs);
    }
    free(ecells);
    dssg_destroy(ctx);
    if (failures) {
        fprintf(stderr, "%d failure(s)\n", failures);
        return 1;
    }
    printf("abi_test ok\n");
    return 0;
}
