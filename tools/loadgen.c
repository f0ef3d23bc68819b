/* Native load generator for the per-request path (bench.py
 * request_latency).  The reference serves one covering + one search per RPC
 * (pkg/scd/operations_handler.go:118-168) from many concurrent handler
 * goroutines; through the drop-in those are concurrent cgo calls into the
 * library.  Python threads cannot issue calls at that rate (the GIL), so the
 * callers are pthreads here:
 *   dssl_batched: `nthreads` callers, each issuing requests back to back
 *                 through dssg_batcher_search_operations for `seconds`;
 *   dssl_alone:   one caller, one request at a time through the unbatched
 *                 ABI (dssg_cover_batch, then dssg_search_operations), both
 *                 following the capacity protocol.
 * Latencies are per request, in ms.  Benchmark infrastructure, not product. */
#include <pthread.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>
#include <time.h>

#include "dssgpu.h"

typedef struct {
    int64_t nq;
    const int32_t *kind;
    const int64_t *voff;
    const double *lat, *lng;
    const float *rad, *alo, *ahi;
    const int64_t *t0, *t1;
    int64_t now_us;
} Workload;

static double now_s(void)
{
    struct timespec ts;
    clock_gettime(CLOCK_MONOTONIC, &ts);
    return (double)ts.tv_sec + 1e-9 * (double)ts.tv_nsec;
}

typedef struct {
    dssg_batcher *b;
    const Workload *w;
    int tid, nthreads;
    double t_end;
    double *lat_ms;  /* this caller's sample slots */
    int64_t cap, n_samples, n_requests, n_errors;
} Caller;

static void *caller_main(void *arg)
{
    Caller *c = (Caller *)arg;
    const Workload *w = c->w;
    int64_t ocap = 4096;
    uint32_t *out = (uint32_t *)malloc(sizeof(uint32_t) * (size_t)ocap);
    int64_t i = c->tid % w->nq;
    while (now_s() < c->t_end) {
        const int64_t v0 = w->voff[i], nv = w->voff[i + 1] - v0;
        int64_t needed = 0;
        int32_t st = 0;
        double area = 0;
        const double t0 = now_s();
        int rc;
        for (;;) {
            rc = dssg_batcher_search_operations(c->b, w->kind[i], nv, w->lat + v0, w->lng + v0, w->rad[i], w->alo[i],
                                                w->ahi[i], w->t0[i], w->t1[i], w->now_us, out, ocap, &needed, &st,
                                                &area);
            if (rc != DSSG_ERR_CAPACITY) break;
            free(out);
            ocap = needed + 1;
            out = (uint32_t *)malloc(sizeof(uint32_t) * (size_t)ocap);
        }
        const double dt = now_s() - t0;
        if (rc != DSSG_OK) c->n_errors++;
        if (c->n_samples < c->cap) c->lat_ms[c->n_samples++] = 1000.0 * dt;
        c->n_requests++;
        i = (i + c->nthreads) % w->nq;
    }
    free(out);
    return NULL;
}

int dssl_batched(dssg_batcher *b, int nthreads, double seconds, int64_t nq, const int32_t *kind, const int64_t *voff,
                 const double *lat, const double *lng, const float *rad, const float *alo, const float *ahi,
                 const int64_t *t0, const int64_t *t1, int64_t now_us, int64_t max_samples, double *lat_ms,
                 int64_t *n_samples, int64_t *n_requests, int64_t *n_errors, double *wall_s)
{
    if (!b || nthreads < 1 || nq < 1 || max_samples < nthreads) return DSSG_ERR_INVALID;
    Workload w = {nq, kind, voff, lat, lng, rad, alo, ahi, t0, t1, now_us};
    Caller *cs = (Caller *)calloc((size_t)nthreads, sizeof(Caller));
    pthread_t *th = (pthread_t *)calloc((size_t)nthreads, sizeof(pthread_t));
    const int64_t per = max_samples / nthreads;
    const double start = now_s();
    for (int t = 0; t < nthreads; t++) {
        cs[t].b = b;
        cs[t].w = &w;
        cs[t].tid = t;
        cs[t].nthreads = nthreads;
        cs[t].t_end = start + seconds;
        cs[t].lat_ms = lat_ms + (int64_t)t * per;
        cs[t].cap = per;
        pthread_create(&th[t], NULL, caller_main, &cs[t]);
    }
    int64_t ns = 0, nr = 0, ne = 0;
    for (int t = 0; t < nthreads; t++) {
        pthread_join(th[t], NULL);
        /* compact the samples to the front */
        memmove(lat_ms + ns, cs[t].lat_ms, sizeof(double) * (size_t)cs[t].n_samples);
        ns += cs[t].n_samples;
        nr += cs[t].n_requests;
        ne += cs[t].n_errors;
    }
    *wall_s = now_s() - start;
    *n_samples = ns;
    *n_requests = nr;
    *n_errors = ne;
    free(cs);
    free(th);
    return DSSG_OK;
}

int dssl_alone(dssg_ctx *ctx, const dssg_index *idx, int64_t count, int64_t nq, const int32_t *kind,
               const int64_t *voff, const double *lat, const double *lng, const float *rad, const float *alo,
               const float *ahi, const int64_t *t0, const int64_t *t1, int64_t now_us, double *lat_ms,
               int64_t *n_errors)
{
    if (!ctx || !idx || count < 0 || nq < 1) return DSSG_ERR_INVALID;
    int64_t ccap = 4096, pcap = 4096, ne = 0;
    uint64_t *cells = (uint64_t *)malloc(sizeof(uint64_t) * (size_t)ccap);
    uint32_t *oq = (uint32_t *)malloc(sizeof(uint32_t) * (size_t)pcap), *oe = (uint32_t *)malloc(sizeof(uint32_t) * (size_t)pcap);
    for (int64_t k = 0; k < count; k++) {
        const int64_t i = k % nq, v0 = voff[i];
        const int64_t lv[2] = {0, voff[i + 1] - v0};
        int64_t offs[2] = {0, 0}, needed = 0;
        int32_t st = 0;
        double area = 0;
        const double ts = now_s();
        int rc;
        for (;;) {
            rc = dssg_cover_batch(ctx, 1, kind + i, lv, lat + v0, lng + v0, rad + i, offs, cells, ccap, &needed, &st,
                                  &area);
            if (rc != DSSG_ERR_CAPACITY) break;
            free(cells);
            ccap = needed + 1;
            cells = (uint64_t *)malloc(sizeof(uint64_t) * (size_t)ccap);
        }
        if (rc == DSSG_OK && st == DSSG_ST_OK && offs[1] > 0) {
            for (;;) {
                rc = dssg_search_operations(ctx, idx, 1, offs, cells, alo + i, ahi + i, t0 + i, t1 + i, now_us, oq, oe,
                                            pcap, &needed);
                if (rc != DSSG_ERR_CAPACITY) break;
                free(oq);
                free(oe);
                pcap = needed + 1;
                oq = (uint32_t *)malloc(sizeof(uint32_t) * (size_t)pcap);
                oe = (uint32_t *)malloc(sizeof(uint32_t) * (size_t)pcap);
            }
        }
        lat_ms[k] = 1000.0 * (now_s() - ts);
        if (rc != DSSG_OK) ne++;
    }
    free(cells);
    free(oq);
    free(oe);
    *n_errors = ne;
    return DSSG_OK;
}
