// C ABI (include/dssgpu.h) over the gfx950 covering and search engines.
#include <dlfcn.h>
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>  // types only: the library is opened at dssg_comm_init (dlopen, RTLD_LOCAL)

#include <algorithm>
#include <cctype>
#include <cerrno>
#include <cmath>
#include <cstdlib>
#include <cstring>
#include <chrono>
#include <condition_variable>
#include <deque>
#include <mutex>
#include <thread>
#include <string>
#include <type_traits>
#include <vector>

#include "common.hpp"
#include "cover.hpp"
#include "ingress.hpp"
#include "radix.hpp"
#include "route.hpp"
#include "search.hpp"
#include "store.hpp"
#include "subs.hpp"

struct dssg_ctx {
    int device = 0;
    hipStream_t stream = nullptr;
    dss::CoverEngine cover;
    dss::SearchEngine search;
    dss::RouteEngine route;
    dss::SubsEngine subs;
    dss::IngressEngine ingress;
    std::string last_error;
    bool timing = false;
    bool route_identity = true;  // sharded step on one rank: the batch is its own (see dssg_sharded_search_device)
    dss::ShardStats shard_stats;  // the most recent sharded step on this context
    hipEvent_t shard_ev[8] = {};
    double cover_ms = 0, join_ms = 0;
    hipEvent_t ev0 = nullptr, ev1 = nullptr;
    // the most recent device covering's output (its buffers belong to the
    // cover engine until the next covering): a search over exactly that CSR
    // takes its cell count from here instead of reading q_offs[nq] back
    const int64_t *cov_offs = nullptr;
    int64_t cov_n = -1, cov_total = -1;
    // host-API staging
    dss::DevBuf<int32_t> d_kind, d_owner;
    dss::DevBuf<int64_t> d_voff, d_qoffs, d_tlo, d_thi;
    dss::DevBuf<double> d_lat, d_lng;
    dss::DevBuf<float> d_rad, d_alo, d_ahi;
    dss::DevBuf<uint64_t> d_cells;
    dss::DevBuf<unsigned char> sort_tmp;
};

namespace {

template <typename F>
int guarded(dssg_ctx *ctx, F &&f)
{
    try {
        if (ctx) DSS_HIP(hipSetDevice(ctx->device));
        f();
        return DSSG_OK;
    } catch (const dss::Error &e) {
        if (ctx) ctx->last_error = e.what();
        return e.code;
    } catch (const std::bad_alloc &) {
        if (ctx) ctx->last_error = "out of host memory";
        return DSSG_ERR_NOMEM;
    } catch (const std::exception &e) {
        if (ctx) ctx->last_error = e.what();
        return DSSG_ERR_DEVICE;
    }
}

template <typename T>
T *upload(dss::DevBuf<T> &b, const T *h, int64_t n, hipStream_t s)
{
    T *d = b.ensure((size_t)(n > 0 ? n : 1));
    if (n > 0) DSS_HIP(hipMemcpyAsync(d, h, sizeof(T) * (size_t)n, hipMemcpyHostToDevice, s));
    return d;
}

// strconv.ParseFloat(s, 64) grammar (Go 1.14): [+-] (decimal | hex-with-p |
// inf | infinity | nan), no underscores in the forms the DSS ever sees; a
// value out of float64 range is an error (ErrRange).  Returns false on error.
bool go_parse_float(const std::string &s, double &out)
{
    if (s.empty()) return false;
    size_t i = 0;
    std::string t = s;
    if (t[0] == '+' || t[0] == '-') i = 1;
    std::string body = t.substr(i);
    std::string lower = body;
    for (auto &c : lower) c = (char)std::tolower((unsigned char)c);
    if (lower == "inf" || lower == "infinity") {
        out = (t[0] == '-') ? -HUGE_VAL : HUGE_VAL;
        return true;
    }
    if (lower == "nan") {
        if (i) return false;  // Go rejects a signed NaN
        out = std::nan("");
        return true;
    }
    bool hex = lower.size() > 2 && lower[0] == '0' && lower[1] == 'x';
    size_t k = hex ? 2 : 0;
    bool digits = false, dot = false, exp = false;
    for (; k < lower.size(); k++) {
        char c = lower[k];
        if ((hex ? std::isxdigit((unsigned char)c) : std::isdigit((unsigned char)c)) != 0) { digits = true; continue; }
        if (c == '.' && !dot) { dot = true; continue; }
        break;
    }
    if (!digits) return false;
    if (k < lower.size()) {
        char c = lower[k];
        if ((hex && c == 'p') || (!hex && c == 'e')) {
            exp = true;
            k++;
            if (k < lower.size() && (lower[k] == '+' || lower[k] == '-')) k++;
            size_t d0 = k;
            while (k < lower.size() && std::isdigit((unsigned char)lower[k])) k++;
            if (k == d0) return false;
        }
    }
    if (k != lower.size()) return false;
    if (hex && !exp) return false;  // "hexadecimal mantissa requires a 'p' exponent"
    errno = 0;
    char *end = nullptr;
    double v = std::strtod(t.c_str(), &end);
    if (end != t.c_str() + t.size()) return false;
    if (errno == ERANGE && std::isinf(v)) return false;
    out = v;
    return true;
}

std::string trim_space(const std::string &s)
{
    size_t a = 0, b = s.size();
    auto sp = [](unsigned char c) { return c == ' ' || c == '\t' || c == '\n' || c == '\v' || c == '\f' || c == '\r'; };
    while (a < b && sp((unsigned char)s[a])) a++;
    while (b > a && sp((unsigned char)s[b - 1])) b--;
    return s.substr(a, b - a);
}

void sort_pairs_host(uint32_t *q, uint32_t *e, int64_t n)
{
    std::vector<uint64_t> k((size_t)n);
    for (int64_t i = 0; i < n; i++) k[i] = ((uint64_t)q[i] << 32) | e[i];
    std::sort(k.begin(), k.end());
    for (int64_t i = 0; i < n; i++) {
        q[i] = (uint32_t)(k[i] >> 32);
        e[i] = (uint32_t)k[i];
    }
}

// Per-query sort + unique of the query cells (CellUnion order; UnionVolumes4D
// hands the store unsorted cells, quirk Q14), uploaded to the context's
// staging buffers.
void stage_query_cells(dssg_ctx *ctx, int64_t nq, const int64_t *q_offs, const uint64_t *q_cells, hipStream_t s,
                       const int64_t **d_offs, const uint64_t **d_cells)
{
    std::vector<int64_t> offs((size_t)nq + 1, 0);
    std::vector<uint64_t> cells;
    cells.reserve((size_t)q_offs[nq]);
    for (int64_t q = 0; q < nq; q++) {
        size_t b = cells.size();
        cells.insert(cells.end(), q_cells + q_offs[q], q_cells + q_offs[q + 1]);
        std::sort(cells.begin() + (long)b, cells.end());
        cells.erase(std::unique(cells.begin() + (long)b, cells.end()), cells.end());
        offs[(size_t)q + 1] = (int64_t)cells.size();
    }
    *d_offs = upload(ctx->d_qoffs, offs.data(), nq + 1, s);
    *d_cells = upload(ctx->d_cells, cells.data(), (int64_t)cells.size(), s);
}

}  // namespace

extern "C" {

const char *dssg_strerror(int code)
{
    switch (code) {
    case DSSG_OK: return "ok";
    case DSSG_ERR_INVALID: return "invalid argument";
    case DSSG_ERR_CAPACITY: return "output capacity too small";
    case DSSG_ERR_DEVICE: return "device error";
    case DSSG_ERR_NOMEM: return "out of memory";
    case DSSG_ERR_NO_DEVICE: return "no gfx950 device";
    default: return "unknown error";
    }
}

const char *dssg_last_error(dssg_ctx *ctx) { return ctx ? ctx->last_error.c_str() : ""; }

int dssg_create(int device, dssg_ctx **out)
{
    if (!out) return DSSG_ERR_INVALID;
    *out = nullptr;
    int count = 0;
    if (hipGetDeviceCount(&count) != hipSuccess || count <= device || device < 0) return DSSG_ERR_NO_DEVICE;
    hipDeviceProp_t prop;
    if (hipGetDeviceProperties(&prop, device) != hipSuccess) return DSSG_ERR_NO_DEVICE;
    if (std::strncmp(prop.gcnArchName, "gfx950", 6) != 0) return DSSG_ERR_NO_DEVICE;
    dssg_ctx *c = new (std::nothrow) dssg_ctx();
    if (!c) return DSSG_ERR_NOMEM;
    c->device = device;
    int rc = guarded(c, [&] { DSS_HIP(hipStreamCreateWithFlags(&c->stream, hipStreamNonBlocking)); });
    if (rc) {
        delete c;
        return rc;
    }
    *out = c;
    return DSSG_OK;
}

void dssg_destroy(dssg_ctx *ctx)
{
    if (!ctx) return;
    (void)hipSetDevice(ctx->device);
    if (ctx->stream) (void)hipStreamSynchronize(ctx->stream);
    if (ctx->ev0) (void)hipEventDestroy(ctx->ev0);
    if (ctx->ev1) (void)hipEventDestroy(ctx->ev1);
    for (hipEvent_t e : ctx->shard_ev)
        if (e) (void)hipEventDestroy(e);
    if (ctx->stream) (void)hipStreamDestroy(ctx->stream);
    delete ctx;
}

void dssg_set_timing(dssg_ctx *ctx, int enabled)
{
    if (!ctx) return;
    ctx->timing = enabled != 0;
    ctx->search.set_timing(ctx->timing);
}

int dssg_set_tuning(dssg_ctx *ctx, const char *key, int64_t value)
{
    if (!ctx || !key) return DSSG_ERR_INVALID;
    if (std::string(key) == "tag_bucket_avg") {
        ctx->search.set_tag_bucket_avg(value);
        return DSSG_OK;
    }
    if (std::string(key) == "lazy_sig_recs") {
        ctx->search.set_lazy_sig_recs(value);
        return DSSG_OK;
    }
    if (std::string(key) == "join_shape") {  // 0 auto (default), 1 sparse 7 x 640, 2 dense 6 x 1024
        if (value < 0 || value > 2) return DSSG_ERR_INVALID;
        ctx->search.set_join_shape((int)value);
        return DSSG_OK;
    }
    if (std::string(key) == "record_order") {  // join records: 0 auto (default), 1 query order, 2 key order
        if (value < 0 || value > 2) return DSSG_ERR_INVALID;
        ctx->search.set_rec_order((int)value);
        return DSSG_OK;
    }
    if (std::string(key) == "index_bands") {  // altitude bands of dense slots (1: none, 2..8; default 4)
        if (value < 1 || value > 8) return DSSG_ERR_INVALID;
        ctx->search.set_bands((int)value, ctx->search.band_dense());
        return DSSG_OK;
    }
    if (std::string(key) == "band_dense") {  // slot size (postings) from which the bands apply (default 4096)
        if (value < 64) return DSSG_ERR_INVALID;
        ctx->search.set_bands(ctx->search.bands(), value);
        return DSSG_OK;
    }
    if (std::string(key) == "index_grain") {  // 0 auto (default), 1 level-13 cells, 2 quads (level-12 cells)
        if (value < 0 || value > 2) return DSSG_ERR_INVALID;
        ctx->search.set_grain((int)value);
        return DSSG_OK;
    }
    if (std::string(key) == "small_search") {  // max queries of the one-launch small-batch join (0: never)
        ctx->search.set_small_max_q(value);
        return DSSG_OK;
    }
    if (std::string(key) == "route_identity") {  // 0: a one-rank sharded step still routes (the general path)
        ctx->route_identity = value != 0;
        return DSSG_OK;
    }
    if (std::string(key) == "cover_slot_order") {  // 1: vertex slots polygons first (default), 0: footprint order
        ctx->cover.set_slot_order(value != 0);
        return DSSG_OK;
    }
    if (std::string(key) == "cover_exact_setup") {  // 1: every general-path footprint through the exact setup (tests)
        ctx->cover.set_all_exact(value != 0);
        return DSSG_OK;
    }
    if (std::string(key) == "cover_wave") {  // max batch of the wave-path covering (0: general pipeline only)
        ctx->cover.set_wave_max(value);
        return DSSG_OK;
    }
    return DSSG_ERR_INVALID;
}

int dssg_phase_times(dssg_ctx *ctx, double *cover_ms, double *join_ms, double *join_kernel_ms)
{
    if (!ctx) return DSSG_ERR_INVALID;
    if (cover_ms) *cover_ms = ctx->cover_ms;
    if (join_ms) *join_ms = ctx->join_ms;
    if (join_kernel_ms) *join_kernel_ms = ctx->search.last_join_kernel_ms();
    return DSSG_OK;
}

int dssg_search_counters(dssg_ctx *ctx, int64_t *keys, int64_t *units, int64_t *runs, int64_t *iters, int64_t *tests)
{
    if (!ctx) return DSSG_ERR_INVALID;
    int64_t r, i, t;
    ctx->search.last_work(&r, &i, &t);
    if (keys) *keys = ctx->search.last_keys();
    if (units) *units = ctx->search.last_units();
    if (runs) *runs = r;
    if (iters) *iters = i;
    if (tests) *tests = t;
    return DSSG_OK;
}

int dssg_join_events(dssg_ctx *ctx, int64_t *flushes, int64_t *merges, int64_t *merge_lanes, int64_t *tagged)
{
    if (!ctx) return DSSG_ERR_INVALID;
    if (tagged) *tagged = ctx->search.last_tagged();
    int64_t f, m, l;
    ctx->search.last_join_events(&f, &m, &l);
    if (flushes) *flushes = f;
    if (merges) *merges = m;
    if (merge_lanes) *merge_lanes = l;
    return DSSG_OK;
}

int dssg_join_longs(dssg_ctx *ctx, int64_t *long_queries, int64_t *long_postings)
{
    if (!ctx) return DSSG_ERR_INVALID;
    int64_t lq, lp;
    ctx->search.last_longs(&lq, &lp);
    if (long_queries) *long_queries = lq;
    if (long_postings) *long_postings = lp;
    return DSSG_OK;
}

int dssg_join_profile(dssg_ctx *ctx, int64_t *out, int n, int *written)
{
    if (!ctx || n < 0 || (n && !out) || !written) return DSSG_ERR_INVALID;
    *written = 0;
    return guarded(ctx, [&] { *written = dss::join_profile_read(out, n); });
}

const char *dssg_join_profile_name(int i) { return dss::join_profile_name(i); }

int dssg_cover_batch_device(dssg_ctx *ctx, int64_t n, const int32_t *d_kind, const int64_t *d_voff, const double *d_lat,
                            const double *d_lng, const float *d_radius_m, void *stream, dssg_cells *out)
{
    if (!ctx || !out || n < 0 || (n > 0 && (!d_kind || !d_voff || !d_lat || !d_lng || !d_radius_m)))
        return DSSG_ERR_INVALID;
    return guarded(ctx, [&] {
        hipStream_t s = stream ? (hipStream_t)stream : ctx->stream;
        if (ctx->timing) {
            if (!ctx->ev0) { DSS_HIP(hipEventCreate(&ctx->ev0)); DSS_HIP(hipEventCreate(&ctx->ev1)); }
            DSS_HIP(hipEventRecord(ctx->ev0, s));
        }
        ctx->cov_offs = nullptr;
        ctx->cover.run(n, d_kind, d_voff, d_lat, d_lng, d_radius_m, s, out);
        ctx->cov_offs = out->offs;
        ctx->cov_n = n;
        ctx->cov_total = out->total_cells;
        if (ctx->timing) {
            DSS_HIP(hipEventRecord(ctx->ev1, s));
            DSS_HIP(hipEventSynchronize(ctx->ev1));
            float ms = 0;
            DSS_HIP(hipEventElapsedTime(&ms, ctx->ev0, ctx->ev1));
            ctx->cover_ms = ms;
        }
    });
}

int dssg_cover_batch(dssg_ctx *ctx, int64_t n, const int32_t *kind, const int64_t *voff, const double *lat,
                     const double *lng, const float *radius_m, int64_t *out_offs, uint64_t *out_cells,
                     int64_t cells_cap, int64_t *cells_needed, int32_t *status, double *area_km2)
{
    if (!ctx || n < 0 || !cells_needed || !out_offs || !status) return DSSG_ERR_INVALID;
    if (n > 0 && (!kind || !voff || !lat || !lng)) return DSSG_ERR_INVALID;
    int64_t nvtx = n > 0 ? voff[n] : 0;
    if (nvtx < 0) return DSSG_ERR_INVALID;
    int code = DSSG_OK;
    int rc = guarded(ctx, [&] {
        hipStream_t s = ctx->stream;
        const int32_t *dk = upload(ctx->d_kind, kind, n, s);
        const int64_t *dv = upload(ctx->d_voff, voff, n + 1, s);
        const double *dla = upload(ctx->d_lat, lat, nvtx, s);
        const double *dln = upload(ctx->d_lng, lng, nvtx, s);
        std::vector<float> zeros;
        if (!radius_m) zeros.assign((size_t)(n > 0 ? n : 1), 0.0f);
        const float *dr = upload(ctx->d_rad, radius_m ? radius_m : zeros.data(), n, s);
        dssg_cells res;
        ctx->cov_offs = nullptr;  // the engine's buffers are rewritten: no device search may take its cached total
        ctx->cover.run(n, dk, dv, dla, dln, dr, s, &res);
        DSS_HIP(hipMemcpyAsync(out_offs, res.offs, sizeof(int64_t) * (size_t)(n + 1), hipMemcpyDeviceToHost, s));
        if (n > 0) DSS_HIP(hipMemcpyAsync(status, res.status, sizeof(int32_t) * (size_t)n, hipMemcpyDeviceToHost, s));
        if (n > 0 && area_km2)
            DSS_HIP(hipMemcpyAsync(area_km2, res.area_km2, sizeof(double) * (size_t)n, hipMemcpyDeviceToHost, s));
        *cells_needed = res.total_cells;
        if (res.total_cells <= cells_cap && res.total_cells > 0) {
            if (!out_cells) throw dss::Error(DSSG_ERR_INVALID, "out_cells is NULL");
            DSS_HIP(hipMemcpyAsync(out_cells, res.cells, sizeof(uint64_t) * (size_t)res.total_cells, hipMemcpyDeviceToHost, s));
        }
        DSS_HIP(hipStreamSynchronize(s));
        if (res.total_cells > cells_cap) code = DSSG_ERR_CAPACITY;
    });
    return rc ? rc : code;
}

int dssg_union_volumes_device(dssg_ctx *ctx, int64_t nvol, const int64_t *d_vol_offs, const int32_t *d_kind,
                              const int64_t *d_voff, const double *d_lat, const double *d_lng, const float *d_radius_m,
                              const uint8_t *d_has_fp, const float *d_alt_lo, const float *d_alt_hi,
                              const int64_t *d_t0, const int64_t *d_t1, void *stream, dssg_volumes *out)
{
    if (!ctx || !out || nvol < 0 || (nvol > 0 && !d_vol_offs)) return DSSG_ERR_INVALID;
    return guarded(ctx, [&] {
        hipStream_t s = stream ? (hipStream_t)stream : ctx->stream;
        int64_t nx = 0;
        if (nvol > 0) {
            DSS_HIP(hipMemcpyAsync(&nx, d_vol_offs + nvol, sizeof(int64_t), hipMemcpyDeviceToHost, s));
            DSS_HIP(hipStreamSynchronize(s));
        }
        if (nx < 0) throw dss::Error(DSSG_ERR_INVALID, "vol_offs must ascend from 0");
        if (nx > 0 && (!d_kind || !d_voff || !d_lat || !d_lng || !d_radius_m || !d_has_fp || !d_alt_lo || !d_alt_hi ||
                       !d_t0 || !d_t1))
            throw dss::Error(DSSG_ERR_INVALID, "extent arrays are NULL");
        ctx->cov_offs = nullptr;  // the union covers through this context's cover engine
        ctx->ingress.union_volumes(ctx->cover, nvol, d_vol_offs, nx, d_kind, d_voff, d_lat, d_lng, d_radius_m, d_has_fp,
                                   d_alt_lo, d_alt_hi, d_t0, d_t1, s, out);
    });
}

int dssg_area_to_cell_ids(dssg_ctx *ctx, const char *area, uint64_t *out_cells, int64_t cap, int64_t *needed,
                          int32_t *status, double *area_km2)
{
    if (!ctx || !area || !needed || !status) return DSSG_ERR_INVALID;
    *needed = 0;
    if (area_km2) *area_km2 = 0;
    // pkg/geo/s2.go:136-142: count check precedes parsing.
    std::string a(area);
    int64_t num_coords = (int64_t)std::count(a.begin(), a.end(), ',') + 1;
    if (num_coords % 2 == 1) { *status = DSSG_ST_ODD_COORDS; return DSSG_OK; }
    if (num_coords / 2 < 3) { *status = DSSG_ST_NOT_ENOUGH_POINTS; return DSSG_OK; }
    std::vector<double> lat, lng;
    size_t pos = 0;
    int64_t counter = 0;
    double la = 0;
    while (true) {  // bufio.Scanner with splitAtComma
        size_t c = a.find(',', pos);
        std::string tok = trim_space(a.substr(pos, c == std::string::npos ? std::string::npos : c - pos));
        double v;
        if (!go_parse_float(tok, v)) { *status = DSSG_ST_BAD_COORD_SET; return DSSG_OK; }
        if (counter % 2 == 0) la = v;
        else { lat.push_back(la); lng.push_back(v); }
        counter++;
        if (c == std::string::npos) break;
        pos = c + 1;
        if (pos == a.size()) break;  // splitAtComma at EOF with no data left: no empty final token
    }
    int32_t kind = DSSG_KIND_POINTS;
    int64_t voff[2] = {0, (int64_t)lat.size()};
    float r = 0;
    int64_t offs[2];
    double ar = 0;
    int rc = dssg_cover_batch(ctx, 1, &kind, voff, lat.data(), lng.data(), &r, offs, out_cells, cap, needed, status, &ar);
    if (area_km2) *area_km2 = ar;
    return rc;
}

int dssg_index_build_range_device(dssg_ctx *ctx, int64_t n, const int64_t *d_cell_offs, const uint64_t *d_cells,
                                  const float *d_alt_lo, const float *d_alt_hi, const int64_t *d_t0, const int64_t *d_t1,
                                  const int32_t *d_owner, uint64_t cell_lo, uint64_t cell_hi, void *stream,
                                  dssg_index **out)
{
    if (!ctx || !out || n < 0 || !d_cell_offs || (n > 0 && (!d_alt_lo || !d_alt_hi || !d_t0 || !d_t1)) ||
        cell_lo > cell_hi)
        return DSSG_ERR_INVALID;
    *out = nullptr;
    dssg_index *idx = new (std::nothrow) dssg_index();
    if (!idx) return DSSG_ERR_NOMEM;
    idx->device = ctx->device;
    int rc = guarded(ctx, [&] {
        hipStream_t s = stream ? (hipStream_t)stream : ctx->stream;
        ctx->search.build(idx, n, d_cell_offs, d_cells, d_alt_lo, d_alt_hi, d_t0, d_t1, d_owner, cell_lo, cell_hi, s);
    });
    if (rc) {
        delete idx;
        return rc;
    }
    *out = idx;
    return DSSG_OK;
}

int dssg_index_build_device(dssg_ctx *ctx, int64_t n, const int64_t *d_cell_offs, const uint64_t *d_cells,
                            const float *d_alt_lo, const float *d_alt_hi, const int64_t *d_t0, const int64_t *d_t1,
                            const int32_t *d_owner, void *stream, dssg_index **out)
{
    return dssg_index_build_range_device(ctx, n, d_cell_offs, d_cells, d_alt_lo, d_alt_hi, d_t0, d_t1, d_owner, 0,
                                         ~0ull, stream, out);
}

int dssg_index_build_range(dssg_ctx *ctx, int64_t n, const int64_t *cell_offs, const uint64_t *cells,
                           const float *alt_lo, const float *alt_hi, const int64_t *t0, const int64_t *t1,
                           const int32_t *owner, uint64_t cell_lo, uint64_t cell_hi, dssg_index **out)
{
    if (!ctx || !out || n < 0 || !cell_offs) return DSSG_ERR_INVALID;
    *out = nullptr;
    int64_t P = cell_offs[n];
    dss::DevBuf<int64_t> offs, dt0, dt1;
    dss::DevBuf<uint64_t> dc;
    dss::DevBuf<float> dlo, dhi;
    dss::DevBuf<int32_t> down;
    const int64_t *o = nullptr, *a0 = nullptr, *a1 = nullptr;
    const uint64_t *c = nullptr;
    const float *lo = nullptr, *hi = nullptr;
    const int32_t *ow = nullptr;
    int rc = guarded(ctx, [&] {
        hipStream_t s = ctx->stream;
        o = upload(offs, cell_offs, n + 1, s);
        c = upload(dc, cells, P, s);
        lo = upload(dlo, alt_lo, n, s);
        hi = upload(dhi, alt_hi, n, s);
        a0 = upload(dt0, t0, n, s);
        a1 = upload(dt1, t1, n, s);
        if (owner) ow = upload(down, owner, n, s);
        DSS_HIP(hipStreamSynchronize(s));
    });
    if (rc) return rc;
    return dssg_index_build_range_device(ctx, n, o, c, lo, hi, a0, a1, ow, cell_lo, cell_hi, nullptr, out);
}

int dssg_index_build(dssg_ctx *ctx, int64_t n, const int64_t *cell_offs, const uint64_t *cells, const float *alt_lo,
                     const float *alt_hi, const int64_t *t0, const int64_t *t1, const int32_t *owner, dssg_index **out)
{
    return dssg_index_build_range(ctx, n, cell_offs, cells, alt_lo, alt_hi, t0, t1, owner, 0, ~0ull, out);
}

void dssg_index_free(dssg_index *idx)
{
    if (!idx) return;
    (void)hipSetDevice(idx->device);
    delete idx;
}
int64_t dssg_index_num_postings(const dssg_index *idx) { return idx ? idx->n_p : 0; }
int64_t dssg_index_num_cells(const dssg_index *idx) { return idx ? idx->n_cells : 0; }
int32_t dssg_index_grain(const dssg_index *idx) { return idx ? (idx->gshift == 37 ? 12 : 13) : 0; }

int dssg_search_device(dssg_ctx *ctx, const dssg_index *idx, int64_t nq, const int64_t *d_q_offs,
                       const uint64_t *d_q_cells, const float *d_q_alt_lo, const float *d_q_alt_hi,
                       const int64_t *d_q_tlo, const int64_t *d_q_thi, const int32_t *d_q_owner, void *stream,
                       dssg_pairs *out)
{
    if (!ctx || !idx || !out || nq < 0 || (nq > 0 && (!d_q_offs || !d_q_alt_lo || !d_q_alt_hi || !d_q_tlo || !d_q_thi)))
        return DSSG_ERR_INVALID;
    return guarded(ctx, [&] {
        hipStream_t s = stream ? (hipStream_t)stream : ctx->stream;
        if (ctx->timing) {
            if (!ctx->ev0) { DSS_HIP(hipEventCreate(&ctx->ev0)); DSS_HIP(hipEventCreate(&ctx->ev1)); }
            DSS_HIP(hipEventRecord(ctx->ev0, s));
        }
        const int64_t nqc = d_q_offs == ctx->cov_offs && nq == ctx->cov_n ? ctx->cov_total : -1;
        ctx->search.search(idx, nq, d_q_offs, d_q_cells, d_q_alt_lo, d_q_alt_hi, d_q_tlo, d_q_thi, d_q_owner, s, out,
                           nqc);
        if (ctx->timing) {
            DSS_HIP(hipEventRecord(ctx->ev1, s));
            DSS_HIP(hipEventSynchronize(ctx->ev1));
            float ms = 0;
            DSS_HIP(hipEventElapsedTime(&ms, ctx->ev0, ctx->ev1));
            ctx->join_ms = ms;
        }
    });
}

int dssg_search(dssg_ctx *ctx, const dssg_index *idx, int64_t nq, const int64_t *q_offs, const uint64_t *q_cells,
                const float *q_alt_lo, const float *q_alt_hi, const int64_t *q_tlo, const int64_t *q_thi,
                const int32_t *q_owner, uint32_t *out_q, uint32_t *out_e, int64_t cap, int64_t *needed)
{
    if (!ctx || !idx || !needed || nq < 0 || !q_offs) return DSSG_ERR_INVALID;
    if (nq > 0 && (!q_alt_lo || !q_alt_hi || !q_tlo || !q_thi)) return DSSG_ERR_INVALID;
    int code = DSSG_OK;
    int rc = guarded(ctx, [&] {
        for (int64_t q = 0; q < nq; q++)
            if (q_tlo[q] == INT64_MIN) throw dss::Error(DSSG_ERR_INVALID, "query tlo must not be NULL");
        hipStream_t s = ctx->stream;
        const int64_t *dqo = nullptr;
        const uint64_t *dqc = nullptr;
        stage_query_cells(ctx, nq, q_offs, q_cells, s, &dqo, &dqc);
        const float *dlo = upload(ctx->d_alo, q_alt_lo, nq, s);
        const float *dhi = upload(ctx->d_ahi, q_alt_hi, nq, s);
        const int64_t *dtl = upload(ctx->d_tlo, q_tlo, nq, s);
        const int64_t *dth = upload(ctx->d_thi, q_thi, nq, s);
        const int32_t *dow = q_owner ? upload(ctx->d_owner, q_owner, nq, s) : nullptr;
        dssg_pairs res;
        ctx->search.search(idx, nq, dqo, dqc, dlo, dhi, dtl, dth, dow, s, &res);
        *needed = res.n;
        if (res.n > cap) {
            code = DSSG_ERR_CAPACITY;
            return;
        }
        if (res.n > 0) {
            if (!out_q || !out_e) throw dss::Error(DSSG_ERR_INVALID, "output pointers are NULL");
            DSS_HIP(hipMemcpyAsync(out_q, res.q, sizeof(uint32_t) * (size_t)res.n, hipMemcpyDeviceToHost, s));
            DSS_HIP(hipMemcpyAsync(out_e, res.e, sizeof(uint32_t) * (size_t)res.n, hipMemcpyDeviceToHost, s));
            DSS_HIP(hipStreamSynchronize(s));
            sort_pairs_host(out_q, out_e, res.n);
        }
    });
    return rc ? rc : code;
}

int dssg_search_operations(dssg_ctx *ctx, const dssg_index *idx, int64_t nq, const int64_t *q_offs,
                           const uint64_t *q_cells, const float *q_alt_lo, const float *q_alt_hi,
                           const int64_t *q_start, const int64_t *q_end, int64_t now_us, uint32_t *out_q,
                           uint32_t *out_e, int64_t cap, int64_t *needed)
{
    if (nq < 0 || (nq > 0 && (!q_start || !q_end))) return DSSG_ERR_INVALID;
    if (now_us == INT64_MIN) return DSSG_ERR_INVALID;
    // operations.go:398-402: COALESCE(ends_at >= start, true) AND ends_at >= now
    std::vector<int64_t> tlo((size_t)nq), thi((size_t)nq);
    for (int64_t q = 0; q < nq; q++) {
        tlo[q] = std::max(q_start[q], now_us);
        thi[q] = q_end[q];
    }
    return dssg_search(ctx, idx, nq, q_offs, q_cells, q_alt_lo, q_alt_hi, tlo.data(), thi.data(), nullptr, out_q, out_e,
                       cap, needed);
}

int dssg_search_isas(dssg_ctx *ctx, const dssg_index *idx, int64_t nq, const int64_t *q_offs, const uint64_t *q_cells,
                     const int64_t *earliest, const int64_t *latest, uint32_t *out_q, uint32_t *out_e, int64_t cap,
                     int64_t *needed)
{
    if (nq < 0 || (nq > 0 && (!earliest || !latest))) return DSSG_ERR_INVALID;
    // identification_service_area.go:176-180: ends_at >= earliest AND
    // COALESCE(starts_at <= latest, true); no altitude predicate.
    std::vector<float> lo((size_t)nq, -INFINITY), hi((size_t)nq, INFINITY);
    return dssg_search(ctx, idx, nq, q_offs, q_cells, lo.data(), hi.data(), earliest, latest, nullptr, out_q, out_e, cap,
                       needed);
}

int dssg_search_subscriptions(dssg_ctx *ctx, const dssg_index *idx, int64_t nq, const int64_t *q_offs,
                              const uint64_t *q_cells, const int32_t *owner, int64_t now_us, uint32_t *out_q,
                              uint32_t *out_e, int64_t cap, int64_t *needed)
{
    if (nq < 0 || now_us == INT64_MIN) return DSSG_ERR_INVALID;
    // subscriptions.go:229-232,256-260: cells && $1 [AND owner = $2] AND ends_at >= now
    std::vector<float> lo((size_t)nq, -INFINITY), hi((size_t)nq, INFINITY);
    std::vector<int64_t> tlo((size_t)nq, now_us), thi((size_t)nq, INT64_MAX);
    return dssg_search(ctx, idx, nq, q_offs, q_cells, lo.data(), hi.data(), tlo.data(), thi.data(), owner, out_q, out_e,
                       cap, needed);
}

int dssg_route_plan_device(dssg_ctx *ctx, int64_t nq, const int64_t *d_q_offs, const uint64_t *d_q_cells,
                           int32_t nparts, const uint64_t *d_part_hi, void *stream, int64_t *row_counts,
                           int64_t *cell_counts, int64_t *seg_bytes)
{
    if (!ctx || nq < 0 || !d_part_hi || !row_counts || !cell_counts || !seg_bytes || nparts < 1 ||
        nparts > DSSG_MAX_PARTS || (nq > 0 && (!d_q_offs || !d_q_cells)))
        return DSSG_ERR_INVALID;
    return guarded(ctx, [&] {
        hipStream_t s = stream ? (hipStream_t)stream : ctx->stream;
        ctx->route.plan(nq, d_q_offs, d_q_cells, nparts, d_part_hi, s, row_counts, cell_counts, seg_bytes);
    });
}

int dssg_route_fill_device(dssg_ctx *ctx, int64_t nq, const int64_t *d_q_offs, const uint64_t *d_q_cells,
                           const float *d_q_alt_lo, const float *d_q_alt_hi, const int64_t *d_q_tlo,
                           const int64_t *d_q_thi, void *stream, void *d_send)
{
    if (!ctx || nq < 0 || (nq > 0 && (!d_q_offs || !d_q_cells || !d_q_alt_lo || !d_q_alt_hi || !d_q_tlo || !d_q_thi ||
                                      !d_send)))
        return DSSG_ERR_INVALID;
    return guarded(ctx, [&] {
        hipStream_t s = stream ? (hipStream_t)stream : ctx->stream;
        ctx->route.fill(nq, d_q_offs, d_q_cells, d_q_alt_lo, d_q_alt_hi, d_q_tlo, d_q_thi, s, d_send);
    });
}

int dssg_unpack_queries_device(dssg_ctx *ctx, const void *d_recv, int32_t nparts, const int64_t *src_rows,
                               const int64_t *src_cells, void *stream, dssg_batch *out)
{
    if (!ctx || !out || !src_rows || !src_cells || nparts < 1 || nparts > DSSG_MAX_PARTS) return DSSG_ERR_INVALID;
    return guarded(ctx, [&] {
        hipStream_t s = stream ? (hipStream_t)stream : ctx->stream;
        ctx->route.unpack(d_recv, nparts, src_rows, src_cells, s, out);
    });
}

int dssg_route_pairs_plan_device(dssg_ctx *ctx, const dssg_batch *batch, const dssg_pairs *pairs, int32_t nparts,
                                 int32_t self_part, void *stream, int64_t *counts)
{
    if (!ctx || !batch || !pairs || !counts || nparts < 1 || nparts > DSSG_MAX_PARTS || pairs->n < 0 ||
        self_part < -1 || self_part >= nparts)
        return DSSG_ERR_INVALID;
    return guarded(ctx, [&] {
        hipStream_t s = stream ? (hipStream_t)stream : ctx->stream;
        ctx->route.pairs_plan(batch, pairs, nparts, self_part, s, counts);
    });
}

int dssg_route_pairs_fill_device(dssg_ctx *ctx, const dssg_batch *batch, const dssg_pairs *pairs, void *stream,
                                 uint64_t *d_send, uint32_t *d_self_q, uint32_t *d_self_e)
{
    if (!ctx || !batch || !pairs || pairs->n < 0) return DSSG_ERR_INVALID;
    return guarded(ctx, [&] {
        hipStream_t s = stream ? (hipStream_t)stream : ctx->stream;
        ctx->route.pairs_fill(batch, pairs, s, d_send, d_self_q, d_self_e);
    });
}

int dssg_unpack_pairs_device(dssg_ctx *ctx, int64_t n, const uint64_t *d_in, uint32_t *d_q, uint32_t *d_e, void *stream)
{
    if (!ctx || n < 0 || (n > 0 && (!d_in || !d_q || !d_e))) return DSSG_ERR_INVALID;
    return guarded(ctx, [&] {
        hipStream_t s = stream ? (hipStream_t)stream : ctx->stream;
        dss::RouteEngine::split_pairs(n, d_in, d_q, d_e, s);
    });
}

int dssg_index_set_notification_index(dssg_ctx *ctx, dssg_index *idx, const int64_t *values)
{
    if (!ctx || !idx || (idx->n_e > 0 && !values)) return DSSG_ERR_INVALID;
    return guarded(ctx, [&] {
        if (idx->n_e > 0)
            DSS_HIP(hipMemcpy(idx->e_notify.p, values, sizeof(int64_t) * (size_t)idx->n_e, hipMemcpyHostToDevice));
    });
}

int dssg_index_get_notification_index(dssg_ctx *ctx, const dssg_index *idx, int64_t *values)
{
    if (!ctx || !idx || (idx->n_e > 0 && !values)) return DSSG_ERR_INVALID;
    return guarded(ctx, [&] {
        if (idx->n_e > 0)
            DSS_HIP(hipMemcpy(values, idx->e_notify.p, sizeof(int64_t) * (size_t)idx->n_e, hipMemcpyDeviceToHost));
    });
}

int dssg_notify_subscriptions(dssg_ctx *ctx, dssg_index *idx, int64_t nq, const int64_t *q_offs, const uint64_t *q_cells,
                              int64_t now_us, uint32_t *out_q, uint32_t *out_e, int64_t *out_index, int64_t cap,
                              int64_t *needed)
{
    if (!ctx || !idx || !needed || nq < 0 || !q_offs || now_us == INT64_MIN) return DSSG_ERR_INVALID;
    int code = DSSG_OK;
    int rc = guarded(ctx, [&] {
        hipStream_t s = ctx->stream;
        const int64_t *dqo = nullptr;
        const uint64_t *dqc = nullptr;
        stage_query_cells(ctx, nq, q_offs, q_cells, s, &dqo, &dqc);
        // RID subscriptions.go:207-212 / SCD subscriptions.go:133-170:
        // cells overlap AND ends_at >= now; no altitude or start predicate
        std::vector<float> lo((size_t)nq + 1, -INFINITY), hi((size_t)nq + 1, INFINITY);
        std::vector<int64_t> tlo((size_t)nq + 1, now_us), thi((size_t)nq + 1, INT64_MAX);
        const float *dlo = upload(ctx->d_alo, lo.data(), nq, s);
        const float *dhi = upload(ctx->d_ahi, hi.data(), nq, s);
        const int64_t *dtl = upload(ctx->d_tlo, tlo.data(), nq, s);
        const int64_t *dth = upload(ctx->d_thi, thi.data(), nq, s);
        dssg_pairs res;
        ctx->search.search(idx, nq, dqo, dqc, dlo, dhi, dtl, dth, nullptr, s, &res);
        *needed = res.n;
        if (res.n > cap) {  // no counter moves unless the caller can take the rows
            code = DSSG_ERR_CAPACITY;
            return;
        }
        if (res.n > 0 && (!out_q || !out_e || !out_index)) throw dss::Error(DSSG_ERR_INVALID, "output pointers are NULL");
        uint32_t *dq, *de;
        int64_t *dv;
        ctx->subs.notify(idx, &res, s, &dq, &de, &dv);
        if (res.n > 0) {
            DSS_HIP(hipMemcpyAsync(out_q, dq, sizeof(uint32_t) * (size_t)res.n, hipMemcpyDeviceToHost, s));
            DSS_HIP(hipMemcpyAsync(out_e, de, sizeof(uint32_t) * (size_t)res.n, hipMemcpyDeviceToHost, s));
            DSS_HIP(hipMemcpyAsync(out_index, dv, sizeof(int64_t) * (size_t)res.n, hipMemcpyDeviceToHost, s));
        }
        DSS_HIP(hipStreamSynchronize(s));
    });
    return rc ? rc : code;
}

int dssg_owner_subscriptions(dssg_ctx *ctx, const dssg_index *idx, int64_t nq, const int32_t *owner, int64_t now_us,
                             uint32_t *out_q, uint32_t *out_e, int64_t cap, int64_t *needed)
{
    if (!ctx || !idx || !needed || nq < 0 || (nq > 0 && !owner) || now_us == INT64_MIN) return DSSG_ERR_INVALID;
    int code = DSSG_OK;
    int rc = guarded(ctx, [&] {
        hipStream_t s = ctx->stream;
        const int32_t *dow = upload(ctx->d_owner, owner, nq, s);
        uint32_t *dq, *de;
        const int64_t n = ctx->subs.owner_subs(idx, nq, dow, now_us, s, &dq, &de);
        *needed = n;
        if (n > cap) {
            code = DSSG_ERR_CAPACITY;
            return;
        }
        if (n > 0) {
            if (!out_q || !out_e) throw dss::Error(DSSG_ERR_INVALID, "output pointers are NULL");
            DSS_HIP(hipMemcpyAsync(out_q, dq, sizeof(uint32_t) * (size_t)n, hipMemcpyDeviceToHost, s));
            DSS_HIP(hipMemcpyAsync(out_e, de, sizeof(uint32_t) * (size_t)n, hipMemcpyDeviceToHost, s));
            DSS_HIP(hipStreamSynchronize(s));
        }
    });
    return rc ? rc : code;
}

int dssg_max_subscription_count(dssg_ctx *ctx, const dssg_index *idx, int64_t nq, const int64_t *q_offs,
                                const uint64_t *q_cells, const int32_t *owner, int64_t now_us, int64_t *out_count)
{
    if (!ctx || !idx || nq < 0 || !q_offs || (nq > 0 && (!owner || !out_count)) || now_us == INT64_MIN)
        return DSSG_ERR_INVALID;
    return guarded(ctx, [&] {
        hipStream_t s = ctx->stream;
        const int64_t nqc = q_offs[nq] - q_offs[0];
        if (nqc < 0 || q_offs[0] != 0) throw dss::Error(DSSG_ERR_INVALID, "q_offs must start at 0 and ascend");
        const int64_t *dqo = upload(ctx->d_qoffs, q_offs, nq + 1, s);
        const uint64_t *dqc = upload(ctx->d_cells, q_cells, nqc, s);
        const int32_t *dow = upload(ctx->d_owner, owner, nq, s);
        ctx->subs.max_count(&idx, 1, nq, dqo, dqc, nqc, dow, now_us, s, out_count);
    });
}

struct dssg_store {
    dss::Store st;
    dssg_store(int device, bool owner) : st(device, owner) {}
};

int dssg_store_create(dssg_ctx *ctx, int32_t with_owner, dssg_store **out)
{
    if (!ctx || !out) return DSSG_ERR_INVALID;
    *out = new (std::nothrow) dssg_store(ctx->device, with_owner != 0);
    return *out ? DSSG_OK : DSSG_ERR_NOMEM;
}

void dssg_store_free(dssg_store *st)
{
    if (!st) return;
    delete st;
}

int dssg_store_upsert(dssg_ctx *ctx, dssg_store *st, int64_t n, const uint32_t *ids, const int64_t *cell_offs,
                      const uint64_t *cells, const float *alt_lo, const float *alt_hi, const int64_t *t0,
                      const int64_t *t1, const int32_t *owner)
{
    if (!ctx || !st || n < 0 || (n > 0 && (!ids || !cell_offs || !alt_lo || !alt_hi || !t0 || !t1)) ||
        (n > 0 && cell_offs[n] > 0 && !cells))
        return DSSG_ERR_INVALID;
    return guarded(ctx, [&] {
        st->st.upsert(ctx->search, n, ids, cell_offs, cells, alt_lo, alt_hi, t0, t1, owner, ctx->stream);
    });
}

int dssg_store_delete(dssg_ctx *ctx, dssg_store *st, int64_t n, const uint32_t *ids, int32_t *found)
{
    if (!ctx || !st || n < 0 || (n > 0 && !ids)) return DSSG_ERR_INVALID;
    return guarded(ctx, [&] { st->st.remove(ctx->search, n, ids, found, ctx->stream); });
}

int dssg_store_compact(dssg_ctx *ctx, dssg_store *st)
{
    if (!ctx || !st) return DSSG_ERR_INVALID;
    return guarded(ctx, [&] { st->st.compact(ctx->search, ctx->stream); });
}

int dssg_store_stats(const dssg_store *st, int64_t *live, int64_t *base, int64_t *delta, int64_t *compactions)
{
    if (!st) return DSSG_ERR_INVALID;
    if (live) *live = st->st.live();
    if (base) *base = st->st.base_size();
    if (delta) *delta = st->st.delta_size();
    if (compactions) *compactions = st->st.compactions();
    return DSSG_OK;
}

int dssg_store_max_subscription_count(dssg_ctx *ctx, dssg_store *st, int64_t nq, const int64_t *q_offs,
                                      const uint64_t *q_cells, const int32_t *owner, int64_t now_us,
                                      int64_t *out_count)
{
    if (!ctx || !st || nq < 0 || !q_offs || (nq > 0 && (!owner || !out_count)) || now_us == INT64_MIN)
        return DSSG_ERR_INVALID;
    return guarded(ctx, [&] {
        if (!st->st.with_owner()) throw dss::Error(DSSG_ERR_INVALID, "store created without owners");
        hipStream_t s = ctx->stream;
        const int64_t nqc = q_offs[nq] - q_offs[0];
        if (nqc < 0 || q_offs[0] != 0) throw dss::Error(DSSG_ERR_INVALID, "q_offs must start at 0 and ascend");
        const int64_t *dqo = upload(ctx->d_qoffs, q_offs, nq + 1, s);
        const uint64_t *dqc = upload(ctx->d_cells, q_cells, nqc, s);
        const int32_t *dow = upload(ctx->d_owner, owner, nq, s);
        const dssg_index *sides[2] = {st->st.base(), st->st.delta()};
        ctx->subs.max_count(sides, 2, nq, dqo, dqc, nqc, dow, now_us, s, out_count);
    });
}

int dssg_store_search(dssg_ctx *ctx, dssg_store *st, int64_t nq, const int64_t *q_offs, const uint64_t *q_cells,
                      const float *q_alt_lo, const float *q_alt_hi, const int64_t *q_tlo, const int64_t *q_thi,
                      const int32_t *q_owner, uint32_t *out_q, uint32_t *out_id, int64_t cap, int64_t *needed)
{
    if (!ctx || !st || !needed || nq < 0 || !q_offs || (nq > 0 && (!q_alt_lo || !q_alt_hi || !q_tlo || !q_thi)))
        return DSSG_ERR_INVALID;
    int code = DSSG_OK;
    int rc = guarded(ctx, [&] {
        for (int64_t q = 0; q < nq; q++)
            if (q_tlo[q] == INT64_MIN) throw dss::Error(DSSG_ERR_INVALID, "query tlo must not be NULL");
        hipStream_t s = ctx->stream;
        const int64_t *dqo = nullptr;
        const uint64_t *dqc = nullptr;
        stage_query_cells(ctx, nq, q_offs, q_cells, s, &dqo, &dqc);
        const float *dlo = upload(ctx->d_alo, q_alt_lo, nq, s);
        const float *dhi = upload(ctx->d_ahi, q_alt_hi, nq, s);
        const int64_t *dtl = upload(ctx->d_tlo, q_tlo, nq, s);
        const int64_t *dth = upload(ctx->d_thi, q_thi, nq, s);
        const int32_t *dow = q_owner ? upload(ctx->d_owner, q_owner, nq, s) : nullptr;
        std::vector<uint64_t> res;
        const int64_t n = st->st.search(ctx->search, nq, dqo, dqc, dlo, dhi, dtl, dth, dow, s, res);
        *needed = n;
        if (n > cap) {
            code = DSSG_ERR_CAPACITY;
            return;
        }
        if (n > 0 && (!out_q || !out_id)) throw dss::Error(DSSG_ERR_INVALID, "output pointers are NULL");
        for (int64_t i = 0; i < n; i++) {
            out_q[i] = (uint32_t)(res[i] >> 32);
            out_id[i] = (uint32_t)res[i];
        }
    });
    return rc ? rc : code;
}

int dssg_search_stats_device(dssg_ctx *ctx, const dssg_index *idx, int64_t nq, const int64_t *d_q_offs,
                             const uint64_t *d_q_cells, void *stream, int64_t *matched, int64_t *distinct)
{
    if (!ctx || !idx || nq < 0 || !matched || !distinct || (nq > 0 && !d_q_offs)) return DSSG_ERR_INVALID;
    return guarded(ctx, [&] {
        hipStream_t s = stream ? (hipStream_t)stream : ctx->stream;
        ctx->search.stats(idx, nq, d_q_offs, d_q_cells, s, matched, distinct);
    });
}

int dssg_search_touched_device(dssg_ctx *ctx, const dssg_index *idx, int64_t nq, const int64_t *d_q_offs,
                               const uint64_t *d_q_cells, void *stream, int64_t *touched)
{
    if (!ctx || !idx || nq < 0 || !touched || (nq > 0 && !d_q_offs)) return DSSG_ERR_INVALID;
    return guarded(ctx, [&] {
        hipStream_t s = stream ? (hipStream_t)stream : ctx->stream;
        *touched = ctx->search.touched(idx, nq, d_q_offs, d_q_cells, s);
    });
}

int dssg_index_info(const dssg_index *idx, int64_t *postings, int64_t *cells, int64_t *long_duration,
                    int64_t *long_footprint, int64_t *max_cell_postings, int64_t *dcap_us)
{
    if (!idx) return DSSG_ERR_INVALID;
    if (postings) *postings = idx->n_p;
    if (cells) *cells = idx->n_cells;
    if (long_duration) *long_duration = idx->n_long;
    if (long_footprint) *long_footprint = idx->n_long_fp;
    if (max_cell_postings) *max_cell_postings = idx->max_cell_postings;
    if (dcap_us) *dcap_us = idx->dcap;
    return DSSG_OK;
}

int dssg_copy_device(dssg_ctx *ctx, void *dst, const void *src, size_t bytes, void *stream)
{
    if (!ctx || (bytes && (!dst || !src))) return DSSG_ERR_INVALID;
    return guarded(ctx, [&] {
        hipStream_t s = stream ? (hipStream_t)stream : ctx->stream;
        dss::device_copy(dst, src, bytes, s);
    });
}

int dssg_copy_to_host(dssg_ctx *ctx, void *dst, const void *src, size_t bytes)
{
    if (!ctx || (bytes && (!dst || !src))) return DSSG_ERR_INVALID;
    return guarded(ctx, [&] {
        if (bytes) DSS_HIP(hipMemcpy(dst, src, bytes, hipMemcpyDeviceToHost));
    });
}

int dssg_radix_sort_device(dssg_ctx *ctx, int key_bytes, int64_t n, int bits, const void *d_keys_in, void *d_keys_out,
                           const uint32_t *d_vals_in, uint32_t *d_vals_out, void *stream, double *ms)
{
    if (!ctx || n < 0 || (key_bytes != 4 && key_bytes != 8) || bits < 0 || bits > 8 * key_bytes) return DSSG_ERR_INVALID;
    if (n > 0 && (!d_keys_in || !d_keys_out || d_keys_in == d_keys_out || (!d_vals_in) != (!d_vals_out) ||
                  (d_vals_in && d_vals_in == d_vals_out)))
        return DSSG_ERR_INVALID;
    if (key_bytes == 4 && !d_vals_in) return DSSG_ERR_INVALID;  // 32-bit keys are sorted with values only
    return guarded(ctx, [&] {
        hipStream_t s = stream ? (hipStream_t)stream : ctx->stream;
        hipEvent_t e0 = nullptr, e1 = nullptr;
        if (ms) {
            DSS_HIP(hipEventCreate(&e0));
            DSS_HIP(hipEventCreate(&e1));
            DSS_HIP(hipEventRecord(e0, s));
        }
        if (key_bytes == 8 && d_vals_in)  // (packed 8-B words when the keys' constant low bits hold the values)
            dss::radix_sort_pairs_packed((const uint64_t *)d_keys_in, (uint64_t *)d_keys_out, d_vals_in, d_vals_out, n,
                                         bits, ctx->sort_tmp, s);
        else if (key_bytes == 8)
            dss::radix_sort_keys((const unsigned long *)d_keys_in, (unsigned long *)d_keys_out, n, bits, ctx->sort_tmp, s);
        else
            dss::radix_sort_pairs((const uint32_t *)d_keys_in, (uint32_t *)d_keys_out, d_vals_in, d_vals_out, n, bits,
                                  ctx->sort_tmp, s);
        if (ms) {
            DSS_HIP(hipEventRecord(e1, s));
            DSS_HIP(hipEventSynchronize(e1));
            float f = 0;
            DSS_HIP(hipEventElapsedTime(&f, e0, e1));
            *ms = f;
            (void)hipEventDestroy(e0);
            (void)hipEventDestroy(e1);
        }
    });
}

int dssg_selftest_math(dssg_ctx *ctx, int op, int64_t n, const double *x, const double *y, double *out)
{
    if (!ctx || n < 0 || (n > 0 && (!x || !out))) return DSSG_ERR_INVALID;
    return guarded(ctx, [&] {
        if (n) dss::selftest_math(op, n, x, y, out, ctx->stream);
    });
}

int dssg_selftest_scan(dssg_ctx *ctx, int64_t n, int shift, const int64_t *in, int64_t *out)
{
    if (!ctx || n < 0 || shift < 0 || shift > 64 || !out || (n > 0 && !in)) return DSSG_ERR_INVALID;
    return guarded(ctx, [&] { dss::selftest_scan(n, shift, in, out, ctx->stream); });
}

}  // extern "C"

/* ======================================================================
 * Native multi-GPU exchange over RCCL (the range partition
 * of scd_cells_operations, pkg/scd/store/cockroach/store.go:140-147).
 * RCCL is opened with dlopen(RTLD_LOCAL) on first use, so the library loads
 * without it and never shares symbols with another RCCL in the process
 * (PyTorch bundles its own).
 * ====================================================================== */
namespace {

struct Rccl {
    bool tried = false, ok = false;
    std::string err;
    decltype(&ncclGetUniqueId) getUniqueId = nullptr;
    decltype(&ncclCommInitRank) commInitRank = nullptr;
    decltype(&ncclCommDestroy) commDestroy = nullptr;
    decltype(&ncclAllGather) allGather = nullptr;
    decltype(&ncclSend) send = nullptr;
    decltype(&ncclRecv) recv = nullptr;
    decltype(&ncclGroupStart) groupStart = nullptr;
    decltype(&ncclGroupEnd) groupEnd = nullptr;
    decltype(&ncclGetErrorString) errorString = nullptr;
};

Rccl &rccl()
{
    static Rccl r;
    static std::once_flag once;
    std::call_once(once, [] {
        void *h = nullptr;
        for (const char *name : {"librccl.so.1", "/opt/rocm/lib/librccl.so.1", "librccl.so"}) {
            h = dlopen(name, RTLD_NOW | RTLD_LOCAL);
            if (h) break;
        }
        if (!h) {
            const char *e = dlerror();
            r.err = std::string("cannot open librccl: ") + (e ? e : "?");
            return;
        }
        bool all = true;
        auto sym = [&](auto &fn, const char *name) {
            fn = reinterpret_cast<std::remove_reference_t<decltype(fn)>>(dlsym(h, name));
            if (!fn) all = false;
        };
        sym(r.getUniqueId, "ncclGetUniqueId");
        sym(r.commInitRank, "ncclCommInitRank");
        sym(r.commDestroy, "ncclCommDestroy");
        sym(r.allGather, "ncclAllGather");
        sym(r.send, "ncclSend");
        sym(r.recv, "ncclRecv");
        sym(r.groupStart, "ncclGroupStart");
        sym(r.groupEnd, "ncclGroupEnd");
        sym(r.errorString, "ncclGetErrorString");
        r.ok = all;
        if (!all) r.err = "librccl lacks an expected symbol";
    });
    return r;
}

void nccl_check(ncclResult_t rc, const char *what)
{
    if (rc != ncclSuccess)
        throw dss::Error(DSSG_ERR_DEVICE, std::string(what) + ": " + rccl().errorString(rc));
}

}  // namespace

struct dssg_comm {
    ncclComm_t comm = nullptr;
    int nranks = 0, rank = 0, device = 0;
    dss::DevBuf<int64_t> d_counts;                 // allgathered count vectors
    int64_t *h_counts = nullptr;                   // pinned: their host copy
    dss::DevBuf<unsigned char> send_q, recv_q;     // fused query segments
    // pairs home, two buffer sets used alternately: with an exchange stream
    // step k's pairs are still in flight while step k+1 fills the other set
    dss::DevBuf<uint64_t> send_pairs[2], recv_pairs[2];  // packed pairs of the other ranks' queries
    dss::DevBuf<uint32_t> out_q[2], out_e[2];
    int flip = 0;
    hipEvent_t ev_fill = nullptr;  // pairs packed on the step's stream -> the exchange stream may send them
    ~dssg_comm()
    {
        if (ev_fill) (void)hipEventDestroy(ev_fill);
        if (h_counts) (void)hipHostFree(h_counts);
    }
};

namespace {

// Every rank's k-vector of int64 counts -> all[s * k + j] = rank s's j-th
// (host, pinned: no staging copy).
const int64_t *allgather_counts(dssg_comm *c, const int64_t *mine, int k, hipStream_t s)
{
    const size_t words = (size_t)k * (c->nranks + 1);
    int64_t *d = c->d_counts.ensure(words);
    if (!c->h_counts) DSS_HIP(hipHostMalloc((void **)&c->h_counts, sizeof(int64_t) * 2 * DSSG_MAX_PARTS *
                                                                       (DSSG_MAX_PARTS + 1), hipHostMallocDefault));
    int64_t *h = c->h_counts;
    std::memcpy(h + (size_t)k * c->nranks, mine, sizeof(int64_t) * k);
    DSS_HIP(hipMemcpyAsync(d + (size_t)k * c->nranks, h + (size_t)k * c->nranks, sizeof(int64_t) * k,
                           hipMemcpyHostToDevice, s));
    nccl_check(rccl().allGather(d + (size_t)k * c->nranks, d, (size_t)k * sizeof(int64_t), ncclChar, c->comm, s),
               "ncclAllGather");
    DSS_HIP(hipMemcpyAsync(h, d, sizeof(int64_t) * (size_t)k * c->nranks, hipMemcpyDeviceToHost, s));
    DSS_HIP(hipStreamSynchronize(s));
    return h;
}

// Grouped point-to-point all-to-all of byte blocks at explicit offsets; the
// caller's own block (p == rank) is not sent (it is copied, or used in place).
void alltoallv(dssg_comm *c, const void *send, const int64_t *soff, const int64_t *sbytes, void *recv,
               const int64_t *roff, const int64_t *rbytes, hipStream_t s)
{
    Rccl &r = rccl();
    nccl_check(r.groupStart(), "ncclGroupStart");
    for (int p = 0; p < c->nranks; p++) {
        if (p == c->rank) continue;
        if (sbytes[p] > 0)
            nccl_check(r.send((const char *)send + soff[p], (size_t)sbytes[p], ncclChar, p, c->comm, s), "ncclSend");
        if (rbytes[p] > 0)
            nccl_check(r.recv((char *)recv + roff[p], (size_t)rbytes[p], ncclChar, p, c->comm, s), "ncclRecv");
    }
    nccl_check(r.groupEnd(), "ncclGroupEnd");
}

}  // namespace

int dssg_comm_unique_id(uint8_t *id)
{
    if (!id) return DSSG_ERR_INVALID;
    Rccl &r = rccl();
    if (!r.ok) return DSSG_ERR_DEVICE;
    ncclUniqueId u;
    if (r.getUniqueId(&u) != ncclSuccess) return DSSG_ERR_DEVICE;
    static_assert(sizeof(u) == DSSG_COMM_ID_BYTES, "ncclUniqueId size");
    std::memcpy(id, &u, sizeof(u));
    return DSSG_OK;
}

int dssg_comm_init(dssg_ctx *ctx, int32_t nranks, int32_t rank, const uint8_t *id, dssg_comm **out)
{
    if (!ctx || !id || !out || nranks < 1 || nranks > DSSG_MAX_PARTS || rank < 0 || rank >= nranks)
        return DSSG_ERR_INVALID;
    return guarded(ctx, [&] {
        Rccl &r = rccl();
        if (!r.ok) throw dss::Error(DSSG_ERR_DEVICE, r.err);
        ncclUniqueId u;
        std::memcpy(&u, id, sizeof(u));
        auto *c = new dssg_comm();
        c->nranks = nranks;
        c->rank = rank;
        c->device = ctx->device;
        const ncclResult_t rc = r.commInitRank(&c->comm, nranks, u, rank);
        if (rc != ncclSuccess) {
            delete c;
            nccl_check(rc, "ncclCommInitRank");
        }
        *out = c;
    });
}

void dssg_comm_free(dssg_comm *comm)
{
    if (!comm) return;
    (void)hipSetDevice(comm->device);
    if (comm->comm) rccl().commDestroy(comm->comm);
    delete comm;
}

int dssg_comm_alltoallv_device(dssg_ctx *ctx, dssg_comm *comm, const void *d_send, const int64_t *send_bytes,
                               void *d_recv, const int64_t *recv_bytes, void *stream)
{
    if (!ctx || !comm || !send_bytes || !recv_bytes) return DSSG_ERR_INVALID;
    return guarded(ctx, [&] {
        hipStream_t s = stream ? (hipStream_t)stream : ctx->stream;
        int64_t so[DSSG_MAX_PARTS], ro[DSSG_MAX_PARTS], a = 0, b = 0;
        for (int p = 0; p < comm->nranks; p++) {
            so[p] = a;
            ro[p] = b;
            a += send_bytes[p];
            b += recv_bytes[p];
        }
        const int me = comm->rank;
        if (send_bytes[me] != recv_bytes[me]) throw dss::Error(DSSG_ERR_INVALID, "alltoallv: own block sizes differ");
        if (send_bytes[me] > 0) dss::device_copy((char *)d_recv + ro[me], (const char *)d_send + so[me], send_bytes[me], s);
        alltoallv(comm, d_send, so, send_bytes, d_recv, ro, recv_bytes, s);
    });
}

namespace {

// Phase events of an instrumented sharded step (timing on): on the step's
// stream route | query exchange | join | pairs packed, on the exchange stream
// the pairs' count exchange + all-to-all + split.
enum { kShRoute0, kShRoute1, kShXq1, kShJoin1, kShPack1, kShXp0, kShXp1, kShEvents };

void sharded_step(dssg_ctx *ctx, dssg_comm *cq, dssg_comm *cx, const dssg_index *shard, const uint64_t *d_part_hi,
                  int64_t nq, const int64_t *d_q_offs, const uint64_t *d_q_cells, const float *d_q_alt_lo,
                  const float *d_q_alt_hi, const int64_t *d_q_tlo, const int64_t *d_q_thi, hipStream_t s,
                  hipStream_t x, dssg_pairs *out)
{
    const int W = cq->nranks, me = cq->rank;
    if (cx->nranks != W || cx->rank != me) throw dss::Error(DSSG_ERR_INVALID, "sharded step: communicators differ");
    // a shard joins up to W * nq routed rows in one search (2^25 queries per call)
    if ((int64_t)W * nq >= ((int64_t)1 << 25))
        throw dss::Error(DSSG_ERR_INVALID, "sharded step: nranks x nq must stay below 2^25 routed rows per shard");
    dss::ShardStats &st = ctx->shard_stats;
    st = dss::ShardStats{};
    hipEvent_t *ev = ctx->shard_ev;
    const bool timing = ctx->timing;
    if (timing && !ev[0])
        for (int k = 0; k < kShEvents; k++) DSS_HIP(hipEventCreate(&ev[k]));
    auto mark = [&](int k, hipStream_t on) {
        if (timing) DSS_HIP(hipEventRecord(ev[k], on));
    };
    mark(kShRoute0, s);
    if (W == 1 && ctx->route_identity) {
        // one part owns every cell: routing is the identity, the batch
        // is joined as given (no copies, no collectives)
        const int64_t nqc = d_q_offs == ctx->cov_offs && nq == ctx->cov_n ? ctx->cov_total : -1;
        ctx->search.search(shard, nq, d_q_offs, d_q_cells, d_q_alt_lo, d_q_alt_hi, d_q_tlo, d_q_thi, nullptr, s, out, nqc);
        if (x != s) {
            // async: like every routed step, the output lives in the buffer
            // set of this step (valid until the second next call) -- the
            // engine's result buffers are swapped into it, no copy
            const int b = cx->flip;
            cx->flip ^= 1;
            if (!ctx->search.adopt_output(*out, cx->out_q[b], cx->out_e[b])) {
                uint32_t *q = cx->out_q[b].ensure((size_t)out->n + 1), *e = cx->out_e[b].ensure((size_t)out->n + 1);
                dss::device_copy(q, out->q, sizeof(uint32_t) * (size_t)out->n, s);
                dss::device_copy(e, out->e, sizeof(uint32_t) * (size_t)out->n, s);
                out->q = q;
                out->e = e;
            }
        }
        out->n_tagged = 0;
        st.join_ms = -1;
        return;
    }
    // (1) route this rank's queries to the parts owning their cells: one
    // fused segment [rows | cells] per part
    int64_t rows_n[DSSG_MAX_PARTS], cells_n[DSSG_MAX_PARTS], seg[DSSG_MAX_PARTS];
    ctx->route.plan(nq, d_q_offs, d_q_cells, W, d_part_hi, s, rows_n, cells_n, seg);
    int64_t so[DSSG_MAX_PARTS], stot = 0;
    for (int p = 0; p < W; p++) {
        so[p] = stot;
        stot += seg[p];
    }
    unsigned char *sq = cq->send_q.ensure((size_t)stot + 32);
    ctx->route.fill(nq, d_q_offs, d_q_cells, d_q_alt_lo, d_q_alt_hi, d_q_tlo, d_q_thi, s, sq);
    mark(kShRoute1, s);
    // (2) one count exchange, one all-to-all of the segments (own segment copied)
    int64_t mine[2 * DSSG_MAX_PARTS];
    for (int p = 0; p < W; p++) {
        mine[p] = rows_n[p];
        mine[W + p] = cells_n[p];
    }
    const int64_t *cnt = allgather_counts(cq, mine, 2 * W, s);
    int64_t src_rows[DSSG_MAX_PARTS], src_cells[DSSG_MAX_PARTS], rb[DSSG_MAX_PARTS], ro[DSSG_MAX_PARTS], rtot = 0;
    int64_t ncells_recv = 0;
    for (int p = 0; p < W; p++) {
        src_rows[p] = cnt[(size_t)p * 2 * W + me];
        src_cells[p] = cnt[(size_t)p * 2 * W + W + me];
        ncells_recv += src_cells[p];
        rb[p] = dss::route_segment_bytes(src_rows[p], src_cells[p]);
        ro[p] = rtot;
        rtot += rb[p];
    }
    unsigned char *rq = cq->recv_q.ensure((size_t)rtot + 32);
    if (seg[me] > 0) dss::device_copy(rq + ro[me], sq + so[me], (size_t)seg[me], s);
    alltoallv(cq, sq, so, seg, rq, ro, rb, s);
    st.q_bytes_sent = stot - seg[me];
    st.q_bytes_recv = rtot - rb[me];
    // (3) the received queries against this rank's shard
    dssg_batch batch{};
    ctx->route.unpack(rq, W, src_rows, src_cells, s, &batch);
    mark(kShXq1, s);
    dssg_pairs pairs{};
    ctx->search.search(shard, batch.n, batch.offs, batch.cells, batch.alt_lo, batch.alt_hi, batch.tlo, batch.thi,
                       nullptr, s, &pairs);
    mark(kShJoin1, s);
    st.rows = batch.n;
    st.cells = ncells_recv;
    st.shard_pairs = pairs.n;
    // (4) pairs home: this rank's own straight into its output, the others'
    // packed (home-local query << 32 | entity) and all-to-all'd -- on the
    // exchange stream x, into the buffer set not used by the previous step
    // (whose pairs may still be in flight there)
    int64_t pn[DSSG_MAX_PARTS];
    ctx->route.pairs_plan(&batch, &pairs, W, me, s, pn);
    mark(kShXp0, x);
    const int64_t *pc = allgather_counts(cx, pn, W, x);  // waits for x: the previous step's pairs have landed
    int64_t psb[DSSG_MAX_PARTS], pso[DSSG_MAX_PARTS], prb[DSSG_MAX_PARTS], pro[DSSG_MAX_PARTS], ps = 0, pr = 0;
    for (int p = 0; p < W; p++) {
        psb[p] = p == me ? 0 : pn[p] * (int64_t)sizeof(uint64_t);
        pso[p] = ps;
        ps += psb[p];
        prb[p] = p == me ? 0 : pc[(size_t)p * W + me] * (int64_t)sizeof(uint64_t);
        pro[p] = pr;
        pr += prb[p];
    }
    const int64_t nself = pn[me], nrecv = pr / (int64_t)sizeof(uint64_t);
    const int b = cx->flip;
    cx->flip ^= 1;
    uint64_t *spairs = cx->send_pairs[b].ensure((size_t)ps / sizeof(uint64_t) + 1);
    uint32_t *q = cx->out_q[b].ensure((size_t)(nself + nrecv) + 1), *e = cx->out_e[b].ensure((size_t)(nself + nrecv) + 1);
    uint64_t *rpairs = cx->recv_pairs[b].ensure((size_t)nrecv + 1);
    ctx->route.pairs_fill(&batch, &pairs, s, spairs, q, e);
    mark(kShPack1, s);
    if (x != s) {
        if (!cx->ev_fill) DSS_HIP(hipEventCreateWithFlags(&cx->ev_fill, hipEventDisableTiming));
        DSS_HIP(hipEventRecord(cx->ev_fill, s));
        DSS_HIP(hipStreamWaitEvent(x, cx->ev_fill, 0));
    }
    alltoallv(cx, spairs, pso, psb, rpairs, pro, prb, x);
    dss::RouteEngine::split_pairs(nrecv, rpairs, q + nself, e + nself, x);
    mark(kShXp1, x);
    st.p_bytes_sent = ps;
    st.p_bytes_recv = pr;
    out->q = q;
    out->e = e;
    out->n = nself + nrecv;
    out->n_tagged = 0;
    if (timing) {
        DSS_HIP(hipStreamSynchronize(x));
        DSS_HIP(hipStreamSynchronize(s));
        auto el = [&](int a, int z) {
            float ms = 0;
            DSS_HIP(hipEventElapsedTime(&ms, ev[a], ev[z]));
            return (double)ms;
        };
        st.route_ms = el(kShRoute0, kShRoute1);
        st.xq_ms = el(kShRoute1, kShXq1);
        st.join_ms = el(kShXq1, kShJoin1);
        st.pack_ms = el(kShJoin1, kShPack1);
        st.xp_ms = el(kShXp0, kShXp1);
        // roofline accounting: postings of the distinct cells this shard was asked for
        st.touched = ctx->search.touched(shard, batch.n, batch.offs, batch.cells, s);
    }
}

}  // namespace

int dssg_sharded_search_device(dssg_ctx *ctx, dssg_comm *comm, const dssg_index *shard, const uint64_t *d_part_hi,
                               int64_t nq, const int64_t *d_q_offs, const uint64_t *d_q_cells,
                               const float *d_q_alt_lo, const float *d_q_alt_hi, const int64_t *d_q_tlo,
                               const int64_t *d_q_thi, void *stream, dssg_pairs *out)
{
    if (!ctx || !comm || !shard || !d_part_hi || !out || nq < 0 ||
        (nq > 0 && (!d_q_offs || !d_q_cells || !d_q_alt_lo || !d_q_alt_hi || !d_q_tlo || !d_q_thi)))
        return DSSG_ERR_INVALID;
    return guarded(ctx, [&] {
        hipStream_t s = stream ? (hipStream_t)stream : ctx->stream;
        sharded_step(ctx, comm, comm, shard, d_part_hi, nq, d_q_offs, d_q_cells, d_q_alt_lo, d_q_alt_hi, d_q_tlo,
                     d_q_thi, s, s, out);
        DSS_HIP(hipStreamSynchronize(s));
    });
}

int dssg_sharded_search_async_device(dssg_ctx *ctx, dssg_comm *comm, dssg_comm *xcomm, const dssg_index *shard,
                                     const uint64_t *d_part_hi, int64_t nq, const int64_t *d_q_offs,
                                     const uint64_t *d_q_cells, const float *d_q_alt_lo, const float *d_q_alt_hi,
                                     const int64_t *d_q_tlo, const int64_t *d_q_thi, void *stream, void *xstream,
                                     dssg_pairs *out)
{
    if (!ctx || !comm || !xcomm || comm == xcomm || !xstream || !shard || !d_part_hi || !out || nq < 0 ||
        (nq > 0 && (!d_q_offs || !d_q_cells || !d_q_alt_lo || !d_q_alt_hi || !d_q_tlo || !d_q_thi)))
        return DSSG_ERR_INVALID;
    return guarded(ctx, [&] {
        hipStream_t s = stream ? (hipStream_t)stream : ctx->stream;
        if ((hipStream_t)xstream == s) throw dss::Error(DSSG_ERR_INVALID, "the exchange stream must differ");
        sharded_step(ctx, comm, xcomm, shard, d_part_hi, nq, d_q_offs, d_q_cells, d_q_alt_lo, d_q_alt_hi, d_q_tlo,
                     d_q_thi, s, (hipStream_t)xstream, out);
    });
}

int dssg_sharded_stats(dssg_ctx *ctx, double *ms, int64_t *counts)
{
    if (!ctx) return DSSG_ERR_INVALID;
    const dss::ShardStats &st = ctx->shard_stats;
    if (ms) {
        ms[0] = st.route_ms;
        ms[1] = st.xq_ms;
        ms[2] = st.join_ms;
        ms[3] = st.pack_ms;
        ms[4] = st.xp_ms;
    }
    if (counts) {
        counts[0] = st.q_bytes_sent;
        counts[1] = st.q_bytes_recv;
        counts[2] = st.p_bytes_sent;
        counts[3] = st.p_bytes_recv;
        counts[4] = st.rows;
        counts[5] = st.shard_pairs;
        counts[6] = st.cells;
        counts[7] = st.touched;
    }
    return DSSG_OK;
}

/* ======================================================================
 * Micro-batcher: the per-RPC path.  The reference runs one covering and one
 * SQL search per request (pkg/scd/operations_handler.go:118-168,
 * pkg/rid/server/isa_handler.go:153-207); here concurrent single requests
 * are coalesced into one cover launch and one join per batch, and each
 * caller gets its own answer back.  Several workers, each with its own
 * context, stream and pinned staging, run batches concurrently: while one
 * batch is on the GPU the next one is collected and started by another
 * worker, so batches form from whatever queued meanwhile (no fixed delay
 * when a worker is idle).  Small batches take the wave-path covering and
 * the one-launch small join (k_small_join).
 * ====================================================================== */
struct dssg_batcher {
    struct Req {
        int32_t kind = 0;
        const double *lat = nullptr, *lng = nullptr;  // the caller's arrays (it blocks until done)
        int64_t nv = 0;
        float radius = 0, alo = 0, ahi = 0;
        int64_t tlo = 0, thi = 0;
        std::vector<uint32_t> ids;
        int32_t status = 0;
        double area = 0;
        int rc = DSSG_OK;
        std::string err;
        bool done = false;
    };
    struct Worker {
        dssg_ctx *ctx = nullptr;
        std::thread th;
        unsigned char *h_in = nullptr, *h_out = nullptr;  // pinned staging
        size_t in_cap = 0, out_cap = 0;
        dss::DevBuf<unsigned char> d_in;
        std::vector<int64_t> cnt;
    };
    const dssg_index *idx = nullptr;
    int max_batch = 1024, max_wait_us = 0;
    std::mutex mu;
    std::condition_variable cv, done_cv;
    std::deque<Req *> queue;
    bool stop = false;
    int busy = 0;
    int64_t n_requests = 0, n_batches = 0;
    std::vector<Worker *> workers;
    // DSSG_BATCHER_PROFILE=1: mean host time per batch of the cover, join and
    // copy-back phases, printed to stderr when the batcher is freed
    bool prof = false;
    double prof_us[3] = {0, 0, 0};
    int64_t prof_n = 0;
    // answers a caller could not take (DSSG_ERR_CAPACITY): kept for its
    // retry, matched on the request's full inputs (the hash only picks
    // candidates) and dropped after kCacheTtl or when 1024 newer ones wait
    struct Cached {
        uint64_t key = 0;
        int32_t kind = 0;
        float radius = 0, alo = 0, ahi = 0;
        int64_t start = 0, end = 0, now = 0;
        std::vector<double> lat, lng;
        double area = 0;
        std::vector<uint32_t> ids;
        std::chrono::steady_clock::time_point at;
    };
    static constexpr std::chrono::milliseconds kCacheTtl{2000};
    std::mutex cache_mu;
    std::deque<Cached> cache;

    static size_t al8(size_t x) { return (x + 7) & ~(size_t)7; }

    static void pinned(unsigned char *&p, size_t &cap, size_t need)
    {
        if (need <= cap) return;
        if (p) (void)hipHostFree(p);
        p = nullptr;
        cap = 0;
        const size_t n = std::max(need + need / 2, (size_t)1 << 16);
        DSS_HIP(hipHostMalloc((void **)&p, n, hipHostMallocDefault));
        cap = n;
    }

    void run_batch(Worker &w, std::vector<Req *> &b)
    {
        const int64_t n = (int64_t)b.size();
        int64_t nv = 0;
        for (Req *r : b) nv += r->nv;
        // packed input layout (8-byte aligned sections), one H2D copy
        const size_t o_kind = 0, o_voff = al8(o_kind + 4 * n), o_lat = al8(o_voff + 8 * (n + 1)),
                     o_lng = o_lat + 8 * nv, o_rad = o_lng + 8 * nv, o_alo = al8(o_rad + 4 * n),
                     o_ahi = al8(o_alo + 4 * n), o_tlo = al8(o_ahi + 4 * n), o_thi = o_tlo + 8 * n,
                     in_bytes = o_thi + 8 * n;
        int64_t npairs = 0;
        const int rc = guarded(w.ctx, [&] {
            hipStream_t s = w.ctx->stream;
            pinned(w.h_in, w.in_cap, in_bytes);
            unsigned char *h = w.h_in;
            int32_t *kind = (int32_t *)(h + o_kind);
            int64_t *voff = (int64_t *)(h + o_voff);
            double *lat = (double *)(h + o_lat), *lng = (double *)(h + o_lng);
            float *rad = (float *)(h + o_rad), *alo = (float *)(h + o_alo), *ahi = (float *)(h + o_ahi);
            int64_t *tlo = (int64_t *)(h + o_tlo), *thi = (int64_t *)(h + o_thi);
            voff[0] = 0;
            for (int64_t i = 0; i < n; i++) {
                const Req *r = b[i];
                kind[i] = r->kind;
                if (r->nv > 0) {
                    std::memcpy(lat + voff[i], r->lat, sizeof(double) * (size_t)r->nv);
                    std::memcpy(lng + voff[i], r->lng, sizeof(double) * (size_t)r->nv);
                }
                voff[i + 1] = voff[i] + r->nv;
                rad[i] = r->radius;
                alo[i] = r->alo;
                ahi[i] = r->ahi;
                tlo[i] = r->tlo;
                thi[i] = r->thi;
            }
            unsigned char *d = w.d_in.ensure(in_bytes + 8);
            DSS_HIP(hipMemcpyAsync(d, h, in_bytes, hipMemcpyHostToDevice, s));
            dssg_cells cov;
            const auto t0 = std::chrono::steady_clock::now();
            w.ctx->cov_offs = nullptr;
            w.ctx->cover.run(n, (const int32_t *)(d + o_kind), (const int64_t *)(d + o_voff), (const double *)(d + o_lat),
                             (const double *)(d + o_lng), (const float *)(d + o_rad), s, &cov);
            // status and area ride along with the pairs' copy (pinned, no extra sync)
            const size_t r_area = 0, r_stat = 8 * n, r_q = al8(r_stat + 4 * n);
            pinned(w.h_out, w.out_cap, r_q + 8);
            DSS_HIP(hipMemcpyAsync(w.h_out + r_area, cov.area_km2, 8 * n, hipMemcpyDeviceToHost, s));
            DSS_HIP(hipMemcpyAsync(w.h_out + r_stat, cov.status, 4 * n, hipMemcpyDeviceToHost, s));
            const auto t1 = std::chrono::steady_clock::now();
            dssg_pairs res{};
            const float *dlo = (const float *)(d + o_alo), *dhi = (const float *)(d + o_ahi);
            const int64_t *dtl = (const int64_t *)(d + o_tlo), *dth = (const int64_t *)(d + o_thi);
            if (cov.total_cells > 0) {
                if (n <= w.ctx->search.small_max_q() && cov.total_cells <= 16 * w.ctx->search.small_max_q() &&
                    idx->n_p > 0)  // the cell count is known here: the small join without a fetch
                    w.ctx->search.search_small(idx, n, cov.offs, cov.cells, dlo, dhi, dtl, dth, nullptr,
                                               cov.total_cells, s, &res);
                else
                    w.ctx->search.search(idx, n, cov.offs, cov.cells, dlo, dhi, dtl, dth, nullptr, s, &res,
                                         cov.total_cells);
            }
            npairs = res.n;
            const auto t2 = std::chrono::steady_clock::now();
            const size_t r_e = r_q + 4 * npairs, out_bytes = r_e + 4 * npairs;
            if (out_bytes + 8 > w.out_cap) {  // regrow: the status/area copies must land first
                DSS_HIP(hipStreamSynchronize(s));
                std::vector<unsigned char> keep(w.h_out, w.h_out + r_q);
                pinned(w.h_out, w.out_cap, out_bytes + 8);
                std::memcpy(w.h_out, keep.data(), r_q);
            }
            if (npairs > 0) {
                DSS_HIP(hipMemcpyAsync(w.h_out + r_q, res.q, 4 * npairs, hipMemcpyDeviceToHost, s));
                DSS_HIP(hipMemcpyAsync(w.h_out + r_e, res.e, 4 * npairs, hipMemcpyDeviceToHost, s));
            }
            DSS_HIP(hipStreamSynchronize(s));
            const auto t3 = std::chrono::steady_clock::now();
            if (prof) {
                auto us = [](auto a, auto b) { return std::chrono::duration<double, std::micro>(b - a).count(); };
                std::lock_guard<std::mutex> lk(mu);
                prof_us[0] += us(t0, t1);
                prof_us[1] += us(t1, t2);
                prof_us[2] += us(t2, t3);
                prof_n++;
            }
            // each request's ids (unsorted here; the caller sorts its own)
            const uint32_t *pq = (const uint32_t *)(w.h_out + r_q), *pe = (const uint32_t *)(w.h_out + r_e);
            w.cnt.assign((size_t)n, 0);
            for (int64_t k = 0; k < npairs; k++) w.cnt[pq[k]]++;
            for (int64_t i = 0; i < n; i++) b[i]->ids.reserve((size_t)w.cnt[i]);
            for (int64_t k = 0; k < npairs; k++) b[pq[k]]->ids.push_back(pe[k]);
            const double *area = (const double *)(w.h_out + r_area);
            const int32_t *st = (const int32_t *)(w.h_out + r_stat);
            for (int64_t i = 0; i < n; i++) {
                b[i]->status = st[i];
                b[i]->area = area[i];
            }
        });
        std::lock_guard<std::mutex> lk(mu);
        for (int64_t i = 0; i < n; i++) {
            Req *r = b[i];
            r->rc = rc;
            if (rc != DSSG_OK) {
                r->err = w.ctx->last_error;
                r->ids.clear();
            }
            r->done = true;
        }
        n_batches++;
        n_requests += n;
        done_cv.notify_all();
    }

    void loop(Worker &w)
    {
        std::unique_lock<std::mutex> lk(mu);
        while (true) {
            cv.wait(lk, [&] { return stop || !queue.empty(); });
            if (queue.empty()) {
                if (stop) return;
                continue;
            }
            // another batch in flight: collect a little longer (bounded), else go now
            if (busy > 0 && max_wait_us > 0 && (int)queue.size() < max_batch) {
                const auto until = std::chrono::steady_clock::now() + std::chrono::microseconds(max_wait_us);
                cv.wait_until(lk, until, [&] { return stop || (int)queue.size() >= max_batch; });
                if (queue.empty()) continue;
            }
            std::vector<Req *> b;
            while (!queue.empty() && (int)b.size() < max_batch) {
                b.push_back(queue.front());
                queue.pop_front();
            }
            busy++;
            lk.unlock();
            run_batch(w, b);
            lk.lock();
            busy--;
        }
    }
};

namespace {
// FNV-1a over a request's inputs: the key of an answer kept for a retry.
uint64_t request_key(int32_t kind, int64_t nv, const double *lat, const double *lng, float radius_m, float alt_lo,
                     float alt_hi, int64_t start, int64_t end, int64_t now_us)
{
    uint64_t h = 1469598103934665603ull;
    auto mix = [&](const void *p, size_t n) {
        const unsigned char *c = (const unsigned char *)p;
        for (size_t i = 0; i < n; i++) h = (h ^ c[i]) * 1099511628211ull;
    };
    mix(&kind, sizeof(kind));
    mix(&nv, sizeof(nv));
    if (nv > 0) {
        mix(lat, sizeof(double) * (size_t)nv);
        mix(lng, sizeof(double) * (size_t)nv);
    }
    mix(&radius_m, 4);
    mix(&alt_lo, 4);
    mix(&alt_hi, 4);
    mix(&start, 8);
    mix(&end, 8);
    mix(&now_us, 8);
    return h;
}
}  // namespace

int dssg_batcher_create(int device, const dssg_index *idx, int32_t max_batch, int32_t max_wait_us, dssg_batcher **out)
{
    if (!idx || !out || max_batch < 1 || max_wait_us < 0) return DSSG_ERR_INVALID;
    if (device != idx->device) return DSSG_ERR_INVALID;  // the workers join against this device's index
    int nw = 2;
    if (const char *e = std::getenv("DSSG_BATCHER_WORKERS")) nw = std::max(1, std::min(16, std::atoi(e)));
    auto *b = new dssg_batcher();
    b->idx = idx;
    b->max_batch = max_batch;
    b->max_wait_us = max_wait_us;
    b->prof = std::getenv("DSSG_BATCHER_PROFILE") != nullptr;
    for (int k = 0; k < nw; k++) {
        auto *w = new dssg_batcher::Worker();
        const int rc = dssg_create(device, &w->ctx);
        if (rc != DSSG_OK) {
            delete w;
            b->stop = true;
            dssg_batcher_free(b);
            return rc;
        }
        b->workers.push_back(w);
    }
    for (auto *w : b->workers) w->th = std::thread([b, w] { b->loop(*w); });
    *out = b;
    return DSSG_OK;
}

void dssg_batcher_free(dssg_batcher *b)
{
    if (!b) return;
    {
        std::lock_guard<std::mutex> lk(b->mu);
        b->stop = true;
    }
    b->cv.notify_all();
    if (b->prof && b->prof_n)
        fprintf(stderr, "[dssg_batcher] %lld batches, %lld requests; mean us per batch: cover %.1f join %.1f copy %.1f\n",
                (long long)b->prof_n, (long long)b->n_requests, b->prof_us[0] / b->prof_n, b->prof_us[1] / b->prof_n,
                b->prof_us[2] / b->prof_n);
    for (auto *w : b->workers) {
        if (w->th.joinable()) w->th.join();
        if (w->ctx) {
            (void)hipSetDevice(w->ctx->device);
            if (w->h_in) (void)hipHostFree(w->h_in);
            if (w->h_out) (void)hipHostFree(w->h_out);
        }
        dssg_destroy(w->ctx);
        delete w;
    }
    delete b;
}

int dssg_batcher_search_operations(dssg_batcher *b, int32_t kind, int64_t nv, const double *lat, const double *lng,
                                   float radius_m, float alt_lo, float alt_hi, int64_t start, int64_t end,
                                   int64_t now_us, uint32_t *out_e, int64_t cap, int64_t *needed, int32_t *status,
                                   double *area_km2)
{
    if (!b || !needed || !status || nv < 0 || (nv > 0 && (!lat || !lng)) || now_us == INT64_MIN ||
        (kind != DSSG_KIND_POLYGON && kind != DSSG_KIND_CIRCLE && kind != DSSG_KIND_POINTS))
        return DSSG_ERR_INVALID;
    dssg_batcher::Req r;
    const uint64_t key = request_key(kind, nv, lat, lng, radius_m, alt_lo, alt_hi, start, end, now_us);
    bool cached = false;
    {  // the retry of a request whose answer did not fit: no second cover + join
        std::lock_guard<std::mutex> lk(b->cache_mu);
        const auto now_t = std::chrono::steady_clock::now();
        while (!b->cache.empty() && now_t - b->cache.front().at > dssg_batcher::kCacheTtl) b->cache.pop_front();
        auto same = [&](const dssg_batcher::Cached &c) {
            return c.key == key && c.kind == kind && (int64_t)c.lat.size() == nv && c.radius == radius_m &&
                   c.alo == alt_lo && c.ahi == alt_hi && c.start == start && c.end == end && c.now == now_us &&
                   (nv == 0 || (std::memcmp(c.lat.data(), lat, sizeof(double) * (size_t)nv) == 0 &&
                                std::memcmp(c.lng.data(), lng, sizeof(double) * (size_t)nv) == 0));
        };
        for (auto it = b->cache.begin(); it != b->cache.end(); ++it)
            if (same(*it) && (int64_t)it->ids.size() <= cap) {
                r.area = it->area;
                r.ids = std::move(it->ids);
                b->cache.erase(it);
                cached = true;
                break;
            }
    }
    if (cached) {
        // the covering succeeded the first time (a capacity answer implies status OK)
        *status = DSSG_ST_OK;
        if (area_km2) *area_km2 = r.area;
    } else {
        r.kind = kind;
        r.nv = nv;
        r.lat = lat;
        r.lng = lng;
        r.radius = radius_m;
        r.alo = alt_lo;
        r.ahi = alt_hi;
        r.tlo = std::max(start, now_us);  // operations.go:398-402
        r.thi = end;
        std::unique_lock<std::mutex> lk(b->mu);
        b->queue.push_back(&r);
        b->cv.notify_one();
        b->done_cv.wait(lk, [&] { return r.done; });
        lk.unlock();
        *status = r.status;
        if (area_km2) *area_km2 = r.area;
        if (r.rc != DSSG_OK) return r.rc;
        std::sort(r.ids.begin(), r.ids.end());
    }
    *needed = (int64_t)r.ids.size();
    if ((int64_t)r.ids.size() > cap) {
        dssg_batcher::Cached c;
        c.key = key;
        c.kind = kind;
        c.radius = radius_m;
        c.alo = alt_lo;
        c.ahi = alt_hi;
        c.start = start;
        c.end = end;
        c.now = now_us;
        if (nv > 0) {
            c.lat.assign(lat, lat + nv);
            c.lng.assign(lng, lng + nv);
        }
        c.area = r.area;
        c.ids = std::move(r.ids);
        c.at = std::chrono::steady_clock::now();
        std::lock_guard<std::mutex> lk(b->cache_mu);
        b->cache.push_back(std::move(c));
        while (b->cache.size() > 1024) b->cache.pop_front();
        return DSSG_ERR_CAPACITY;
    }
    if (!r.ids.empty()) {
        if (!out_e) return DSSG_ERR_INVALID;
        std::memcpy(out_e, r.ids.data(), sizeof(uint32_t) * r.ids.size());
    }
    return DSSG_OK;
}

int dssg_batcher_stats(dssg_batcher *b, int64_t *requests, int64_t *batches)
{
    if (!b) return DSSG_ERR_INVALID;
    std::lock_guard<std::mutex> lk(b->mu);
    if (requests) *requests = b->n_requests;
    if (batches) *batches = b->n_batches;
    return DSSG_OK;
}
