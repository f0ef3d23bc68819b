// Write path over the HBM entity index.
//
// The reference keeps operations in CockroachDB and rewrites the posting rows
// on every write: UpsertOperation -> pushOperation (UPSERT the row, UPSERT one
// scd_cells_operations row per cell, DELETE the cells no longer covered,
// pkg/scd/store/cockroach/operations.go:119-193, 304-372), DeleteOperation
// (:239-301), RID InsertISA / DeleteISA (pkg/rid/cockroach/
// identification_service_area.go:97-160).  Searches see every committed write.
//
// Here an immutable, fully built index (the base) serves most entities; the
// entities written since the base was built live in a small delta index,
// rebuilt on each write batch, and a tombstone bitmap on the base masks the
// base copies of rewritten or deleted entities inside the join kernel
// (load_slot) and the subscription queries.  A search runs against both and
// maps each side's dense entity index back to the caller's id.  When the
// delta outgrows a fraction of the base the two are folded into a new base.
// The authoritative rows stay in host memory (the store is the system of
// record for the GPU copy), so a rebuild never reads the device.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <vector>

#include "store.hpp"

namespace dss {
namespace {

constexpr unsigned kBlock = 256;

__global__ void k_remap(int64_t n, uint32_t *e, const uint32_t *ids)
{
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n) e[i] = ids[e[i]];
}

}  // namespace

Store::~Store()
{
    if (base_) dssg_index_free(base_);
    if (delta_) dssg_index_free(delta_);
}

void Store::check_ids(int64_t n, const uint32_t *ids) const
{
    for (int64_t i = 0; i < n; i++)
        if (ids[i] == 0xffffffffu) throw Error(DSSG_ERR_INVALID, "store: id 0xffffffff is reserved");
}

void Store::upsert(SearchEngine &se, int64_t n, const uint32_t *ids, const int64_t *offs, const uint64_t *cells,
                   const float *alo, const float *ahi, const int64_t *t0, const int64_t *t1, const int32_t *owner,
                   hipStream_t s)
{
    check_ids(n, ids);
    if (with_owner_ && n > 0 && !owner) throw Error(DSSG_ERR_INVALID, "store: owners required");
    for (int64_t i = 0; i < n; i++) {
        const uint32_t id = ids[i];
        if (id >= rows_.size()) rows_.resize((size_t)id + 1);
        Row &r = rows_[id];
        if (!r.live) live_++;
        r.live = true;
        r.cells.assign(cells + offs[i], cells + offs[i + 1]);
        r.alo = alo[i];
        r.ahi = ahi[i];
        r.t0 = t0[i];
        r.t1 = t1[i];
        r.owner = owner ? owner[i] : 0;
        if (!r.in_delta) delta_list_.push_back(id);
        r.in_delta = true;
        tomb(id);
    }
    refresh(se, s);
}

void Store::remove(SearchEngine &se, int64_t n, const uint32_t *ids, int32_t *found, hipStream_t s)
{
    check_ids(n, ids);
    for (int64_t i = 0; i < n; i++) {
        const uint32_t id = ids[i];
        const bool f = id < rows_.size() && rows_[id].live;
        if (found) found[i] = f ? 1 : 0;
        if (!f) continue;
        Row &r = rows_[id];
        r.live = false;  // stays in delta_list_ until the next refresh drops it
        r.cells.clear();
        live_--;
        tomb(id);
    }
    refresh(se, s);
}

// Mask the base copy of `id`, if it has one.
void Store::tomb(uint32_t id)
{
    if (id < base_pos_.size() && base_pos_[id] >= 0) {
        const uint32_t e = (uint32_t)base_pos_[id];
        dead_h_[e >> 5] |= 1u << (e & 31);
        dead_dirty_ = true;
    }
}

// Build an index over the given ids (their current rows); returns the dense
// index -> id map in `map`.
dssg_index *Store::build(SearchEngine &se, const std::vector<uint32_t> &ids, hipStream_t s, DevBuf<uint32_t> &map)
{
    const int64_t n = (int64_t)ids.size();
    std::vector<int64_t> offs((size_t)n + 1, 0);
    for (int64_t i = 0; i < n; i++) offs[i + 1] = offs[i] + (int64_t)rows_[ids[i]].cells.size();
    std::vector<uint64_t> cells((size_t)offs[n]);
    std::vector<float> lo((size_t)n), hi((size_t)n);
    std::vector<int64_t> a0((size_t)n), a1((size_t)n);
    std::vector<int32_t> ow((size_t)n);
    for (int64_t i = 0; i < n; i++) {
        const Row &r = rows_[ids[i]];
        std::copy(r.cells.begin(), r.cells.end(), cells.begin() + offs[i]);
        lo[i] = r.alo;
        hi[i] = r.ahi;
        a0[i] = r.t0;
        a1[i] = r.t1;
        ow[i] = r.owner;
    }
    auto up = [&](auto &buf, const auto &v) {
        auto *d = buf.ensure(v.size() + 1);
        if (!v.empty()) DSS_HIP(hipMemcpyAsync(d, v.data(), sizeof(v[0]) * v.size(), hipMemcpyHostToDevice, s));
        return d;
    };
    const int64_t *d_offs = up(u_offs_, offs);
    const uint64_t *d_cells = up(u_cells_, cells);
    const float *d_lo = up(u_lo_, lo), *d_hi = up(u_hi_, hi);
    const int64_t *d_a0 = up(u_t0_, a0), *d_a1 = up(u_t1_, a1);
    const int32_t *d_ow = with_owner_ ? up(u_ow_, ow) : nullptr;
    up(map, ids);
    dssg_index *idx = new dssg_index();
    idx->device = device_;
    try {
        se.build(idx, n, d_offs, d_cells, d_lo, d_hi, d_a0, d_a1, d_ow, 0, ~0ull, s);
    } catch (...) {
        delete idx;
        throw;
    }
    return idx;
}

// Rebuild the delta index (or fold everything into a new base when the delta
// has grown past max(kMinDelta, base / kDeltaFrac)), then upload tombstones.
void Store::refresh(SearchEngine &se, hipStream_t s)
{
    // the delta's ids come from the write list (O(delta), not O(max id));
    // deleted ones leave it here
    std::vector<uint32_t> dids;
    size_t keep = 0;
    for (const uint32_t id : delta_list_) {
        Row &r = rows_[id];
        if (!r.live) {
            r.in_delta = false;
            continue;
        }
        delta_list_[keep++] = id;
        dids.push_back(id);
    }
    delta_list_.resize(keep);
    std::sort(dids.begin(), dids.end());
    const int64_t nbase = base_ ? base_->n_e : 0;
    if ((int64_t)dids.size() > std::max<int64_t>(kMinDelta, nbase / kDeltaFrac)) {
        compact(se, s);
        return;
    }
    if (delta_) {
        dssg_index_free(delta_);
        delta_ = nullptr;
    }
    if (!dids.empty()) delta_ = build(se, dids, s, delta_ids_);
    if (base_ && dead_dirty_) {
        uint32_t *d = base_->dead.ensure(dead_h_.size() + 1);
        DSS_HIP(hipMemcpyAsync(d, dead_h_.data(), sizeof(uint32_t) * dead_h_.size(), hipMemcpyHostToDevice, s));
        base_->has_dead = true;
        dead_dirty_ = false;
    }
    DSS_HIP(hipStreamSynchronize(s));
}

void Store::compact(SearchEngine &se, hipStream_t s)
{
    std::vector<uint32_t> ids;
    for (uint32_t id = 0; id < rows_.size(); id++)
        if (rows_[id].live) ids.push_back(id);
    if (base_) dssg_index_free(base_);
    if (delta_) dssg_index_free(delta_);
    base_ = delta_ = nullptr;
    base_pos_.assign(rows_.size(), -1);
    for (size_t i = 0; i < ids.size(); i++) base_pos_[ids[i]] = (int64_t)i;
    for (Row &r : rows_) r.in_delta = false;
    delta_list_.clear();
    dead_h_.assign(ids.size() / 32 + 1, 0u);
    dead_dirty_ = false;
    if (!ids.empty()) base_ = build(se, ids, s, base_ids_);
    compactions_++;
    DSS_HIP(hipStreamSynchronize(s));
}

int64_t Store::search(SearchEngine &se, int64_t nq, const int64_t *d_offs, const uint64_t *d_cells, const float *d_alo,
                      const float *d_ahi, const int64_t *d_tlo, const int64_t *d_thi, const int32_t *d_owner,
                      hipStream_t s, std::vector<uint64_t> &out)
{
    out.clear();
    dssg_index *sides[2] = {base_, delta_};
    DevBuf<uint32_t> *maps[2] = {&base_ids_, &delta_ids_};
    for (int k = 0; k < 2; k++) {
        if (!sides[k]) continue;
        if (d_owner && !sides[k]->has_owner) throw Error(DSSG_ERR_INVALID, "store: built without owners");
        dssg_pairs p;
        se.search(sides[k], nq, d_offs, d_cells, d_alo, d_ahi, d_tlo, d_thi, d_owner, s, &p);
        if (p.n == 0) continue;
        // dense entity index -> caller id, in place (the engine's buffer)
        hipLaunchKernelGGL(k_remap, dim3(grid_for(p.n, kBlock)), dim3(kBlock), 0, s, p.n, const_cast<uint32_t *>(p.e),
                           maps[k]->p);
        std::vector<uint32_t> q((size_t)p.n), e((size_t)p.n);
        DSS_HIP(hipMemcpyAsync(q.data(), p.q, sizeof(uint32_t) * p.n, hipMemcpyDeviceToHost, s));
        DSS_HIP(hipMemcpyAsync(e.data(), p.e, sizeof(uint32_t) * p.n, hipMemcpyDeviceToHost, s));
        DSS_HIP(hipStreamSynchronize(s));
        for (int64_t i = 0; i < p.n; i++) out.push_back(((uint64_t)q[i] << 32) | e[i]);
    }
    std::sort(out.begin(), out.end());
    return (int64_t)out.size();
}

}  // namespace dss
