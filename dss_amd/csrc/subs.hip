// Subscription-store queries on the HBM entity index:
//
//  * notification fan-out -- RID UpdateNotificationIdxsInCells
//    (pkg/rid/cockroach/subscriptions.go:204-219) and SCD
//    fetchSubscriptionsForNotification (pkg/scd/store/cockroach/
//    subscriptions.go:128-173): the overlap join (search.hip, predicate
//    `ends_at >= now`) finds the pairs; here they are ordered by (entity,
//    query) and every entity's notification_index advances once per query
//    that met it, in batch order, each pair returning the value after its
//    own increment (the UPDATE ... RETURNING of that query);
//  * owner-only subscription search -- SCD SearchSubscriptions
//    (pkg/scd/store/cockroach/subscriptions.go:497-545): its LEFT JOIN keeps
//    every row, so the result is every unexpired subscription of the owner
//    and the cells do not filter (quirk Q7);
//  * max subscriptions per cell -- RID MaxSubscriptionCountInCellsByOwner
//    (pkg/rid/cockroach/subscriptions.go:83-116) and SCD
//    fetchMaxSubscriptionCountByCellAndOwner (pkg/scd/store/cockroach/
//    subscriptions.go:255-283): max over the query cells of the owner's
//    unexpired subscriptions in that cell, counting repeats of the cell in a
//    stored array (RID `unnest(cells)`) -- b_mult.
#include <hip/hip_runtime.h>


#include "index_view.cuh"
#include "radix.hpp"
#include "subs.hpp"

namespace dss {
namespace {

constexpr unsigned kBlock = 256;

// Query of every query cell.
__global__ void k_cell_q(int64_t nq, const int64_t *offs, uint32_t *cq)
{
    const int64_t q = tid64();
    if (q >= nq) return;
    for (int64_t k = offs[q]; k < offs[q + 1]; k++) cq[k] = (uint32_t)q;
}

// One thread per query cell: the owner's unexpired entities posted in the
// cell, repeats counted, added to the cell's count (one index of several:
// a store's base and delta hold disjoint live entities).
__global__ void k_cell_count(IndexView a, int64_t nqc, const uint64_t *cells, const uint32_t *cq, const int32_t *owner,
                             long long now, unsigned long long *cell_cnt)
{
    const int64_t k = tid64();
    if (k >= nqc) return;
    uint32_t slot = 0;
    uint64_t s = 0, e = 0;
    if (!find_slot(a, cells[k], slot)) return;
    slot_range(a, slot, s, e);
    const int32_t own = owner[cq[k]];
    const uint32_t bit = child_bit(cells[k], a.gshift);
    unsigned long long cnt = 0;
    for (uint64_t p = s; p < e; p++) {  // the quad's postings that hold this cell
        if (!(a.b_meta[p] & bit)) continue;
        const uint32_t ent = a.b_e[p] & ~kFirstBit;
        if (a.e_owner[ent] == own && a.e_t1[ent] >= now && !is_dead(a, ent)) cnt += child_mult(a, p, bit);
    }
    cell_cnt[k] += cnt;  // (one thread per cell; the sides run one after another)
}

// The query keeps the max over its cells.
__global__ void k_cell_max(int64_t nqc, const uint32_t *cq, const unsigned long long *cell_cnt, unsigned long long *out)
{
    const int64_t k = tid64();
    if (k >= nqc) return;
    if (cell_cnt[k]) atomicMax(&out[cq[k]], cell_cnt[k]);
}

__device__ __forceinline__ uint32_t lower_bound_u32(const uint32_t *x, uint32_t n, uint32_t v)
{
    uint32_t lo = 0, hi = n;
    while (lo < hi) {
        const uint32_t m = (lo + hi) >> 1;
        if (x[m] < v) lo = m + 1;
        else hi = m;
    }
    return lo;
}

// One thread per query: the owner's entities with ends_at >= now.  PASS 0
// counts, PASS 1 writes at off[q].
template <int PASS>
__global__ void k_owner_subs(int64_t nq, const int32_t *owner, long long now, const uint32_t *o_key, const uint32_t *o_ent,
                             uint32_t n, const int64_t *e_t1, const uint32_t *dead, int64_t *cnt, const int64_t *off,
                             uint32_t *out_q, uint32_t *out_e)
{
    const int64_t q = tid64();
    if (q >= nq) return;
    const uint32_t key = (uint32_t)owner[q] ^ 0x80000000u;
    const uint32_t b = lower_bound_u32(o_key, n, key);
    const uint32_t e = key == 0xffffffffu ? n : lower_bound_u32(o_key, n, key + 1);
    int64_t c = 0, w = PASS ? off[q] : 0;
    for (uint32_t i = b; i < e; i++) {
        const uint32_t ent = o_ent[i];
        if (e_t1[ent] < now || (dead && ((dead[ent >> 5] >> (ent & 31)) & 1u))) continue;
        if (PASS) {
            out_q[w] = (uint32_t)q;
            out_e[w] = ent;
            w++;
        } else {
            c++;
        }
    }
    if (!PASS) cnt[q] = c;
}

__global__ void k_pair_keys(int64_t n, const uint32_t *q, const uint32_t *e, unsigned long long *key)
{
    const int64_t i = tid64();
    if (i < n) key[i] = ((unsigned long long)e[i] << 32) | q[i];
}

// First index in the sorted keys with entity `ent` (keys[0..hi] sorted).
__device__ __forceinline__ int64_t run_start(const unsigned long long *key, int64_t hi, uint32_t ent)
{
    const unsigned long long v = (unsigned long long)ent << 32;
    int64_t lo = 0;
    while (lo < hi) {
        const int64_t m = (lo + hi) >> 1;
        if (key[m] < v) lo = m + 1;
        else hi = m;
    }
    return lo;
}

// Pairs sorted by (entity, query): the k-th query (batch order) meeting an
// entity sees its counter + k + 1.
__global__ void k_notify_values(int64_t n, const unsigned long long *key, const int64_t *counter, uint32_t *out_q,
                                uint32_t *out_e, int64_t *out_v)
{
    const int64_t i = tid64();
    if (i >= n) return;
    const uint32_t ent = (uint32_t)(key[i] >> 32);
    const int64_t r = i - run_start(key, i, ent);
    out_q[i] = (uint32_t)key[i];
    out_e[i] = ent;
    out_v[i] = counter[ent] + r + 1;
}
// The last pair of each entity's run commits the new counter (after
// k_notify_values has read every old one).
__global__ void k_notify_commit(int64_t n, const unsigned long long *key, const int64_t *val, int64_t *counter)
{
    const int64_t i = tid64();
    if (i >= n) return;
    const uint32_t ent = (uint32_t)(key[i] >> 32);
    if (i == n - 1 || (uint32_t)(key[i + 1] >> 32) != ent) counter[ent] = val[i];
}

int bits_for_n(int64_t n)
{
    int b = 1;
    while (b < 63 && ((int64_t)1 << b) <= n) b++;
    return b;
}

}  // namespace

void SubsEngine::max_count(const dssg_index *const *sides, int nsides, int64_t nq, const int64_t *offs,
                           const uint64_t *cells, int64_t nqc, const int32_t *owner, int64_t now, hipStream_t s,
                           int64_t *out)
{
    for (int k = 0; k < nsides; k++)
        if (sides[k] && !sides[k]->has_owner)
            throw Error(DSSG_ERR_INVALID, "max subscription count on an index built without owners");
    unsigned long long *d = cnt_.ensure(nq + 1);
    DSS_HIP(hipMemsetAsync(d, 0, sizeof(unsigned long long) * (nq + 1), s));
    if (nqc > 0) {
        uint32_t *cq = cq_.ensure(nqc + 1);
        unsigned long long *cc = k0_.ensure(nqc + 1);
        DSS_HIP(hipMemsetAsync(cc, 0, sizeof(unsigned long long) * nqc, s));
        hipLaunchKernelGGL(k_cell_q, dim3(grid_for(nq, kBlock)), dim3(kBlock), 0, s, nq, offs, cq);
        for (int k = 0; k < nsides; k++)
            if (sides[k] && sides[k]->n_p > 0)
                hipLaunchKernelGGL(k_cell_count, dim3(grid_for(nqc, kBlock)), dim3(kBlock), 0, s, view_of(sides[k]), nqc,
                                   cells, cq, owner, (long long)now, cc);
        hipLaunchKernelGGL(k_cell_max, dim3(grid_for(nqc, kBlock)), dim3(kBlock), 0, s, nqc, cq, cc, d);
    }
    if (nq > 0) DSS_HIP(hipMemcpyAsync(out, d, sizeof(int64_t) * nq, hipMemcpyDeviceToHost, s));
    DSS_HIP(hipStreamSynchronize(s));
}

int64_t SubsEngine::owner_subs(const dssg_index *idx, int64_t nq, const int32_t *owner, int64_t now, hipStream_t s,
                               uint32_t **out_q, uint32_t **out_e)
{
    if (!idx->has_owner) throw Error(DSSG_ERR_INVALID, "owner search on an index built without owners");
    int64_t *cnt = c_.ensure(nq + 1), *off = o_.ensure(nq + 2);
    const uint32_t n = (uint32_t)idx->n_e;
    if (nq > 0)
        hipLaunchKernelGGL(k_owner_subs<0>, dim3(grid_for(nq, kBlock)), dim3(kBlock), 0, s, nq, owner, (long long)now,
                           idx->o_key.p, idx->o_ent.p, n, idx->e_t1.p, idx->has_dead ? idx->dead.p : nullptr, cnt,
                           nullptr, nullptr, nullptr);
    exclusive_scan_i64(cnt, off, nq, tmp_, s);
    int64_t total = 0;
    DSS_HIP(hipMemcpyAsync(&total, off + nq, sizeof(int64_t), hipMemcpyDeviceToHost, s));
    DSS_HIP(hipStreamSynchronize(s));
    uint32_t *oq = q_.ensure(total + 1), *oe = e_.ensure(total + 1);
    if (nq > 0 && total > 0)
        hipLaunchKernelGGL(k_owner_subs<1>, dim3(grid_for(nq, kBlock)), dim3(kBlock), 0, s, nq, owner, (long long)now,
                           idx->o_key.p, idx->o_ent.p, n, idx->e_t1.p, idx->has_dead ? idx->dead.p : nullptr, nullptr,
                           off, oq, oe);
    DSS_HIP(hipStreamSynchronize(s));
    *out_q = oq;
    *out_e = oe;
    return total;
}

void SubsEngine::notify(dssg_index *idx, const dssg_pairs *p, hipStream_t s, uint32_t **out_q, uint32_t **out_e,
                        int64_t **out_v)
{
    const int64_t n = p->n;
    unsigned long long *k0 = k0_.ensure(n + 1), *k1 = k1_.ensure(n + 1);
    uint32_t *oq = q_.ensure(n + 1), *oe = e_.ensure(n + 1);
    int64_t *ov = v_.ensure(n + 1);
    if (n > 0) {
        hipLaunchKernelGGL(k_pair_keys, dim3(grid_for(n, kBlock)), dim3(kBlock), 0, s, n, p->q, p->e, k0);
        radix_sort_keys(k0, k1, n, 32 + bits_for_n(idx->n_e), tmp_, s);
        hipLaunchKernelGGL(k_notify_values, dim3(grid_for(n, kBlock)), dim3(kBlock), 0, s, n, k1, idx->e_notify.p, oq, oe, ov);
        hipLaunchKernelGGL(k_notify_commit, dim3(grid_for(n, kBlock)), dim3(kBlock), 0, s, n, k1, ov, idx->e_notify.p);
    }
    DSS_HIP(hipStreamSynchronize(s));
    *out_q = oq;
    *out_e = oe;
    *out_v = ov;
}

}  // namespace dss
