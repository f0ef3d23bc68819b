// Device-wide scans (hipcub / rocPRIM) used by the covering and search
// pipelines for order-preserving compaction.
#include <hipcub/hipcub.hpp>

#include "common.hpp"

namespace dss {

void exclusive_scan_i64(const int64_t *in, int64_t *out, int64_t n, DevBuf<unsigned char> &tmp, hipStream_t s)
{
    DSS_HIP(hipMemsetAsync(out, 0, sizeof(int64_t), s));
    if (n <= 0) return;
    size_t bytes = 0;
    DSS_HIP(hipcub::DeviceScan::InclusiveSum(nullptr, bytes, in, out + 1, (int)n, s));
    tmp.ensure(bytes + 16);
    DSS_HIP(hipcub::DeviceScan::InclusiveSum(tmp.p, bytes, in, out + 1, (int)n, s));
}

namespace {
struct NotCircle {
    __host__ __device__ bool operator()(int32_t k) const { return k != DSSG_KIND_CIRCLE; }
};
}  // namespace

void partition_polygons_first(const int32_t *kind, uint32_t *perm, unsigned long long *nsel, int64_t n,
                              DevBuf<unsigned char> &tmp, hipStream_t s)
{
    if (n <= 0) return;
    hipcub::CountingInputIterator<uint32_t> idx(0);
    hipcub::TransformInputIterator<bool, NotCircle, const int32_t *> flags(kind, NotCircle());
    size_t bytes = 0;
    DSS_HIP(hipcub::DevicePartition::Flagged(nullptr, bytes, idx, flags, perm, nsel, (int)n, s));
    tmp.ensure(bytes + 16);
    DSS_HIP(hipcub::DevicePartition::Flagged(tmp.p, bytes, idx, flags, perm, nsel, (int)n, s));
}

}  // namespace dss
