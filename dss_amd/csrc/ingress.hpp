// Host-side driver of batched ingress (ingress.hip): UnionVolumes4D.
#pragma once
#include "common.hpp"
#include "cover.hpp"

namespace dss {

class IngressEngine {
   public:
    // Extents [vol_offs[v], vol_offs[v+1]) form volume v; extent x has a
    // footprint iff has_fp[x] (else its cells and status are ignored),
    // altitude NaN = NULL, t0 INT64_MIN / t1 INT64_MAX = NULL.
    void union_volumes(CoverEngine &ce, int64_t nvol, const int64_t *vol_offs, int64_t nx, const int32_t *kind,
                       const int64_t *voff, const double *lat, const double *lng, const float *radius_m,
                       const uint8_t *has_fp, const float *alo, const float *ahi, const int64_t *t0, const int64_t *t1,
                       hipStream_t s, dssg_volumes *out);

   private:
    DevBuf<unsigned char> tmp_;
    DevBuf<uint32_t> evol_;
    DevBuf<unsigned long long> k0_, k1_, vcnt_;
    DevBuf<int64_t> flag_, pos_, v64_, offs_, t0_, t1_;
    DevBuf<uint64_t> cells_;
    DevBuf<int32_t> status_;
    DevBuf<double> area_;
    DevBuf<float> lo_, hi_;
    DevBuf<uint8_t> fp_;
};

}  // namespace dss
