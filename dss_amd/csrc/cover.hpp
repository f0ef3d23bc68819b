// Host-side driver of the covering kernels (cover.hip).
#pragma once
#include "common.hpp"

namespace dss {

struct Frontier {
    DevBuf<uint32_t> f;
    DevBuf<uint64_t> id;
    DevBuf<uint32_t> i, j, meta;
    void ensure(size_t n)
    {
        f.ensure(n);
        id.ensure(n);
        i.ensure(n);
        j.ensure(n);
        meta.ensure(n);
    }
};

class CoverEngine {
   public:
    // Device pointers in, context-owned device buffers out (see dssg_cells).
    void run(int64_t n, const int32_t *kind, const int64_t *voff, const double *lat, const double *lng,
             const float *radius_m, hipStream_t s, dssg_cells *out);

   private:
    DevBuf<int64_t> cnt_, xoff_, eoff_, soff_, offs_, ncnt_, npos_, fc64_;
    DevBuf<int32_t> status_, nvx_;
    DevBuf<double> area_, xyz_;
    DevBuf<uint8_t> mode_, orig_, fmask_, flags_, cflags_, act_;
    DevBuf<uint32_t> slow_, vown_;
    DevBuf<uint8_t> fanf_, ninner_;
    DevBuf<uint32_t> perm_, towner_;
    DevBuf<uint8_t> omode_;
    DevBuf<int64_t> tcnt_, toff_;
    DevBuf<double> fwd_, rev_;
    DevBuf<unsigned char> frames_;
    DevBuf<unsigned int> slow_n_;
    DevBuf<double4> clipf_, clipc_;
    DevBuf<unsigned char> tmp_, tmp2_;
    DevBuf<int> flag_;
    DevBuf<unsigned long long> fcnt_;
    DevBuf<uint64_t> cells_;
    DevBuf<uint32_t> big_;
    Frontier fr_[2];
    // direct candidate path
    DevBuf<double2> uv_;
    DevBuf<uint64_t> st_id_;
    DevBuf<uint32_t> st_i_, st_j_, finfo_, cand_f_;
    DevBuf<int64_t> ncand_, coff_, gcnt_, gpos_, dc64_, dpre_;
    DevBuf<unsigned long long> kmask_;
    DevBuf<uint4> fbox_;
    bool tables_ = false;
};

}  // namespace dss
