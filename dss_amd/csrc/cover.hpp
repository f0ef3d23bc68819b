// Host-side driver of the covering kernels (cover.hip).
#pragma once
#include <vector>

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
    CoverEngine() = default;
    CoverEngine(const CoverEngine &) = delete;
    CoverEngine &operator=(const CoverEngine &) = delete;
    ~CoverEngine()
    {
        // the last upload out of the pinned offsets must have landed first
        if (h_ev_) (void)hipEventSynchronize(h_ev_);
        if (h_offs_) (void)hipHostFree(h_offs_);
        if (h_ev_) (void)hipEventDestroy(h_ev_);
        if (mail_h_) (void)hipHostFree(mail_h_);
    }
    // Device pointers in, context-owned device buffers out (see dssg_cells).
    // The wave path (one wavefront per footprint) covers every footprint it
    // can decide; the rest go through the general pipeline (run_general) as
    // one compacted sub-batch.
    void run(int64_t n, const int32_t *kind, const int64_t *voff, const double *lat, const double *lng,
             const float *radius_m, hipStream_t s, dssg_cells *out);
    // batches of at most `n` footprints take the wave path (0: never; tests
    // force it for every batch)
    void set_wave_max(int64_t n) { wave_ = n > 0; wave_max_ = n; }
    int64_t last_slow() const { return last_slow_; }
    // (tests) every general-path footprint through the exact setup
    void set_all_exact(bool on) { all_exact_ = on; }
    // vertex slots in k_setup's footprint order (default) or in footprint order
    void set_slot_order(bool kind_major) { slot_order_ = kind_major; }

   private:
    void run_general(int64_t n, const int32_t *kind, const int64_t *voff, const double *lat, const double *lng,
                     const float *radius_m, hipStream_t s, dssg_cells *out);
    void init_tables(hipStream_t s);
    bool wave_ = true;
    bool all_exact_ = false;
#ifndef DSS_SLOT_ORDER
#define DSS_SLOT_ORDER 1
#endif
    bool slot_order_ = DSS_SLOT_ORDER != 0;
    int64_t wave_max_ = 16384;
    int64_t last_slow_ = 0;
    // wave path: per-footprint outputs, the slow sub-batch, the merged CSR
    DevBuf<int32_t> w_status_, s_kind_;
    DevBuf<double> w_area_, s_lat_, s_lng_;
    DevBuf<int64_t> w_cnt_, w_offs_, s_nv_, s_voff_, w_tot_;
    DevBuf<unsigned char> w_rec_;
    DevBuf<uint8_t> w_slow_;
    DevBuf<uint32_t> s_list_;
    DevBuf<float> s_rad_;
    DevBuf<uint64_t> w_cells_;
    std::vector<int64_t> h_cnt_;
    int64_t *h_offs_ = nullptr, h_offs_cap_ = 0;  // pinned
    // the general path's counts, written by the kernels that produce them
    // into fine-grained host memory (no copy launch per read-back)
    int64_t *mail_h_ = nullptr, *mail_d_ = nullptr;
    int64_t *mailbox();
    hipEvent_t h_ev_ = nullptr;                   // the last upload from h_offs_
    std::vector<uint8_t> h_slow_;
    DevBuf<int64_t> cnt_, xoff_, eoff_, soff_, offs_, ncnt_, npos_, fc64_, nvp_, xoffp_;
    DevBuf<int32_t> status_, nvx_;
    DevBuf<double> area_, xyz_;
    DevBuf<uint8_t> mode_, orig_, fmask_, flags_, cflags_, act_;
    DevBuf<uint32_t> slow_, vown_, eown_, dlist_, xlist_;
    DevBuf<unsigned int> dlist_n_, xlist_n_;
    DevBuf<uint8_t> fanf_, ninner_, badv_;
    DevBuf<unsigned char> sdesc_;      // k_start13's start cells
    DevBuf<unsigned int> sdesc_n_;
    DevBuf<uint32_t> perm_, towner_;
    DevBuf<uint8_t> omode_, revf_;
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
    DevBuf<uint32_t> st_i_, st_j_, finfo_;
    DevBuf<int64_t> dc64_, dpre_;
    DevBuf<unsigned long long> kmask_;
    DevBuf<uint32_t> ulist_;          // footprints with undecided candidates
    DevBuf<unsigned int> ulist_n_;
    DevBuf<uint4> fbox_;
    bool tables_ = false;
};

}  // namespace dss
