// Shared host-side plumbing for the dss_amd HIP library: error handling,
// grow-only device buffers, scans.  No torch types anywhere in the library.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <algorithm>
#include <stdexcept>
#include <string>

#include "../../include/dssgpu.h"

namespace dss {

struct Error : std::runtime_error {
    int code;
    Error(int c, const std::string &m) : std::runtime_error(m), code(c) {}
};

#define DSS_HIP(expr)                                                                                     \
    do {                                                                                                  \
        hipError_t e_ = (expr);                                                                           \
        if (e_ != hipSuccess)                                                                             \
            throw ::dss::Error(DSSG_ERR_DEVICE, std::string(#expr) + ": " + hipGetErrorString(e_));      \
    } while (0)

// Grow-only device allocation; contents are not preserved on growth.
template <typename T>
struct DevBuf {
    T *p = nullptr;
    size_t cap = 0;
    DevBuf() = default;
    DevBuf(const DevBuf &) = delete;
    DevBuf &operator=(const DevBuf &) = delete;
    ~DevBuf() { release(); }
    void release()
    {
        if (p) (void)hipFree(p);
        p = nullptr;
        cap = 0;
    }
    T *ensure(size_t n)
    {
        if (n <= cap && p) return p;
        release();
        // 25 % growth slack, at most 256 MiB of it
        const size_t slack = std::min(n / 4, ((size_t)256 << 20) / sizeof(T));
        size_t c = n < 16 ? 16 : n + slack;
        alloc(c);
        return p;
    }
    // no growth slack: for the long-lived index arrays (tens of GB at the
    // largest airspaces)
    T *ensure_exact(size_t n)
    {
        if (n <= cap && p) return p;
        release();
        const size_t c = n < 16 ? 16 : n;
        alloc(c);
        return p;
    }
    void alloc(size_t c)
    {
        const hipError_t e = hipMalloc(&p, c * sizeof(T));
        if (e != hipSuccess) {
            p = nullptr;
            cap = 0;
            (void)hipGetLastError();
            throw Error(DSSG_ERR_DEVICE, "hipMalloc of " + std::to_string(c * sizeof(T)) + " bytes: " + hipGetErrorString(e));
        }
        cap = c;
    }
};

inline unsigned grid_for(int64_t n, unsigned block) { return (unsigned)((n + block - 1) / block); }

// Device-to-device copy by a kernel (16-byte vectors when both ends allow),
// any size: the runtime's blit path is not relied on for multi-GB copies.
void device_copy(void *dst, const void *src, size_t bytes, hipStream_t s);

// With DSSG_SYNC_CHECK=1 in the environment: synchronize and raise with the
// stage's name on any device error (localizes a fault to a build stage).
void stage_check(hipStream_t s, const char *stage);

// Exclusive prefix sum of n int64 values into out (n+1 entries, out[n] = total),
// hand-written reduce-then-scan in scan.hip (in != out).
void selftest_math(int op, int64_t n, const double *x, const double *y, double *out, hipStream_t s);
void selftest_scan(int64_t n, int shift, const int64_t *in, int64_t *out, hipStream_t s);
// mail (optional): a device-visible host word that also receives out[n]
// (the total), written by the scan's last element -- read after a stream
// sync without a copy launch
void exclusive_scan_i64(const int64_t *in, int64_t *out, int64_t n, DevBuf<unsigned char> &tmp, hipStream_t s,
                        int64_t *mail = nullptr);
// up to three device uint32 counters into device-visible host words (one launch)
void mail_counters(const unsigned int *a, const unsigned int *b, const unsigned int *c, int64_t *mail, hipStream_t s);
// perm = footprint indices with every non-circle before every circle (order
// within each part unspecified): per-footprint kernels then run one kind's
// code path per wave.
void partition_polygons_first(const int32_t *kind, uint32_t *perm, unsigned long long *nsel, int64_t n,
                              DevBuf<unsigned char> &tmp, DevBuf<unsigned char> &tmp2, hipStream_t s);

}  // namespace dss
