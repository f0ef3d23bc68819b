// Diagnostics: evaluate the device restatements of Go's math routines and the
// S2 projections on host-supplied inputs, so tests can compare them bit for bit
// with the CPU oracle (the covering is only bit-exact if these are).
#include <hip/hip_runtime.h>

#include "common.hpp"
#include "s2dev.cuh"

namespace dss {
namespace {
__global__ void k_math(int op, int64_t n, const double *x, const double *y, double *out)
{
    int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    double a = x[i], b = y ? y[i] : 0.0, r = 0;
    using namespace gomath;
    switch (op) {
    case 0: r = go_sin(a); break;
    case 1: r = go_cos(a); break;
    case 2: r = go_tan(a); break;
    case 3: r = go_atan(a); break;
    case 4: r = go_atan2(a, b); break;
    case 5: r = go_asin(a); break;
    case 6: r = __builtin_sqrt(a); break;
    case 7: r = a / b; break;
    case 8: r = s2::st_to_uv(a); break;
    case 9: r = s2::uv_to_st(a); break;
    case 10: { s2::V3 p = s2::point_from_degrees(a, b); r = p.x + 0 * p.y; out[i] = r; return; }
    default: r = 0;
    }
    out[i] = r;
}
}  // namespace

void selftest_math(int op, int64_t n, const double *x, const double *y, double *out, hipStream_t s)
{
    DevBuf<double> dx, dy, dout;
    double *px = dx.ensure(n), *py = y ? dy.ensure(n) : nullptr, *po = dout.ensure(n);
    DSS_HIP(hipMemcpyAsync(px, x, sizeof(double) * n, hipMemcpyHostToDevice, s));
    if (y) DSS_HIP(hipMemcpyAsync(py, y, sizeof(double) * n, hipMemcpyHostToDevice, s));
    hipLaunchKernelGGL(k_math, dim3(grid_for(n, 256)), dim3(256), 0, s, op, n, px, py, po);
    DSS_HIP(hipMemcpyAsync(out, po, sizeof(double) * n, hipMemcpyDeviceToHost, s));
    DSS_HIP(hipStreamSynchronize(s));
}

// Exclusive scan of n host int64 values through the device scan, with the
// input placed `shift` elements into its buffer (shift odd: a pointer that is
// 8- but not 16-byte aligned, as call sites that scan inside shared buffers
// pass).  out: n + 1 values.
void selftest_scan(int64_t n, int shift, const int64_t *in, int64_t *out, hipStream_t s)
{
    DevBuf<int64_t> din, dout;
    DevBuf<unsigned char> tmp;
    int64_t *pi = din.ensure(n + shift + 1) + shift, *po = dout.ensure(n + 1);
    if (n) DSS_HIP(hipMemcpyAsync(pi, in, sizeof(int64_t) * n, hipMemcpyHostToDevice, s));
    exclusive_scan_i64(pi, po, n, tmp, s);
    DSS_HIP(hipMemcpyAsync(out, po, sizeof(int64_t) * (n + 1), hipMemcpyDeviceToHost, s));
    DSS_HIP(hipStreamSynchronize(s));
}
}  // namespace dss
