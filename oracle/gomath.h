/* ORACLE / TEST INFRASTRUCTURE ONLY -- never linked into the product path.
 *
 * Restatement of the pure-Go math routines that golang/geo calls on the
 * covering path.  Go 1.14 on amd64 (reference Dockerfile:6, golang:1.14.3)
 * implements Sin, Cos, Tan, Atan, Atan2 and Asin in pure Go (Cephes ports,
 * math/stubs_amd64.s only jumps to them), and never contracts a*b+c into an
 * FMA on amd64.  Sqrt is the IEEE instruction.  This file must therefore be
 * compiled with -ffp-contract=off and without -ffast-math.
 *
 * Followed: Go 1.14 math/sin.go (sin, cos), math/tan.go (tan), math/atan.go
 * (xatan, satan, atan), math/atan2.go (atan2), math/asin.go (asin),
 * math/trig_reduce.go (trigReduce, mPi4).
 */
#ifndef DSS_ORACLE_GOMATH_H
#define DSS_ORACLE_GOMATH_H

#include <math.h>
#include <stdint.h>
#include <string.h>

#include "go_constants.h"

static const uint64_t orc_mpi4[20] = ORC_MPI4_INIT;

static inline uint64_t orc_f2u(double x) { uint64_t u; memcpy(&u, &x, 8); return u; }
static inline double orc_u2f(uint64_t u) { double x; memcpy(&x, &u, 8); return x; }

/* math/trig_reduce.go: Payne-Hanek reduction for x >= 2^29. */
static void go_trig_reduce(double x, uint64_t *jout, double *zout)
{
    const double PI4 = ORC_PI_4;
    if (x < PI4) { *jout = 0; *zout = x; return; }
    uint64_t ix = orc_f2u(x);
    int exp = (int)((ix >> 52) & 0x7ff) - 1023 - 52;
    ix &= ~((uint64_t)0x7ff << 52);
    ix |= (uint64_t)1 << 52;
    unsigned digit = (unsigned)(exp + 61) / 64, bitshift = (unsigned)(exp + 61) % 64;
#define ORC_SHR(v, s) ((s) >= 64 ? 0ULL : ((v) >> (s)))
    uint64_t z0 = (orc_mpi4[digit] << bitshift) | ORC_SHR(orc_mpi4[digit + 1], 64 - bitshift);
    uint64_t z1 = (orc_mpi4[digit + 1] << bitshift) | ORC_SHR(orc_mpi4[digit + 2], 64 - bitshift);
    uint64_t z2 = (orc_mpi4[digit + 2] << bitshift) | ORC_SHR(orc_mpi4[digit + 3], 64 - bitshift);
    unsigned __int128 p2 = (unsigned __int128)z2 * ix;
    unsigned __int128 p1 = (unsigned __int128)z1 * ix;
    uint64_t z2hi = (uint64_t)(p2 >> 64);
    uint64_t z1hi = (uint64_t)(p1 >> 64), z1lo = (uint64_t)p1;
    uint64_t z0lo = z0 * ix;
    uint64_t lo = z1lo + z2hi;
    uint64_t c = lo < z1lo;
    uint64_t hi = z0lo + z1hi + c;
    uint64_t j = hi >> 61;
    hi = hi << 3 | lo >> 61;
    unsigned lz = (unsigned)__builtin_clzll(hi);
    uint64_t e = (uint64_t)(1023 - (lz + 1));
    hi = (hi << (lz + 1)) | ORC_SHR(lo, 64 - (lz + 1));
    hi >>= 64 - 52;
    hi |= e << 52;
#undef ORC_SHR
    double z = orc_u2f(hi);
    if (j & 1) { j++; j &= 7; z--; }
    *jout = j;
    *zout = z * PI4;
}

static const double orc_sin_c[6] = {
    1.58962301576546568060e-10, -2.50507477628578072866e-8, 2.75573136213857245213e-6,
    -1.98412698295895385996e-4, 8.33333333332211858878e-3, -1.66666666666666307295e-1,
};
static const double orc_cos_c[6] = {
    -1.13585365213876817300e-11, 2.08757008419747316778e-9, -2.75573141792967388112e-7,
    2.48015872888517045348e-5, -1.38888888888730564116e-3, 4.16666666666665929218e-2,
};
#define ORC_PI4A 7.85398125648498535156e-1
#define ORC_PI4B 3.77489470793079817668e-8
#define ORC_PI4C 2.69515142907905952645e-15
#define ORC_REDUCE_THRESHOLD ((double)(1 << 29))

/* math/sin.go: cos */
static double go_cos(double x)
{
    if (isnan(x) || isinf(x)) return NAN;
    int sign = 0;
    x = fabs(x);
    uint64_t j;
    double y, z;
    if (x >= ORC_REDUCE_THRESHOLD) {
        go_trig_reduce(x, &j, &z);
    } else {
        j = (uint64_t)(x * ORC_FOUR_OVER_PI);
        y = (double)j;
        if (j & 1) { j++; y++; }
        j &= 7;
        z = ((x - y * ORC_PI4A) - y * ORC_PI4B) - y * ORC_PI4C;
    }
    if (j > 3) { j -= 4; sign = !sign; }
    if (j > 1) sign = !sign;
    double zz = z * z;
    if (j == 1 || j == 2) {
        y = z + z * zz * ((((((orc_sin_c[0] * zz) + orc_sin_c[1]) * zz + orc_sin_c[2]) * zz + orc_sin_c[3]) * zz + orc_sin_c[4]) * zz + orc_sin_c[5]);
    } else {
        y = 1.0 - 0.5 * zz + zz * zz * ((((((orc_cos_c[0] * zz) + orc_cos_c[1]) * zz + orc_cos_c[2]) * zz + orc_cos_c[3]) * zz + orc_cos_c[4]) * zz + orc_cos_c[5]);
    }
    if (sign) y = -y;
    return y;
}

/* math/sin.go: sin */
static double go_sin(double x)
{
    if (x == 0 || isnan(x)) return x;
    if (isinf(x)) return NAN;
    int sign = 0;
    if (x < 0) { x = -x; sign = 1; }
    uint64_t j;
    double y, z;
    if (x >= ORC_REDUCE_THRESHOLD) {
        go_trig_reduce(x, &j, &z);
    } else {
        j = (uint64_t)(x * ORC_FOUR_OVER_PI);
        y = (double)j;
        if (j & 1) { j++; y++; }
        j &= 7;
        z = ((x - y * ORC_PI4A) - y * ORC_PI4B) - y * ORC_PI4C;
    }
    if (j > 3) { sign = !sign; j -= 4; }
    double zz = z * z;
    if (j == 1 || j == 2) {
        y = 1.0 - 0.5 * zz + zz * zz * ((((((orc_cos_c[0] * zz) + orc_cos_c[1]) * zz + orc_cos_c[2]) * zz + orc_cos_c[3]) * zz + orc_cos_c[4]) * zz + orc_cos_c[5]);
    } else {
        y = z + z * zz * ((((((orc_sin_c[0] * zz) + orc_sin_c[1]) * zz + orc_sin_c[2]) * zz + orc_sin_c[3]) * zz + orc_sin_c[4]) * zz + orc_sin_c[5]);
    }
    if (sign) y = -y;
    return y;
}

/* math/tan.go: tan */
static double go_tan(double x)
{
    static const double P[3] = {-1.30936939181383777646e4, 1.15351664838587416140e6, -1.79565251976484877988e7};
    static const double Q[5] = {1.0, 1.36812963470692954678e4, -1.32089234440210967447e6, 2.50083801823357915839e7, -5.38695755929454629881e7};
    if (x == 0 || isnan(x)) return x;
    if (isinf(x)) return NAN;
    int sign = 0;
    if (x < 0) { x = -x; sign = 1; }
    uint64_t j;
    double y, z;
    if (x >= ORC_REDUCE_THRESHOLD) {
        go_trig_reduce(x, &j, &z);
    } else {
        j = (uint64_t)(x * ORC_FOUR_OVER_PI);
        y = (double)j;
        if (j & 1) { j++; y++; }
        z = ((x - y * ORC_PI4A) - y * ORC_PI4B) - y * ORC_PI4C;
    }
    double zz = z * z;
    if (zz > 1e-14) {
        y = z + z * (zz * (((P[0] * zz) + P[1]) * zz + P[2]) / ((((zz + Q[1]) * zz + Q[2]) * zz + Q[3]) * zz + Q[4]));
    } else {
        y = z;
    }
    if (j & 2) y = -1 / y;
    if (sign) y = -y;
    return y;
}

/* math/atan.go */
static double go_xatan(double x)
{
    const double P0 = -8.750608600031904122785e-01, P1 = -1.615753718733365076637e+01,
                 P2 = -7.500855792314704667340e+01, P3 = -1.228866684490136173410e+02,
                 P4 = -6.485021904942025371773e+01;
    const double Q0 = +2.485846490142306297962e+01, Q1 = +1.650270098316988542046e+02,
                 Q2 = +4.328810604912902668951e+02, Q3 = +4.853903996359136964868e+02,
                 Q4 = +1.945506571482613964425e+02;
    double z = x * x;
    z = z * ((((P0 * z + P1) * z + P2) * z + P3) * z + P4) / (((((z + Q0) * z + Q1) * z + Q2) * z + Q3) * z + Q4);
    z = x * z + x;
    return z;
}

static double go_satan(double x)
{
    const double Morebits = 6.123233995736765886130e-17;
    const double Tan3pio8 = 2.41421356237309504880;
    if (x <= 0.66) return go_xatan(x);
    if (x > Tan3pio8) return ORC_PI_2 - go_xatan(1 / x) + Morebits;
    return ORC_PI_4 + go_xatan((x - 1) / (x + 1)) + 0.5 * Morebits;
}

static double go_atan(double x)
{
    if (x == 0) return x;
    if (x > 0) return go_satan(x);
    return -go_satan(-x);
}

/* math/atan2.go */
static double go_atan2(double y, double x)
{
    if (isnan(y) || isnan(x)) return NAN;
    if (y == 0) {
        if (x >= 0 && !signbit(x)) return copysign(0, y);
        return copysign(ORC_PI, y);
    }
    if (x == 0) return copysign(ORC_PI_2, y);
    if (isinf(x)) {
        if (x > 0) {
            if (isinf(y)) return copysign(ORC_PI_4, y);
            return copysign(0, y);
        }
        if (isinf(y)) return copysign(ORC_PI3_4, y);
        return copysign(ORC_PI, y);
    }
    if (isinf(y)) return copysign(ORC_PI_2, y);
    double q = go_atan(y / x);
    if (x < 0) {
        if (q <= 0) return q + ORC_PI;
        return q - ORC_PI;
    }
    return q;
}

/* math/asin.go */
static double go_asin(double x)
{
    if (x == 0) return x;
    int sign = 0;
    if (x < 0) { x = -x; sign = 1; }
    if (x > 1) return NAN;
    double temp = sqrt(1 - x * x);
    if (x > 0.7) temp = ORC_PI_2 - go_satan(temp / x);
    else temp = go_satan(x / temp);
    if (sign) temp = -temp;
    return temp;
}

/* Go's math.Max / math.Min special-case +-Inf, NaN and signed zeros. */
static inline double go_max(double x, double y)
{
    if (isinf(x) && x > 0) return x;
    if (isinf(y) && y > 0) return y;
    if (isnan(x) || isnan(y)) return NAN;
    if (x == 0 && x == y) return signbit(x) ? y : x;
    return x > y ? x : y;
}
static inline double go_min(double x, double y)
{
    if (isinf(x) && x < 0) return x;
    if (isinf(y) && y < 0) return y;
    if (isnan(x) || isnan(y)) return NAN;
    if (x == 0 && x == y) return signbit(x) ? x : y;
    return x < y ? x : y;
}

#endif
