// The single-precision log and exp of the reference's host association (filter_overlaps,
// src/SfM_CUDA/tsdf.cu:318,329,343: `log(max(float, float))`, `exp(float / uint32)` in host
// code, i.e. the C library's logf / expf), restated so that the device computes the very
// same f32 values: the association decisions compare sums and exponentials of these values
// bit for bit.
//
// The host library of this platform is glibc 2.35 on x86-64, whose logf/expf are IFUNCs that
// select an FMA-compiled variant on CPUs with FMA + AVX2.  Both follow the published
// algorithms of Arm's optimized-routines (logf: 16-interval table + degree-3 polynomial in
// double; expf: 2^(k/32) table + degree-3 polynomial in double); the FMA variant contracts
// specific multiply-adds, which decides the last bit of some results.  The functions below
// evaluate the same double-precision expression graph with the same fused operations (read
// from the FMA variant's instruction sequence), and the same constants (the tables of that
// library, tools/gen_libm_consts.py).  glibc is not correctly rounded: 142 176 of the 36.9 M
// floats in [0.05, 1] get a logf result other than the correctly rounded one, and 71 603 of
// the 1.08 G floats in [log 0.05, 0] an expf result, so the device cannot use its own
// (correctly rounded or not) log/exp.  Checked exhaustively against the host library over the
// association's whole input domain: on the CPU (tests/test_libm_port.py) and on the GPU
// (tests/test_gpu_assoc_exact.py).
//
// Device code under HIP; plain C++ otherwise (`SEMTSDF_HD` is then empty), so the CPU test
// compiles this header with g++.  Requires -ffp-contract=off (every fused operation is an
// explicit fma()).
#pragma once
#include <stdint.h>
#include <string.h>
#include <math.h>

#if defined(__HIPCC__)
#define SEMTSDF_HD __device__
#else
#define SEMTSDF_HD
#endif

namespace semtsdf {
namespace glibc {

SEMTSDF_HD inline uint32_t f2u(float f) { uint32_t u; memcpy(&u, &f, 4); return u; }
SEMTSDF_HD inline float u2f(uint32_t u) { float f; memcpy(&f, &u, 4); return f; }
SEMTSDF_HD inline uint64_t d2u(double d) { uint64_t u; memcpy(&u, &d, 8); return u; }
SEMTSDF_HD inline double u2d(uint64_t u) { double d; memcpy(&d, &u, 8); return d; }

// logf: x = 2^k z, z in [0x3f330000, 2 * 0x3f330000) as a float bit pattern; c_i near the
// centre of subinterval i; log(x) = k ln2 + log(c_i) + log1p(z / c_i - 1).
struct LogfEntry { double invc, logc; };
#if defined(__HIPCC__)
__device__ __constant__
#endif
static const LogfEntry kLogfTab[16] = {
    {0x1.661ec79f8f3bep+0, -0x1.57bf7808caadep-2}, {0x1.571ed4aaf883dp+0, -0x1.2bef0a7c06ddbp-2},
    {0x1.49539f0f010b0p+0, -0x1.01eae7f513a67p-2}, {0x1.3c995b0b80385p+0, -0x1.b31d8a68224e9p-3},
    {0x1.30d190c8864a5p+0, -0x1.6574f0ac07758p-3}, {0x1.25e227b0b8ea0p+0, -0x1.1aa2bc79c8100p-3},
    {0x1.1bb4a4a1a343fp+0, -0x1.a4e76ce8c0e5ep-4}, {0x1.12358f08ae5bap+0, -0x1.1973c5a611cccp-4},
    {0x1.0953f419900a7p+0, -0x1.252f438e10c1ep-5}, {0x1.0000000000000p+0, 0x0.0p+0},
    {0x1.e608cfd9a47acp-1, 0x1.aa5aa5df25984p-5},  {0x1.ca4b31f026aa0p-1, 0x1.c5e53aa362eb4p-4},
    {0x1.b2036576afce6p-1, 0x1.526e57720db08p-3},  {0x1.9c2d163a1aa2dp-1, 0x1.bc2860d224770p-3},
    {0x1.886e6037841edp-1, 0x1.1058bc8a07ee1p-2},  {0x1.767dcf5534862p-1, 0x1.4043057b6ee09p-2},
};
constexpr double kLogfLn2 = 0x1.62e42fefa39efp-1;
constexpr double kLogfA0 = -0x1.00ea348b88334p-2;
constexpr double kLogfA1 = 0x1.5575b0be00b6ap-2;
constexpr double kLogfA2 = -0x1.ffffef20a4123p-2;

// logf of a positive normal or subnormal float (the association's arguments lie in
// [prior_mrcnn_err_rate, 1]); zero, negative, inf and NaN follow IEEE log.
SEMTSDF_HD inline float logf(float x) {
    uint32_t ix = f2u(x);
    if (ix == 0x3f800000u) return 0.0f;
    if (ix - 0x00800000u >= 0x7f800000u - 0x00800000u) {
        if (ix * 2u == 0u) return -INFINITY;
        if (ix == 0x7f800000u) return x;
        if ((ix & 0x80000000u) || ix * 2u >= 0xff000000u) return NAN;
        ix = f2u(x * 0x1p23f) - (23u << 23);  // subnormal: normalise
    }
    const uint32_t tmp = ix - 0x3f330000u;
    const int i = (int)((tmp >> 19) & 15u);
    const int k = (int32_t)tmp >> 23;
    const uint32_t iz = ix - (tmp & 0xff800000u);
    const double invc = kLogfTab[i].invc, logc = kLogfTab[i].logc;
    const double z = (double)u2f(iz);
    const double r = fma(z, invc, -1.0);
    const double y0 = fma((double)k, kLogfLn2, logc);
    const double r2 = r * r;
    double y = fma(r, kLogfA1, kLogfA2);
    y = fma(r2, kLogfA0, y);
    const double t = r + y0;
    y = fma(r2, y, t);
    return (float)y;
}

// expf: k = round(x 32 / ln2), r = x 32 / ln2 - k, exp(x) = 2^(k/32) * poly(r).
#if defined(__HIPCC__)
__device__ __constant__
#endif
static const uint64_t kExpfTab[32] = {
    0x3ff0000000000000ull, 0x3fefd9b0d3158574ull, 0x3fefb5586cf9890full, 0x3fef9301d0125b51ull,
    0x3fef72b83c7d517bull, 0x3fef54873168b9aaull, 0x3fef387a6e756238ull, 0x3fef1e9df51fdee1ull,
    0x3fef06fe0a31b715ull, 0x3feef1a7373aa9cbull, 0x3feedea64c123422ull, 0x3feece086061892dull,
    0x3feebfdad5362a27ull, 0x3feeb42b569d4f82ull, 0x3feeab07dd485429ull, 0x3feea47eb03a5585ull,
    0x3feea09e667f3bcdull, 0x3fee9f75e8ec5f74ull, 0x3feea11473eb0187ull, 0x3feea589994cce13ull,
    0x3feeace5422aa0dbull, 0x3feeb737b0cdc5e5ull, 0x3feec49182a3f090ull, 0x3feed503b23e255dull,
    0x3feee89f995ad3adull, 0x3feeff76f2fb5e47ull, 0x3fef199bdd85529cull, 0x3fef3720dcef9069ull,
    0x3fef5818dcfba487ull, 0x3fef7c97337b9b5full, 0x3fefa4afa2a490daull, 0x3fefd0765b6e4540ull,
};
constexpr double kExpfShift = 0x1.8p+52;
constexpr double kExpfInvLn2N = 0x1.71547652b82fep+5;
constexpr double kExpfC0 = 0x1.c6af84b912394p-20;
constexpr double kExpfC1 = 0x1.ebfce50fac4f3p-13;
constexpr double kExpfC2 = 0x1.62e42ff0c52d6p-6;

// expf for |x| below 80 (the library's bit-pattern test: top 12 bits of |x| <= 0x42a; no
// overflow or underflow handling is needed there); the association's arguments are averages
// of logs in [log(prior), 0].  Beyond it the result is exp computed in double (not used).
SEMTSDF_HD inline float expf(float x) {
    const double xd = (double)x;
    const uint32_t abstop = (f2u(x) >> 20) & 0x7ffu;
    if (abstop > 0x42au) return (float)exp(xd);
    const double kd = fma(kExpfInvLn2N, xd, kExpfShift);
    const uint64_t ki = d2u(kd);
    const double kd2 = kd - kExpfShift;
    const double r = fma(kExpfInvLn2N, xd, -kd2);
    const double s = u2d(kExpfTab[ki & 31u] + (ki << 47));
    const double z = fma(r, kExpfC0, kExpfC1);
    const double r2 = r * r;
    double y = fma(r, kExpfC2, 1.0);
    y = fma(z, r2, y);
    y = y * s;
    return (float)y;
}

}  // namespace glibc
}  // namespace semtsdf
