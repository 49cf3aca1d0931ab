// glibc's logf / expf (glibc >= 2.28, the image's 2.35), restated for the device so that the
// draws that feed them arbitrary f32 arguments -- the FromBeta Dirichlet of rand_distr 0.5.1,
// Cheng's Beta algorithm BC (rand_distr.h) -- reproduce what Rust's f32::ln / f32::exp return on
// the reference's Linux hosts (Rust calls the platform libm).  Neither function is correctly
// rounded (logf differs from the correctly rounded value on ~2e-4 of its inputs, expf on ~8e-5),
// so the device's own logf / expf cannot stand in for them.
//
// The algorithms are the published ones glibc took from Arm's optimized-routines
// (sysdeps/ieee754/flt-32/e_logf.c, e_expf.c; data in e_logf_data.c, e_exp2f_data.c):
//   logf  x = 2^k z, z in [0x3f330000, 2 * 0x3f330000) split into 16 subintervals by the top
//         fraction bits; r = z / c - 1 with c near the subinterval's centre (invc, logc
//         tabulated); log x = log1p(r) + log c + k ln 2, log1p by a degree-3 polynomial, all in
//         double, rounded once to float;
//   expf  z = x * 32 / ln 2 rounded to an integer k by the 0x1.8p52 shift, r = z - k;
//         exp x = 2^(k/32) * 2^(r/32), the first from a 32-entry table with k's high bits added
//         to the exponent, the second by a cubic in r; double throughout, rounded once.
// On x86-64 glibc selects its FMA builds (e_logf-fma.c / e_expf-fma.c, compiled with -mfma)
// whenever the CPU has FMA and AVX2 -- both the build container's Xeon and the GPU box's EPYC do
// -- and GCC contracts every multiply-add of those sources.  The restatement writes those fused
// multiply-adds explicitly (fma), and nothing else may be contracted: the library is compiled
// with -ffp-contract=off.  tests/native/libm_check.cpp compares both functions with the host's
// glibc on all 2^32 inputs; tests/test_gpu_parity.py::test_device_libm_f32 does the same for
// the device build through dk_f32_libm_async.
#pragma once
#include <math.h>
#include <stdint.h>
#include "common.h"

namespace dk {
namespace lm {

// e_logf_data.c: {invc, logc} per subinterval, ln 2, and the log1p polynomial
static constexpr double LOGF_INVC[16] = {
    0x1.661ec79f8f3bep+0, 0x1.571ed4aaf883dp+0, 0x1.49539f0f010bp+0,  0x1.3c995b0b80385p+0,
    0x1.30d190c8864a5p+0, 0x1.25e227b0b8eap+0,  0x1.1bb4a4a1a343fp+0, 0x1.12358f08ae5bap+0,
    0x1.0953f419900a7p+0, 0x1p+0,               0x1.e608cfd9a47acp-1, 0x1.ca4b31f026aap-1,
    0x1.b2036576afce6p-1, 0x1.9c2d163a1aa2dp-1, 0x1.886e6037841edp-1, 0x1.767dcf5534862p-1};
static constexpr double LOGF_LOGC[16] = {
    -0x1.57bf7808caadep-2, -0x1.2bef0a7c06ddbp-2, -0x1.01eae7f513a67p-2, -0x1.b31d8a68224e9p-3,
    -0x1.6574f0ac07758p-3, -0x1.1aa2bc79c81p-3,   -0x1.a4e76ce8c0e5ep-4, -0x1.1973c5a611cccp-4,
    -0x1.252f438e10c1ep-5, 0x0p+0,                0x1.aa5aa5df25984p-5,  0x1.c5e53aa362eb4p-4,
    0x1.526e57720db08p-3,  0x1.bc2860d22477p-3,   0x1.1058bc8a07ee1p-2,  0x1.4043057b6ee09p-2};
static constexpr double LOGF_LN2 = 0x1.62e42fefa39efp-1;
static constexpr double LOGF_A0 = -0x1.00ea348b88334p-2, LOGF_A1 = 0x1.5575b0be00b6ap-2,
                        LOGF_A2 = -0x1.ffffef20a4123p-2;

// e_exp2f_data.c: bits of 2^(i/32) minus i << 47, the scaled 1/ln2, the shift and the cubic
static constexpr uint64_t EXPF_TAB[32] = {
    0x3ff0000000000000ull, 0x3fefd9b0d3158574ull, 0x3fefb5586cf9890full, 0x3fef9301d0125b51ull,
    0x3fef72b83c7d517bull, 0x3fef54873168b9aaull, 0x3fef387a6e756238ull, 0x3fef1e9df51fdee1ull,
    0x3fef06fe0a31b715ull, 0x3feef1a7373aa9cbull, 0x3feedea64c123422ull, 0x3feece086061892dull,
    0x3feebfdad5362a27ull, 0x3feeb42b569d4f82ull, 0x3feeab07dd485429ull, 0x3feea47eb03a5585ull,
    0x3feea09e667f3bcdull, 0x3fee9f75e8ec5f74ull, 0x3feea11473eb0187ull, 0x3feea589994cce13ull,
    0x3feeace5422aa0dbull, 0x3feeb737b0cdc5e5ull, 0x3feec49182a3f090ull, 0x3feed503b23e255dull,
    0x3feee89f995ad3adull, 0x3feeff76f2fb5e47ull, 0x3fef199bdd85529cull, 0x3fef3720dcef9069ull,
    0x3fef5818dcfba487ull, 0x3fef7c97337b9b5full, 0x3fefa4afa2a490daull, 0x3fefd0765b6e4540ull};
static constexpr double EXPF_INVLN2N = 0x1.71547652b82fep+0 * 32;
static constexpr double EXPF_SHIFT = 0x1.8p+52;
static constexpr double EXPF_C0 = 0x1.c6af84b912394p-5 / 32 / 32 / 32, EXPF_C1 = 0x1.ebfce50fac4f3p-3 / 32 / 32,
                        EXPF_C2 = 0x1.62e42ff0c52d6p-1 / 32;

DK_HD uint32_t f2u(float x) { return __builtin_bit_cast(uint32_t, x); }
DK_HD float u2f(uint32_t u) { return __builtin_bit_cast(float, u); }

// e_logf.c __logf
DK_HD float logf_glibc(float x) {
    uint32_t ix = f2u(x);
    if (ix == 0x3f800000u) return 0.0f;
    if (ix - 0x00800000u >= 0x7f800000u - 0x00800000u) {
        if (ix * 2 == 0) return -INFINITY;                                 // __math_divzerof(1)
        if (ix == 0x7f800000u) return x;                                   // log(inf)
        if ((ix & 0x80000000u) || ix * 2 >= 0xff000000u) return (x - x) / (x - x);   // __math_invalidf
        ix = f2u(x * 0x1p23f);                                             // subnormal: normalise
        ix -= 23u << 23;
    }
    const uint32_t tmp = ix - 0x3f330000u;
    const int i = (int)((tmp >> (23 - 4)) % 16);
    const int k = (int32_t)tmp >> 23;
    const uint32_t iz = ix - (tmp & 0x1ffu << 23);
    const double invc = LOGF_INVC[i], logc = LOGF_LOGC[i];
    const double z = (double)u2f(iz);
    const double r = __builtin_fma(z, invc, -1.0);
    const double y0 = __builtin_fma((double)k, LOGF_LN2, logc);
    const double r2 = r * r;
    double y = __builtin_fma(LOGF_A1, r, LOGF_A2);
    y = __builtin_fma(LOGF_A0, r2, y);
    y = __builtin_fma(y, r2, y0 + r);
    return (float)y;
}

// e_expf.c __expf (no TOINT intrinsics on x86-64: the shift rounds z)
DK_HD float expf_glibc(float x) {
    const double xd = (double)x;
    const uint32_t abstop = (f2u(x) >> 20) & 0x7ff;
    if (abstop >= (f2u(88.0f) >> 20)) {
        if (f2u(x) == f2u(-INFINITY)) return 0.0f;
        if (abstop >= (f2u(INFINITY) >> 20)) return x + x;
        if (x > 0x1.62e42ep6f) return INFINITY;                            // __math_oflowf
        if (x < -0x1.9fe368p6f) return 0.0f;                               // __math_uflowf
    }
    const double kd0 = __builtin_fma(EXPF_INVLN2N, xd, EXPF_SHIFT);        // z + shift, z = InvLn2N x
    const uint64_t ki = __builtin_bit_cast(uint64_t, kd0);
    const double kd = kd0 - EXPF_SHIFT;
    const double r = __builtin_fma(EXPF_INVLN2N, xd, -kd);                 // z - kd
    uint64_t t = EXPF_TAB[ki % 32];
    t += ki << (52 - 5);
    const double s = __builtin_bit_cast(double, t);
    const double zc = __builtin_fma(EXPF_C0, r, EXPF_C1);
    const double r2 = r * r;
    double y = __builtin_fma(EXPF_C2, r, 1.0);
    y = __builtin_fma(zc, r2, y);
    y = y * s;
    return (float)y;
}

}  // namespace lm
}  // namespace dk
