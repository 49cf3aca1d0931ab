// rand_distr 0.5.1 (Cargo.lock:1948-1949) Dirichlet<f32> on the search's SmallRng, for the
// AlphaZero root noise: `Dirichlet::new([dirichlet_alpha; 39]).unwrap().sample(rng)`
// (rs-doko-alpha-zero/src/alpha_zero/mcts/async_mcts.rs:111-113).  The crate is not vendored
// under /root/reference; this restates its published algorithms in its draw order:
//   Dirichlet::new      alpha not > 0 or not finite: error; every alpha <= 0.1 -> FromBeta,
//                       else FromGamma: one Gamma(alpha, 1) per component, in index order,
//                       each normalised by 1 / sum (f32, sequential sum)
//   FromBeta            stick breaking: beta_i ~ Beta(alpha_i, alpha_{i+1} + .. + alpha_{N-1})
//                       (reverse cumulative sums in f32 from the end); draw_i = acc * beta_i,
//                       acc *= 1 - beta_i; draw_{N-1} = acc
//   Beta::new(a, b)     Cheng (1978): the smaller parameter > 1 -> algorithm BB, else BC (with
//                       the larger as `a`); StandardUniform<f32> u1, u2 per trial; w / (b + w),
//                       or b / (b + w) when the parameters were switched
//   Gamma::new          shape == 1 -> Exp(1 / scale); shape < 1 -> GammaSmallShape; else
//                       GammaLargeShape (Marsaglia & Tsang 2000)
//   GammaSmallShape     u = Open01 FIRST, then large(shape + 1) * u^(1 / shape)
//   GammaLargeShape     d = shape - 1/3, c = 1 / sqrt(9 d); loop { x = StandardNormal;
//                       v = (1 + c x)^3 (retry if 1 + c x <= 0); u = Open01; accept if
//                       u < 1 - 0.0331 x^4 or ln u < x^2 / 2 + d (1 - v + ln v) } -> d v scale
//   StandardNormal<f32> the f64 ziggurat (256 layers, symmetric, tail by Marsaglia's method)
//                       cast to f32;  Exp1<f32> likewise (asymmetric, tail R - ln U)
//   Open01<f32>         (next_u32 >> 9) as the mantissa of [1, 2), minus 1 - 2^-24
//   Open01<f64>         (next_u64 >> 12) likewise, minus 1 - 2^-53
//   StandardUniform f32 (next_u32 >> 8) * 2^-24
//   StandardUniform f64 (next_u64 >> 11) * 2^-53                   (rand 0.9 distr/float.rs)
// All f32 arithmetic is in the crate's operation order (the library is built with
// -ffp-contract=off, as Rust never contracts).  Libm values:
//   * u^(1 / shape) and ln u for an Open01<f32> u: u takes only 2^23 values, so the context
//     passes tables of the glibc powf / logf values (`Open01Tab`, built on the host like the
//     ln(N) table of the UCT search); bit-exact for every draw;
//   * ln v (the acceptance test's right side), the ziggurat pdfs (f64 exp) and the tails (f64
//     ln): (float)log((double)v), exp / log in f64.  These feed comparisons (or an f64 value
//     rounded to f32): a last-bit difference from glibc flips an outcome only when the two
//     sides are within an ulp.  tests/native/dirichlet_check.cpp compares this code with the
//     oracle (glibc throughout) draw for draw.
// Beta's f32 ln / exp of arbitrary arguments are glibc's logf / expf restated (libm_f32.h, checked
// against glibc on every f32 input).
// Parity unpinned: the reference holds no vector for any of these draws.
#pragma once
#include <float.h>
#include <math.h>
#include "common.h"
#include "libm_f32.h"
#include "rng.h"
#include "ziggurat_tables.h"

namespace dk {
namespace rd {

DK_HD double f64_bits(uint64_t b) { return __builtin_bit_cast(double, b); }
DK_HD float f32_bits(uint32_t b) { return __builtin_bit_cast(float, b); }

// Open01<f32>; *k = the 23-bit fraction (the index of the glibc tables)
DK_HD float open01_f32(Rng& r, uint32_t* k) {
    const uint32_t f = r.next_u32() >> 9;
    *k = f;
    return f32_bits(f | 0x3F800000u) - (1.0f - FLT_EPSILON / 2.0f);
}
DK_HD double open01_f64(Rng& r) { return f64_bits((r.next_u64() >> 12) | 0x3FF0000000000000ull) - (1.0 - DBL_EPSILON / 2.0); }
DK_HD double std_f64(Rng& r) { return (double)(r.next_u64() >> 11) * 0x1p-53; }
DK_HD float std_f32(Rng& r) { return (float)(r.next_u32() >> 8) * 0x1p-24f; }   // StandardUniform<f32>

// utils.rs ziggurat(): i = the low 8 bits, u from the high 52 bits
template <bool SYM>
DK_HD double ziggurat(Rng& r, const double* X, const double* F) {
    for (;;) {
        const uint64_t bits = r.next_u64();
        const uint32_t i = (uint32_t)bits & 0xFFu;
        const double u = SYM ? f64_bits((bits >> 12) | 0x4000000000000000ull) - 3.0
                             : f64_bits((bits >> 12) | 0x3FF0000000000000ull) - (1.0 - DBL_EPSILON / 2.0);
        const double x = u * X[i];
        const double tx = SYM ? fabs(x) : x;
        if (tx < X[i + 1]) return x;
        if (i == 0) {
            if constexpr (SYM) {   // StandardNormal zero_case: the tail beyond R
                double xt = 1.0, y = 0.0;
                while (-2.0 * y < xt * xt) {
                    const double x_ = open01_f64(r);
                    const double y_ = open01_f64(r);
                    xt = log(x_) / zig::NORM_R;
                    y = log(y_);
                }
                return u < 0.0 ? xt - zig::NORM_R : zig::NORM_R - xt;
            } else {               // Exp1 zero_case
                return zig::EXP_R - log(std_f64(r));
            }
        }
        const double pdf = SYM ? exp(-x * x / 2.0) : exp(-x);
        if (F[i + 1] + (F[i] - F[i + 1]) * std_f64(r) < pdf) return x;
    }
}
DK_HD float normal_f32(Rng& r) { return (float)ziggurat<true>(r, zig::NORM_X, zig::NORM_F); }
DK_HD float exp1_f32(Rng& r) { return (float)ziggurat<false>(r, zig::EXP_X, zig::EXP_F); }

// glibc powf(u, 1 / shape) and logf(u) for the 2^23 Open01<f32> values (index = fraction)
struct Open01Tab {
    const float* pw;   // powf(u_k, inv_shape) (small shapes only)
    const float* ln;   // logf(u_k)
};

// Gamma<f32>::new(shape, 1) (gamma.rs), parameters computed in f32 as the crate does
struct GammaF32 {
    int kind;          // 0 = large shape, 1 = small shape (< 1), 2 = shape 1 (Exp)
    float d, c;        // GammaLargeShape of shape (large) or shape + 1 (small)
    float inv_shape;   // small: 1 / shape
    float lambda_inv;  // Exp: 1 / (1 / scale)
    float scale;
};
DK_HD GammaF32 gamma_new(float shape) {
    GammaF32 g{};
    const float scale = 1.0f;
    g.scale = scale;
    if (shape == 1.0f) {
        g.kind = 2;
        g.lambda_inv = 1.0f / (1.0f / scale);
        return g;
    }
    const float ls = shape < 1.0f ? shape + 1.0f : shape;
    g.kind = shape < 1.0f ? 1 : 0;
    g.inv_shape = 1.0f / shape;
    g.d = ls - (float)(1.0 / 3.0);
    g.c = 1.0f / sqrtf(9.0f * g.d);
    return g;
}
DK_HD float ln_f32(float v) { return (float)log((double)v); }   // (see the header)
DK_HD float gamma_large(const GammaF32& g, Rng& r, const Open01Tab& t) {
    for (;;) {
        const float x = normal_f32(r);
        const float v_cbrt = 1.0f + g.c * x;
        if (v_cbrt <= 0.0f) continue;
        const float v = v_cbrt * v_cbrt * v_cbrt;
        uint32_t k;
        const float u = open01_f32(r, &k);
        const float x_sqr = x * x;
        if (u < 1.0f - (float)0.0331 * x_sqr * x_sqr || t.ln[k] < 0.5f * x_sqr + g.d * (1.0f - v + ln_f32(v)))
            return g.d * v * g.scale;
    }
}
DK_HD float gamma_sample(const GammaF32& g, Rng& r, const Open01Tab& t) {
    if (g.kind == 2) return exp1_f32(r) * g.lambda_inv;
    if (g.kind == 1) {
        uint32_t k;
        (void)open01_f32(r, &k);                  // u first (GammaSmallShape::sample)
        return gamma_large(g, r, t) * t.pw[k];    // * u.powf(inv_shape)
    }
    return gamma_large(g, r, t);
}

// beta.rs Beta<f32>::new(alpha, beta), parameters in f32 as the crate computes them
struct BetaF32 {
    bool bb, switched;
    float a, b, alpha, beta, gamma, kappa1, kappa2;
};
DK_HD BetaF32 beta_new(float alpha0, float beta0) {
    BetaF32 p{};
    const bool lo_first = alpha0 < beta0;
    const float mn = lo_first ? alpha0 : beta0, mx = lo_first ? beta0 : alpha0;
    p.switched = !lo_first;
    if (mn > 1.0f) {                       // BB: a = the smaller
        p.bb = true;
        p.a = mn; p.b = mx;
        p.alpha = p.a + p.b;
        p.beta = sqrtf((p.alpha - 2.0f) / (2.0f * p.a * p.b - p.alpha));
        p.gamma = p.a + 1.0f / p.beta;
    } else {                               // BC: a = the larger, the switch flag flipped
        p.bb = false;
        p.a = mx; p.b = mn;
        p.switched = !p.switched;
        p.alpha = p.a + p.b;
        p.beta = 1.0f / p.b;
        const float delta = 1.0f + p.a - p.b;
        p.kappa1 = delta * ((float)(1. / 18. / 4.) + (float)(3. / 4. / 18.) * p.b) / (p.a * p.beta - (float)(14. / 18.));
        p.kappa2 = 0.25f + (0.5f + 0.25f / delta) * p.b;
    }
    return p;
}
DK_HD float beta_sample(const BetaF32& p, Rng& r) {
    using lm::expf_glibc;
    using lm::logf_glibc;
    float w;
    if (p.bb) {
        for (;;) {
            const float u1 = std_f32(r), u2 = std_f32(r);
            const float v = p.beta * logf_glibc(u1 / (1.0f - u1));
            w = p.a * expf_glibc(v);
            const float z = u1 * u1 * u2;
            const float rr = p.gamma * v - logf_glibc(4.0f);
            const float s = p.a + rr - w;
            if (s + 2.609438f >= 5.0f * z) break;
            const float t = logf_glibc(z);
            if (s >= t) break;
            if (!(rr + p.alpha * logf_glibc(p.alpha / (p.b + w)) < t)) break;
        }
    } else {
        for (;;) {
            const float u1 = std_f32(r), u2 = std_f32(r);
            float z;
            if (u1 < 0.5f) {
                const float y = u1 * u2;
                z = u1 * y;
                if (0.25f * u2 + z - y >= p.kappa1) continue;
            } else {
                z = u1 * u1 * u2;
                if (z <= 0.25f) {
                    w = p.a * expf_glibc(p.beta * logf_glibc(u1 / (1.0f - u1)));
                    break;
                }
                if (z >= p.kappa2) continue;
            }
            const float v = p.beta * logf_glibc(u1 / (1.0f - u1));
            w = p.a * expf_glibc(v);
            if (!(p.alpha * (logf_glibc(p.alpha / (p.b + w)) + v) - 1.3862944f < logf_glibc(z))) break;
        }
    }
    if (!p.switched) return w == INFINITY ? 1.0f : w / (p.b + w);
    return p.b == INFINITY ? 0.0f : p.b / (p.b + w);
}

// Dirichlet<f32, 39>::sample with all 39 alphas equal: FromBeta when alpha <= 0.1 (no tables
// read), else FromGamma (the Open01 tables of the context).
DK_HD void dirichlet39(float alpha, Rng& r, const Open01Tab& t, float out[39]) {
    if (alpha <= 0.1f) {
        float csum = alpha;                // alpha_{i+1} + ... + alpha_38, summed from the end
        float rev[38];
        rev[37] = csum;
        for (int k = 36; k >= 0; --k) rev[k] = csum = csum + alpha;
        float acc = 1.0f;
        for (int i = 0; i < 38; ++i) {
            const float bs = beta_sample(beta_new(alpha, rev[i]), r);
            out[i] = acc * bs;
            acc = acc * (1.0f - bs);
        }
        out[38] = acc;
        return;
    }
    const GammaF32 g = gamma_new(alpha);
    float sum = 0.0f;
    for (int i = 0; i < 39; ++i) {
        out[i] = gamma_sample(g, r, t);
        sum = sum + out[i];
    }
    const float invacc = 1.0f / sum;
    for (int i = 0; i < 39; ++i) out[i] = out[i] * invacc;
}
// Dirichlet::new's errors: an alpha that is not > 0 or not finite
DK_HD bool dirichlet_alpha_ok(float alpha) { return alpha > 0.0f && alpha < INFINITY; }
DK_HD bool dirichlet_needs_tables(float alpha) { return alpha > 0.1f; }

}  // namespace rd
}  // namespace dk
