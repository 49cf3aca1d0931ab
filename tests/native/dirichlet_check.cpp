// TEST INFRASTRUCTURE: host build of engine/rand_distr.h (the AlphaZero root noise the GPU
// draws) checked against the ORACLE restatement of rand_distr 0.5.1 (oracle/rand_distr05.hpp):
//   1. the committed ziggurat tables (engine/ziggurat_tables.h, tools/gen_ziggurat.py) equal
//      the ones the oracle recomputes by the crate's generator, bit for bit;
//   2. StandardNormal / Exp1 f64 streams, Gamma<f32> and Dirichlet<f32, 39> draws are
//      identical value for value, and so is the RNG stream position after every draw, for
//      shapes on all three Gamma paths (< 1, == 1, > 1), Beta<f32> draws on both of Cheng's
//      algorithms (BB, BC), and the FromBeta Dirichlet (alpha <= 0.1).  The engine runs with the Open01
//      tables the context builds (glibc logf / powf of the 2^23 Open01 values) and its own
//      ln v = (float)log((double)v); the oracle calls glibc throughout.
// Usage: dirichlet_check <draws per alpha> <seed>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

#include "../../master_doko_reinforcement_learning_amd/csrc/engine/rand_distr.h"
#include "../../oracle/rand_distr05.hpp"

using namespace oracle;

static dk::Rng to_dk(const SmallRng& r) { dk::Rng d; d.s0 = r.s[0]; d.s1 = r.s[1]; d.s2 = r.s[2]; d.s3 = r.s[3]; return d; }
static bool same(const dk::Rng& d, const SmallRng& r) { return d.s0 == r.s[0] && d.s1 == r.s[1] && d.s2 == r.s[2] && d.s3 == r.s[3]; }

int main(int argc, char** argv) {
    const long draws = argc > 1 ? atol(argv[1]) : 20000;
    const uint64_t seed = argc > 2 ? strtoull(argv[2], 0, 10) : 1;
    // 1. tables
    const rdist::Zig& z = rdist::zig();
    if (memcmp(z.nx, dk::zig::NORM_X, sizeof z.nx) || memcmp(z.nf, dk::zig::NORM_F, sizeof z.nf) ||
        memcmp(z.ex, dk::zig::EXP_X, sizeof z.ex) || memcmp(z.ef, dk::zig::EXP_F, sizeof z.ef) ||
        z.norm_r != dk::zig::NORM_R || z.exp_r != dk::zig::EXP_R) {
        printf("MISMATCH ziggurat tables\n");
        return 1;
    }
    // Open01 tables as the context builds them (doko_amd.hip rd_tables)
    constexpr uint32_t K = 1u << 23;
    std::vector<float> ln(K), pw(K);
    auto u_of = [](uint32_t k) { return __builtin_bit_cast(float, k | 0x3F800000u) - (1.0f - FLT_EPSILON / 2.0f); };
    for (uint32_t k = 0; k < K; ++k) ln[k] = logf(u_of(k));
    long checked = 0;
    // 2a. ziggurat streams
    {
        SmallRng o = SmallRng::seed_from_u64(seed);
        dk::Rng d = to_dk(o);
        for (long i = 0; i < 20 * draws; ++i) {
            const double a = rdist::normal_f64(o), b = dk::rd::ziggurat<true>(d, dk::zig::NORM_X, dk::zig::NORM_F);
            const double e = rdist::exp1_f64(o), f = dk::rd::ziggurat<false>(d, dk::zig::EXP_X, dk::zig::EXP_F);
            if (memcmp(&a, &b, 8) || memcmp(&e, &f, 8) || !same(d, o)) { printf("MISMATCH ziggurat draw %ld\n", i); return 1; }
            checked += 2;
        }
    }
    // 2b. Beta on both algorithms (the FromBeta Dirichlet's pairs among them: (0.1, 3.8), (0.05, 0.05))
    const float pairs[][2] = {{0.1f, 3.8f}, {0.05f, 0.05f}, {0.05f, 1.9f}, {0.5f, 0.5f}, {3.0f, 0.7f}, {2.5f, 4.0f}};
    for (const auto& pr : pairs) {
        SmallRng o = SmallRng::seed_from_u64(seed * 613 + (uint64_t)(pr[0] * 1000) * 7 + (uint64_t)(pr[1] * 1000));
        dk::Rng d = to_dk(o);
        const rdist::Beta ob(pr[0], pr[1]);
        const dk::rd::BetaF32 db = dk::rd::beta_new(pr[0], pr[1]);
        for (long i = 0; i < 10 * draws; ++i) {
            const float a = ob.sample(o), b = dk::rd::beta_sample(db, d);
            if (memcmp(&a, &b, 4) || !same(d, o)) {
                printf("MISMATCH beta (%g, %g) draw %ld: %a vs %a\n", pr[0], pr[1], i, a, b);
                return 1;
            }
            checked++;
        }
    }
    // 2c. Gamma and Dirichlet on every path (alpha <= 0.1: the FromBeta construction)
    const float alphas[] = {0.05f, 0.1f, 0.3f, 0.5f, 0.8f, 1.0f, 1.5f, 3.0f};
    for (float alpha : alphas) {
        const float inv_shape = 1.0f / alpha;
        if (alpha < 1.0f)
            for (uint32_t k = 0; k < K; ++k) pw[k] = powf(u_of(k), inv_shape);
        const dk::rd::Open01Tab tab{pw.data(), ln.data()};
        SmallRng o = SmallRng::seed_from_u64(seed * 977 + (uint64_t)(alpha * 1000));
        dk::Rng d = to_dk(o);
        const rdist::Gamma og(alpha);
        const dk::rd::GammaF32 dg = dk::rd::gamma_new(alpha);
        for (long i = 0; i < 10 * draws; ++i) {
            const float a = og.sample(o), b = dk::rd::gamma_sample(dg, d, tab);
            if (memcmp(&a, &b, 4) || !same(d, o)) { printf("MISMATCH gamma alpha %g draw %ld: %a vs %a\n", alpha, i, a, b); return 1; }
            checked++;
        }
        float al[39], on[39], dn[39];
        for (float& x : al) x = alpha;
        for (long i = 0; i < draws; ++i) {
            if (!rdist::dirichlet(al, 39, o, on)) { printf("REFUSED alpha %g\n", alpha); return 1; }
            dk::rd::dirichlet39(alpha, d, tab, dn);
            if (memcmp(on, dn, sizeof on) || !same(d, o)) { printf("MISMATCH dirichlet alpha %g draw %ld\n", alpha, i); return 1; }
            checked++;
        }
    }
    printf("OK %ld draws\n", checked);
    return 0;
}
