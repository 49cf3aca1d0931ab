// TEST INFRASTRUCTURE: the search's UCT picks (pick_child_x over 16-B or, with
// -DDK_PICK8, 8-B records, with -DDK_HOT16L the long 16-B records whose means compare by 64-bit
// cross products; pick_child_reg over 32-B records in DK_HOT16=0 builds) against the plain
// two-pass f64 UCT of the reference (node.rs:202-277) on random and near-tied
// child blocks, with the f32 reciprocal / sqrt perturbed by up to 4 ulp (the
// GPU's v_rcp_f32 / v_sqrt_f32 are within 1 ulp).  Prints "OK <n>".
#define DK_APPROX_HOOKS
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <random>

#include "../../master_doko_reinforcement_learning_amd/csrc/engine/search_core.h"

static std::mt19937_64 g_pert(7);
static float perturb(float y) {
    const int k = (int)(g_pert() % 9) - 4;
    for (int i = 0; i < k; ++i) y = nextafterf(y, INFINITY);
    for (int i = 0; i > k; --i) y = nextafterf(y, -INFINITY);
    return y;
}
float dk::rcp_approx(float x) { return perturb(1.0f / x); }
float dk::sqrt_approx(float x) { return perturb(sqrtf(x)); }
float dk::rsqrt_approx(float x) { return perturb(1.0f / sqrtf(x)); }

struct NullMem {   // chain-end prefetch target (never a forced node here: info = j*13 << 6 has nchild 0)
    dk::NodeHot load_hot(uint32_t) const { dk::NodeHot h; memset(&h, 0, sizeof(h)); return h; }
    void touch_next(uint32_t, uint32_t, uint32_t) const {}
};

static uint32_t naive(const dk::NodeHot* rec, uint32_t n, double lnN, double c) {
    double min_q = INFINITY, max_q = -INFINITY;
    for (uint32_t j = 0; j < n; ++j) {
        const double q = dk::mean_of(rec[j].stats);
        min_q = q < min_q ? q : min_q;
        max_q = q > max_q ? q : max_q;
    }
    const bool flat = fabs(max_q - min_q) < dk::DK_F64_EPSILON;
    double best = -INFINITY;
    uint32_t pick = 0;
    for (uint32_t j = 0; j < n; ++j) {
        const double u = dk::uct_exact(rec[j].stats, dk::mean_of(rec[j].stats), flat, min_q, max_q, lnN, c);
        if (u > best) { best = u; pick = j; }
    }
    return pick;
}

int main(int argc, char** argv) {
    const long cases = argc > 1 ? atol(argv[1]) : 1000000;
    std::mt19937_64 r(argc > 2 ? strtoull(argv[2], 0, 10) : 1);
    long ties = 0;
    for (long t = 0; t < cases; ++t) {
        dk::NodeHot rec[dk::SCAN_REG];
        memset(rec, 0, sizeof(rec));
        const uint32_t n = 2 + (uint32_t)(r() % 11);
        const int mode = (int)(r() % 8);
        // 16-B builds compare means by 24-bit cross products, exact for v <= P24_MAX_ITERS
        // and |mean| <= 123 (search_core.h); mode 5 probes large visit counts within that
#if DK_PICK8
        const uint32_t VBOUND = dk::P8_MAX_ITERS;
#elif defined(DK_HOT16L) && DK_HOT16L
        const uint32_t VBOUND = dk::NI_MAX_STATES - 1;   // the long records: any search length
#else
        const uint32_t VBOUND = dk::P24_MAX_ITERS;
#endif
        const uint32_t vmax = mode == 5 ? (DK_HOT16 ? VBOUND : 100000u) : 1000u;
        uint32_t total = 0;
        // mode 6: Farey neighbours a/b and c/d (|ad - bc| = 1, b, d in [500, 1000]) around a
        // common integer part k differ by 1/(bd) ~ 1e-6, ~3e-8 relative at |mean| ~ 40:
        // far below the f32 estimates' resolution, so the exact tie-break decides
        int64_t fk = (int64_t)(r() % 81) - 40, fb = 500 + (int64_t)(r() % 501), fd = 500 + (int64_t)(r() % 501);
        {
            auto gcd = [](int64_t x, int64_t y) { while (y) { const int64_t t = x % y; x = y; y = t; } return x; };
            while (gcd(fb, fd) != 1) ++fd;
        }
        int64_t fa = 0;
        for (int64_t x = 0; x < fb; ++x) if ((x * fd + 1) % fb == 0) { fa = x; break; }
        const int64_t fc = (fa * fd + 1) / fb;
        for (uint32_t j = 0; j < n; ++j) {
            uint32_t v = 1 + (uint32_t)(r() % vmax);
            int32_t s;
            if (mode == 0) s = (int32_t)(r() % (2 * 60 * v + 1)) - (int32_t)(60 * v);     // any mean in [-60, 60]
            else if (mode == 1) { const int32_t q = (int32_t)(r() % 7) - 3; s = q * (int32_t)v; }   // equal means
            else if (mode == 2) { s = (int32_t)(r() % 5) - 2; }                             // means near 0
            else if (mode == 3) { v = 1 + (uint32_t)(r() % 3); s = (int32_t)(r() % 9) - 4; } // tiny visits
            else if (mode == 4 && j > 0) { v = (uint32_t)rec[0].stats + (uint32_t)(r() % 3); s = (int32_t)(rec[0].stats >> 32) + (int32_t)(r() % 3) - 1; }
            else if (mode == 6) {   // a near-tie pair (see below), alternating over the children
                const bool first = (j % 2) == 0;
                v = (uint32_t)(first ? fb : fd);
                s = (int32_t)(first ? fa + fk * fb : fc + fk * fd);
            }
            else if (mode == 7) {   // the bound itself: |w| up to 123 v at v up to P24_MAX_ITERS
                v = VBOUND - (uint32_t)(r() % 64);
                s = (int32_t)(r() % (2 * 123 * v + 1)) - (int32_t)(123 * v);
            }
            else s = (int32_t)(r() % (2 * 20 * v + 1)) - (int32_t)(20 * v);
            rec[j].stats = (uint64_t)v | ((uint64_t)(uint32_t)s << 32);
            total += v;
        }
        // (no unvisited child: the search's picks only scan visited children, checked there)
        for (uint32_t j = 0; j < n; ++j) rec[j] = dk::make_hot<dk::NodeHot>(rec[j].stats, 0, 0);   // as the backup leaves it
        const double lnN = std::log((double)(total + (uint32_t)(r() % 5)));
        const double c = (r() % 4 == 0) ? 0.7 + (double)(r() % 100) / 10.0 : 2.5;
        uint64_t gs; uint32_t gc, gi;
        dk::NodeHot end; bool end_ok;
        NullMem nm;
        const uint32_t b = naive(rec, n, lnN, c);
        auto cb_of = [](uint32_t j) { return j * 14u; };
        auto info_of = [](uint32_t j) { return (j * 13u) << 6; };   // player / flags / state bits, nchild 0
#if DK_PICK8
        dk::Block8 blk;
        for (int j = 0; j < dk::SCAN_REG; ++j) {
            blk.w0[j] = dk::p8_w0(rec[j].stats);
            blk.w1[j] = dk::p8_w1(cb_of((uint32_t)j), info_of((uint32_t)j));
        }
        const uint32_t a = dk::pick_child_x<dk::Raw8>(blk, n, lnN, c, nm, &gs, &gc, &gi, &end, &end_ok, 0u);
        const uint32_t want_info = dk::p8_info(dk::p8_w1(cb_of(b), info_of(b)));
#else
        dk::Block blk;
        for (int j = 0; j < dk::SCAN_REG; ++j) {
            blk.st[j] = rec[j].stats; blk.cb[j] = cb_of((uint32_t)j); blk.inf[j] = info_of((uint32_t)j);
            blk.q[j] = dk::hot_q(rec[j]); blk.isv[j] = dk::hot_isv(rec[j]);
        }
#if defined(DK_HOT16L) && DK_HOT16L
        const uint32_t a = dk::pick_child_x<dk::Raw16L>(blk, n, lnN, c, nm, &gs, &gc, &gi, &end, &end_ok, 0u);
#elif DK_HOT16
        const uint32_t a = dk::pick_child_x<dk::Raw16>(blk, n, lnN, c, nm, &gs, &gc, &gi, &end, &end_ok, 0u);
#else
        const uint32_t a = dk::pick_child_reg(blk, n, lnN, c, nm, &gs, &gc, &gi, &end, &end_ok);
#endif
        const uint32_t want_info = info_of(b);
#endif
        if (a != b || gs != rec[b].stats || gc != cb_of(b) || gi != want_info) {
            printf("MISMATCH case %ld n %u mode %d: got %u want %u\n", t, n, mode, a, b);
            return 1;
        }
        ties += mode == 1 || mode == 4;
    }
    printf("OK %ld\n", cases);
    return 0;
}
