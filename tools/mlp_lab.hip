// Measurement harness for the d = 160 f32 MLP half as the x-only chain runs it
// (mlp_ln_f32x3_kernel<160, 32, 4, true>: x normalised with the producer's row statistics, x and the
// next statistics written, no h).  Compiles the kernel header alone (seconds, not the library's
// minutes), so that -D variants of the header can be timed and compared:
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 -ffp-contract=off [-DVARIANT...] -o tools/mlp_lab tools/mlp_lab.hip
//   tools/mlp_lab [rows] [reps] [dump-file]
// Prints one JSON line: median / min kernel ms (HIP events, one launch each), the FNV-1a hash of
// the outputs (x and the statistics: equal hashes = bit-identical results across variants), and in
// DK_NET_PROF builds wave 0's phase clocks (prologue, GEMM1 + DMA issue, GELU + split, GEMM2,
// wait + barrier, epilogue) in shader cycles per chunk-wave.  Inputs are seeded and identical
// for every variant; x is restored before every launch.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

#include "../master_doko_reinforcement_learning_amd/csrc/az_net_kernels.h"
#include "../master_doko_reinforcement_learning_amd/csrc/az_net_f32_kernels.h"

#define CK(x)                                                                                      \
    do {                                                                                           \
        hipError_t e_ = (x);                                                                       \
        if (e_ != hipSuccess) {                                                                    \
            fprintf(stderr, "%s failed: %s (%s:%d)\n", #x, hipGetErrorString(e_), __FILE__, __LINE__); \
            exit(1);                                                                               \
        }                                                                                          \
    } while (0)

static uint64_t lcg(uint64_t& s) { s = s * 6364136223846793005ull + 1442695040888963407ull; return s >> 33; }
static float unif(uint64_t& s) { return (float)((double)lcg(s) / 2147483648.0 - 1.0); }   // [-1, 1)
static uint16_t bf16_rn(float f) {
    uint32_t u;
    memcpy(&u, &f, 4);
    return (uint16_t)((u + 0x7FFFu + ((u >> 16) & 1u)) >> 16);
}
static float bf16_f(uint16_t b) { uint32_t u = (uint32_t)b << 16; float f; memcpy(&f, &u, 4); return f; }

int main(int argc, char** argv) {
    constexpr int D = 160, N = 640;
    const uint32_t rows = argc > 1 ? (uint32_t)atoi(argv[1]) : 507904u;
    const int reps = argc > 2 ? atoi(argv[2]) : 20;
    uint64_t s = 12345;
    std::vector<float> x((size_t)rows * D), st(2 * (size_t)rows), gin(D), bin(D), g(D), be(D), b1(N), b2(D);
    for (auto& v : x) v = 2.0f * unif(s);
    for (uint32_t r = 0; r < rows; ++r) {   // the producer's two-pass statistics, eps 1e-5
        double m = 0, q = 0;
        for (int k = 0; k < D; ++k) m += x[(size_t)r * D + k];
        m /= D;
        for (int k = 0; k < D; ++k) { const double dv = x[(size_t)r * D + k] - m; q += dv * dv; }
        st[2 * r] = (float)m;
        st[2 * r + 1] = (float)(1.0 / std::sqrt(q / D + 1e-5));
    }
    for (int k = 0; k < D; ++k) { gin[k] = 1.0f + 0.1f * unif(s); bin[k] = 0.1f * unif(s); g[k] = 1.0f + 0.1f * unif(s); be[k] = 0.1f * unif(s); b2[k] = 0.1f * unif(s); }
    for (auto& v : b1) v = 0.1f * unif(s);
    // weights (W1 [N][D], W2 [D][N]) split into bf16 hi / lo
    std::vector<uint16_t> w1h((size_t)N * D), w1l((size_t)N * D), w2h((size_t)D * N), w2l((size_t)D * N);
    for (size_t i = 0; i < w1h.size(); ++i) {
        const float w = unif(s) / std::sqrt((float)D);
        w1h[i] = bf16_rn(w);
        w1l[i] = bf16_rn(w - bf16_f(w1h[i]));
    }
    for (size_t i = 0; i < w2h.size(); ++i) {
        const float w = unif(s) / std::sqrt((float)N);
        w2h[i] = bf16_rn(w);
        w2l[i] = bf16_rn(w - bf16_f(w2h[i]));
    }
    auto up = [](const void* h, size_t bytes) { void* d; CK(hipMalloc(&d, bytes)); CK(hipMemcpy(d, h, bytes, hipMemcpyHostToDevice)); return d; };
    float* dx0 = (float*)up(x.data(), x.size() * 4);
    float* dx;
    CK(hipMalloc(&dx, x.size() * 4));
    float* dst = (float*)up(st.data(), st.size() * 4);
    float* dso;
    CK(hipMalloc(&dso, st.size() * 4));
    float *dgin = (float*)up(gin.data(), D * 4), *dbin = (float*)up(bin.data(), D * 4), *dg = (float*)up(g.data(), D * 4),
          *dbe = (float*)up(be.data(), D * 4), *db1 = (float*)up(b1.data(), N * 4), *db2 = (float*)up(b2.data(), D * 4);
    uint16_t *dw1h = (uint16_t*)up(w1h.data(), w1h.size() * 2), *dw1l = (uint16_t*)up(w1l.data(), w1l.size() * 2),
             *dw2h = (uint16_t*)up(w2h.data(), w2h.size() * 2), *dw2l = (uint16_t*)up(w2l.data(), w2l.size() * 2);
#ifndef LAB_WAVES
#define LAB_WAVES 4
#endif
    constexpr uint32_t RW = 32u * LAB_WAVES;   // rows per workgroup
    auto launch = [&]() {
        hipLaunchKernelGGL((dk::net::mlp_ln_f32x3_kernel<160, 32, LAB_WAVES, true>), dim3((rows + RW - 1) / RW), dim3(64u * LAB_WAVES), 0, 0,
                           (const float*)nullptr, dx, dw1h, dw1l, db1, dw2h, dw2l, db2, rows, (uint32_t)N, dg, dbe, 1e-5f,
                           (float*)nullptr, dgin, dbin, (const float2*)dst, (float2*)dso);
    };
    std::vector<float> ms;
    hipEvent_t a, b;
    CK(hipEventCreate(&a));
    CK(hipEventCreate(&b));
#ifdef DK_NET_PROF
    const uint64_t z[16] = {};
#endif
    for (int r = 0; r < reps + 1; ++r) {
        CK(hipMemcpy(dx, dx0, x.size() * 4, hipMemcpyDeviceToDevice));
#ifdef DK_NET_PROF
        CK(hipMemcpyToSymbol(HIP_SYMBOL(dk::net::dk_mlp_prof_acc), z, sizeof(z)));
#endif
        CK(hipDeviceSynchronize());
        CK(hipEventRecord(a));
        launch();
        CK(hipEventRecord(b));
        CK(hipEventSynchronize(b));
        float t;
        CK(hipEventElapsedTime(&t, a, b));
        if (r) ms.push_back(t);   // (the first launch warms)
    }
    std::vector<float> xo(x.size()), so(st.size());
    CK(hipMemcpy(xo.data(), dx, xo.size() * 4, hipMemcpyDeviceToHost));
    CK(hipMemcpy(so.data(), dso, so.size() * 4, hipMemcpyDeviceToHost));
    uint64_t hsh = 1469598103934665603ull;
    auto mix = [&](const void* p, size_t n) { const uint8_t* c = (const uint8_t*)p; for (size_t i = 0; i < n; ++i) { hsh ^= c[i]; hsh *= 1099511628211ull; } };
    mix(xo.data(), xo.size() * 4);
    mix(so.data(), so.size() * 4);
    if (argc > 3) {
        FILE* f = fopen(argv[3], "wb");
        if (f) { fwrite(xo.data(), 4, xo.size(), f); fwrite(so.data(), 4, so.size(), f); fclose(f); }
    }
    std::sort(ms.begin(), ms.end());
    printf("{\"rows\": %u, \"median_ms\": %.4f, \"min_ms\": %.4f, \"hash\": \"%016llx\"", rows, ms[ms.size() / 2], ms[0],
           (unsigned long long)hsh);
#ifdef DK_NET_PROF
    uint64_t acc[16];
    CK(hipMemcpyFromSymbol(acc, HIP_SYMBOL(dk::net::dk_mlp_prof_acc), sizeof(acc)));
    const double cw = (double)((rows + RW - 1) / RW) * (N / 32);   // chunk-waves of wave 0 over the last launch
    printf(", \"phase_cycles_per_chunk_wave0\": [%.0f, %.0f, %.0f, %.0f, %.0f, %.0f]", acc[0] / cw, acc[1] / cw, acc[2] / cw,
           acc[3] / cw, acc[4] / cw, acc[5] / cw);
    printf(", \"sclk_mhz\": %.1f, \"wg_life_us\": %.2f", acc[7] ? 100.0 * (double)acc[6] / (double)acc[7] : 0.0,
           acc[7] / 100.0 / (double)((rows + RW - 1) / RW));
#endif
    printf("}\n");
    return 0;
}
