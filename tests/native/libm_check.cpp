// TEST INFRASTRUCTURE: the device's restatement of glibc's logf / expf (engine/libm_f32.h, used by
// the FromBeta Dirichlet root noise) against the host's glibc, on every f32 input whose bits are
// first + i * stride (stride 1: all 2^32 of them), bit for bit (NaNs compare equal to NaNs).
// Usage: libm_check <stride> [threads]        prints "OK <inputs checked>"
#include <atomic>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <thread>
#include <vector>

#include "../../master_doko_reinforcement_learning_amd/csrc/engine/libm_f32.h"

static bool same(float a, float b) { return (a != a && b != b) || std::memcmp(&a, &b, 4) == 0; }

int main(int argc, char** argv) {
    const uint64_t stride = argc > 1 ? strtoull(argv[1], 0, 10) : 1;
    const int nt = argc > 2 ? atoi(argv[2]) : 8;
    if (!stride || nt < 1) return 2;
    const uint64_t n = ((1ull << 32) + stride - 1) / stride;
    std::atomic<uint64_t> bad{0};
    std::vector<std::thread> th;
    for (int t = 0; t < nt; ++t)
        th.emplace_back([&, t] {
            uint64_t b = 0;
            for (uint64_t i = t; i < n; i += nt) {
                const uint32_t bits = (uint32_t)(i * stride);
                float x;
                std::memcpy(&x, &bits, 4);
                const float l0 = logf(x), l1 = dk::lm::logf_glibc(x);
                const float e0 = expf(x), e1 = dk::lm::expf_glibc(x);
                if (!same(l0, l1) || !same(e0, e1)) {
                    if (b++ < 4) printf("MISMATCH x %a (%08x): logf %a / %a, expf %a / %a\n", x, bits, l0, l1, e0, e1);
                }
            }
            bad += b;
        });
    for (auto& x : th) x.join();
    if (bad) { printf("MISMATCH %llu inputs\n", (unsigned long long)bad.load()); return 1; }
    printf("OK %llu\n", (unsigned long long)n);
    return 0;
}
