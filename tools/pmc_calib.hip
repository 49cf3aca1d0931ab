// PMC calibration kernels for the search kernel's roofline ("Measured bound").
//
// Each kernel does a KNOWN amount of work of one access or instruction pattern the search
// kernel is made of, so that rocprofv3 counters can be read against it:
//   valu<W>     : W waves per SIMD of independent 32-bit integer VALU chains (what the
//                 counters report for a saturated / a single-wave VALU pipe)
//   rd<B,N>     : every lane reads N consecutive B-byte vectors at a random B-aligned
//                 address of a 16 GiB buffer (beyond L2 and the 256 MiB Infinity Cache):
//                 rd<16,1> = one 16-B load (a child pair, a state quarter), rd<16,4> = a 64-B
//                 node state, rd<16,6> = a 12-child block, rd<8,1> = one 8-B record
//   stream16    : coalesced 16 B per lane streaming read (the guide's calibration case)
//   wr<B,N>     : random stores of the same shapes (the backup / expansion stores)
// The program prints one JSON line per kernel with its algorithmic bytes (or VALU
// instructions) per launch and the event-timed duration; tools/pmc_calib_report.py joins
// them with the counter passes.  Every launch is bounded (fixed trip counts).
#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>

#define CK(x)                                                                               \
    do {                                                                                    \
        hipError_t e_ = (x);                                                                \
        if (e_ != hipSuccess) {                                                             \
            fprintf(stderr, "%s failed: %s (%s:%d)\n", #x, hipGetErrorString(e_), __FILE__, __LINE__); \
            exit(1);                                                                        \
        }                                                                                   \
    } while (0)

__device__ __forceinline__ uint64_t mix64(uint64_t z) {
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ULL;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBULL;
    return z ^ (z >> 31);
}

// 8 independent integer chains of full-rate VALU ops (add, xor, shift-add)
template <int TAG>
__global__ void __launch_bounds__(64) valu_kernel(uint32_t* out, int iters) {
    uint32_t a = threadIdx.x, b = a * 3u + 1u, c = a ^ 0x55u, d = a + 7u, e = a ^ 0x1234u, f = a + 99u,
             g = a * 5u, h = a ^ 0xF0F0u;
    for (int i = 0; i < iters; ++i) {
#pragma unroll
        for (int k = 0; k < 8; ++k) {
            a = (a ^ (b << 3)) + 0x9E37u; b = (b ^ (c << 5)) + 0x79B9u; c = (c ^ (d << 7)) + 0x7F4Au;
            d = (d ^ (a << 1)) + 0x7C15u; e = (e ^ (f << 3)) + 0x1F35u; f = (f ^ (g << 5)) + 0x3B71u;
            g = (g ^ (h << 7)) + 0x5A3Cu; h = (h ^ (e << 1)) + 0x0DE1u;
        }
    }
    out[blockIdx.x * 64 + threadIdx.x] = a ^ b ^ c ^ d ^ e ^ f ^ g ^ h;
}

struct alignas(16) V16 { uint32_t x, y, z, w; };

template <int B, int N>
__global__ void __launch_bounds__(256) rd_kernel(const uint8_t* buf, uint64_t slots, int loads, uint32_t* out) {
    const uint64_t t = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    uint32_t acc = 0;
    for (int k = 0; k < loads; ++k) {
        const uint64_t s = mix64(t * 0x9E3779B97F4A7C15ULL + (uint64_t)k) % slots;
        const uint8_t* p = buf + s * (uint64_t)(B * N);
#pragma unroll
        for (int j = 0; j < N; ++j) {
            if constexpr (B == 16) {
                const V16 v = *reinterpret_cast<const V16*>(p + 16 * j);
                acc += v.x ^ v.y ^ v.z ^ v.w;
            } else if constexpr (B == 8) {
                const uint2 v = *reinterpret_cast<const uint2*>(p + 8 * j);
                acc += v.x ^ v.y;
            } else {
                acc += *reinterpret_cast<const uint32_t*>(p + 4 * j);
            }
        }
    }
    out[t] = acc;
}

template <int B, int N>
__global__ void __launch_bounds__(256) wr_kernel(uint8_t* buf, uint64_t slots, int stores) {
    const uint64_t t = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    for (int k = 0; k < stores; ++k) {
        const uint64_t s = mix64(t * 0x9E3779B97F4A7C15ULL + (uint64_t)k + 0x5555ULL) % slots;
        uint8_t* p = buf + s * (uint64_t)(B * N);
#pragma unroll
        for (int j = 0; j < N; ++j) {
            if constexpr (B == 16) {
                V16 v; v.x = (uint32_t)t; v.y = (uint32_t)k; v.z = (uint32_t)s; v.w = 1u;
                *reinterpret_cast<V16*>(p + 16 * j) = v;
            } else if constexpr (B == 8) {
                *reinterpret_cast<uint2*>(p + 8 * j) = make_uint2((uint32_t)t, (uint32_t)k);
            } else {
                *reinterpret_cast<uint32_t*>(p + 4 * j) = (uint32_t)t;
            }
        }
    }
}

__global__ void __launch_bounds__(256) stream16_kernel(const V16* buf, uint64_t n, uint32_t* out) {
    uint32_t acc = 0;
    const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
    for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride) {
        const V16 v = buf[i];
        acc += v.x ^ v.y ^ v.z ^ v.w;
    }
    out[(uint64_t)blockIdx.x * blockDim.x + threadIdx.x] = acc;
}

static hipEvent_t e0, e1;

template <class F>
static float timed(F launch) {
    launch();                      // warm-up launch (its counters are the first dispatch)
    CK(hipDeviceSynchronize());
    CK(hipEventRecord(e0, 0));
    launch();
    CK(hipEventRecord(e1, 0));
    CK(hipEventSynchronize(e1));
    float ms = 0;
    CK(hipEventElapsedTime(&ms, e0, e1));
    return ms;
}

int main(int argc, char** argv) {
    const char* only = argc > 1 ? argv[1] : "";
    hipDeviceProp_t prop;
    CK(hipGetDeviceProperties(&prop, 0));
    const int cus = prop.multiProcessorCount;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    const uint64_t BUF = 16ULL << 30;
    uint8_t* buf = nullptr;
    uint32_t* out = nullptr;
    CK(hipMalloc(&buf, BUF));
    CK(hipMemset(buf, 0, BUF));
    const uint64_t lanes = 1ULL << 20;   // 4096 workgroups of 256
    CK(hipMalloc(&out, lanes * 4 * 8));
    auto want = [&](const char* n) { return !*only || strstr(n, only); };

    // VALU: 1, 2, 3 and 8 waves per SIMD, fixed instruction count per wave
    const int viters = 20000;
    for (int w : {1, 2, 3, 8}) {
        char name[32];
        snprintf(name, sizeof name, "valu_w%d", w);
        if (!want(name)) continue;
        const unsigned grid = (unsigned)(cus * 4 * w);
        float ms;
        switch (w) {
            case 1: ms = timed([&] { hipLaunchKernelGGL(valu_kernel<1>, dim3(grid), dim3(64), 0, 0, out, viters); }); break;
            case 2: ms = timed([&] { hipLaunchKernelGGL(valu_kernel<2>, dim3(grid), dim3(64), 0, 0, out, viters); }); break;
            case 3: ms = timed([&] { hipLaunchKernelGGL(valu_kernel<3>, dim3(grid), dim3(64), 0, 0, out, viters); }); break;
            default: ms = timed([&] { hipLaunchKernelGGL(valu_kernel<8>, dim3(grid), dim3(64), 0, 0, out, viters); }); break;
        }
        // 8 chains x 8 unrolled x 2 VALU ops (xor-shift, add) per step: a lower bound on the
        // wave's VALU instructions; SQ_INSTS_VALU gives the exact count
        printf("{\"test\": \"%s\", \"kernel\": \"valu_kernel<%d>\", \"waves\": %u, \"waves_per_simd\": %d, \"ms\": %.4f}\n",
               name, w, grid, w, ms);
    }
    const int loads = 64;
    const unsigned grid = (unsigned)(lanes / 256);
    struct RdCase { const char* name; const char* kernel; int b, n; };
    const RdCase rds[] = {{"rd8x1", "rd_kernel<8, 1>", 8, 1}, {"rd16x1", "rd_kernel<16, 1>", 16, 1},
                          {"rd16x4", "rd_kernel<16, 4>", 16, 4}, {"rd16x6", "rd_kernel<16, 6>", 16, 6}};
    for (const RdCase& c : rds) {
        if (!want(c.name)) continue;
        const uint64_t slots = BUF / (uint64_t)(c.b * c.n);
        float ms;
        if (c.b == 8) ms = timed([&] { hipLaunchKernelGGL((rd_kernel<8, 1>), dim3(grid), dim3(256), 0, 0, buf, slots, loads, out); });
        else if (c.n == 1) ms = timed([&] { hipLaunchKernelGGL((rd_kernel<16, 1>), dim3(grid), dim3(256), 0, 0, buf, slots, loads, out); });
        else if (c.n == 4) ms = timed([&] { hipLaunchKernelGGL((rd_kernel<16, 4>), dim3(grid), dim3(256), 0, 0, buf, slots, loads, out); });
        else ms = timed([&] { hipLaunchKernelGGL((rd_kernel<16, 6>), dim3(grid), dim3(256), 0, 0, buf, slots, loads, out); });
        const double bytes = (double)lanes * loads * c.b * c.n;
        printf("{\"test\": \"%s\", \"kernel\": \"%s\", \"accesses\": %.0f, \"alg_bytes\": %.0f, \"ms\": %.4f, \"gbs\": %.1f}\n",
               c.name, c.kernel, (double)lanes * loads, bytes, ms, bytes / ms / 1e6);
    }
    const RdCase wrs[] = {{"wr8x1", "wr_kernel<8, 1>", 8, 1}, {"wr16x4", "wr_kernel<16, 4>", 16, 4}};
    for (const RdCase& c : wrs) {
        if (!want(c.name)) continue;
        const uint64_t slots = BUF / (uint64_t)(c.b * c.n);
        float ms;
        if (c.b == 8) ms = timed([&] { hipLaunchKernelGGL((wr_kernel<8, 1>), dim3(grid), dim3(256), 0, 0, buf, slots, loads); });
        else ms = timed([&] { hipLaunchKernelGGL((wr_kernel<16, 4>), dim3(grid), dim3(256), 0, 0, buf, slots, loads); });
        const double bytes = (double)lanes * loads * c.b * c.n;
        printf("{\"test\": \"%s\", \"kernel\": \"%s\", \"accesses\": %.0f, \"alg_bytes\": %.0f, \"ms\": %.4f, \"gbs\": %.1f}\n",
               c.name, c.kernel, (double)lanes * loads, bytes, ms, bytes / ms / 1e6);
    }
    if (want("stream16")) {
        const uint64_t n = BUF / 4 / 16;   // 4 GiB
        const float ms = timed([&] { hipLaunchKernelGGL(stream16_kernel, dim3(grid), dim3(256), 0, 0, (const V16*)buf, n, out); });
        printf("{\"test\": \"stream16\", \"kernel\": \"stream16_kernel\", \"alg_bytes\": %.0f, \"ms\": %.4f, \"gbs\": %.1f}\n",
               (double)n * 16, ms, (double)n * 16 / ms / 1e6);
    }
    CK(hipFree(buf));
    CK(hipFree(out));
    return 0;
}
