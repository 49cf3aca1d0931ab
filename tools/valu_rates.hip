// Issue cost of the integer VALU instructions the rollout is made of (gfx950), measured:
// each kernel runs 8 independent chains of ONE instruction kind (16-fold unrolled), W waves per
// SIMD, and stamps s_memtime (shader clock) / s_memrealtime (100 MHz) around the loop.  Output:
// one JSON line per (kind, waves) with cycles per wave-instruction per SIMD and the shader clock
// the stamps imply.  Used to price the rollout's per-ply code (profiles/r06/valu_rates.json).
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 -o tools/valu_rates tools/valu_rates.hip
#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstdio>
#include <cstdlib>

#define CK(x)                                                                                      \
    do {                                                                                           \
        hipError_t e_ = (x);                                                                       \
        if (e_ != hipSuccess) {                                                                    \
            fprintf(stderr, "%s failed: %s (%s:%d)\n", #x, hipGetErrorString(e_), __FILE__, __LINE__); \
            exit(1);                                                                               \
        }                                                                                          \
    } while (0)

enum Kind { ADD, MAD64, MULHI, MULLO, MUL24, BCNT, ALIGNBIT, ADD64, BITOP3, BFE, LSHLADD, CNDMASK, NKIND };
static const char* NAMES[NKIND] = {"v_add_u32", "v_mad_u64_u32", "v_mul_hi_u32", "v_mul_lo_u32", "v_mul_u32_u24",
                                   "v_bcnt_u32_b32", "v_alignbit_b32", "v_lshl_add_u64", "v_bitop3_b32", "v_bfe_u32",
                                   "v_lshl_add_u32", "v_cndmask_b32"};

// one instruction of the kind, as inline asm so that the compiler neither folds nor rewrites it
template <int K>
__device__ __forceinline__ void step(uint32_t& x, uint64_t& y, uint32_t k, uint64_t m) {
    if constexpr (K == ADD) asm volatile("v_add_u32 %0, %0, %1" : "+v"(x) : "v"(k));
    else if constexpr (K == MAD64) { uint64_t cc; asm volatile("v_mad_u64_u32 %0, %1, %2, %3, %0" : "+v"(y), "=s"(cc) : "v"(x), "v"(k)); }
    else if constexpr (K == MULHI) asm volatile("v_mul_hi_u32 %0, %0, %1" : "+v"(x) : "v"(k));
    else if constexpr (K == MULLO) asm volatile("v_mul_lo_u32 %0, %0, %1" : "+v"(x) : "v"(k));
    else if constexpr (K == MUL24) asm volatile("v_mul_u32_u24 %0, %0, %1" : "+v"(x) : "v"(k));
    else if constexpr (K == BCNT) asm volatile("v_bcnt_u32_b32 %0, %0, %1" : "+v"(x) : "v"(k));
    else if constexpr (K == ALIGNBIT) asm volatile("v_alignbit_b32 %0, %0, %1, 9" : "+v"(x) : "v"(k));
    else if constexpr (K == ADD64) asm volatile("v_lshl_add_u64 %0, %0, 0, %1" : "+v"(y) : "v"(m));
    else if constexpr (K == BITOP3) asm volatile("v_bitop3_b32 %0, %0, %1, %2 bitop3:0x96" : "+v"(x) : "v"(k), "v"((uint32_t)m));
    else if constexpr (K == BFE) asm volatile("v_bfe_u32 %0, %0, %1, 9" : "+v"(x) : "v"(k));
    else if constexpr (K == LSHLADD) asm volatile("v_lshl_add_u32 %0, %0, 3, %1" : "+v"(x) : "v"(k));
    else if constexpr (K == CNDMASK) asm volatile("v_cndmask_b32_e64 %0, %0, %1, %2" : "+v"(x) : "v"(k), "s"(m));
}

template <int K>
__global__ void __launch_bounds__(64) rate_kernel(uint32_t* out, uint64_t* stamps, int iters) {
    uint32_t x[8];
    uint64_t y[8];
#pragma unroll
    for (int c = 0; c < 8; ++c) { x[c] = threadIdx.x * (c + 3) + c; y[c] = x[c] * 0x9E3779B97F4A7C15ull; }
    const uint32_t k = blockIdx.x | 0x10001u;
    const uint64_t mm = 0x5555555555555555ull ^ blockIdx.x;
    const uint64_t t0 = __builtin_amdgcn_s_memtime(), r0 = __builtin_amdgcn_s_memrealtime();
    for (int i = 0; i < iters; ++i) {
#pragma unroll
        for (int u = 0; u < 16; ++u) {
#pragma unroll
            for (int c = 0; c < 8; ++c) step<K>(x[c], y[c], k + c, mm);
        }
    }
    __builtin_amdgcn_s_waitcnt(0);
    const uint64_t t1 = __builtin_amdgcn_s_memtime(), r1 = __builtin_amdgcn_s_memrealtime();
    uint32_t acc = 0;
#pragma unroll
    for (int c = 0; c < 8; ++c) acc ^= x[c] ^ (uint32_t)y[c] ^ (uint32_t)(y[c] >> 32);
    out[blockIdx.x * 64 + threadIdx.x] = acc;
    if (threadIdx.x == 0) { stamps[4 * blockIdx.x] = t1 - t0; stamps[4 * blockIdx.x + 1] = r1 - r0; }
}

template <int K>
void run(int cus, int waves, int iters, uint32_t* out, uint64_t* st) {
    const int blocks = cus * 4 * waves;
    hipLaunchKernelGGL(rate_kernel<K>, dim3(blocks), dim3(64), 0, 0, out, st, iters);   // warm
    CK(hipDeviceSynchronize());
    hipEvent_t a, b;
    CK(hipEventCreate(&a)); CK(hipEventCreate(&b));
    CK(hipEventRecord(a));
    hipLaunchKernelGGL(rate_kernel<K>, dim3(blocks), dim3(64), 0, 0, out, st, iters);
    CK(hipEventRecord(b));
    CK(hipEventSynchronize(b));
    float ms = 0;
    CK(hipEventElapsedTime(&ms, a, b));
    uint64_t* h = (uint64_t*)malloc(sizeof(uint64_t) * 4 * blocks);
    CK(hipMemcpy(h, st, sizeof(uint64_t) * 4 * blocks, hipMemcpyDeviceToHost));
    double cyc = 0, rt = 0;
    for (int i = 0; i < blocks; ++i) { cyc += (double)h[4 * i]; rt += (double)h[4 * i + 1]; }
    cyc /= blocks; rt /= blocks;
    const double n = (double)iters * 16 * 8;   // instructions of the kind per wave (source level)
    // per SIMD: `waves` waves share the SIMD, so a wave's cycles / n / waves... reported both ways
    printf("{\"kind\": \"%s\", \"waves_per_simd\": %d, \"cycles_per_wave_inst\": %.3f, \"cycles_per_inst_per_simd\": %.3f, "
           "\"sclk_mhz\": %.1f, \"ms\": %.3f}\n",
           NAMES[K], waves, cyc / n, cyc / n / waves, cyc / (rt / 100.0), ms);
    free(h);
    CK(hipEventDestroy(a)); CK(hipEventDestroy(b));
}

template <int K>
void run_all(int cus, int iters, uint32_t* out, uint64_t* st) {
    for (int w : {1, 3}) run<K>(cus, w, iters, out, st);
    if constexpr (K + 1 < NKIND) run_all<K + 1>(cus, iters, out, st);
}

int main(int argc, char** argv) {
    const int iters = argc > 1 ? atoi(argv[1]) : 2000;
    hipDeviceProp_t p;
    CK(hipGetDeviceProperties(&p, 0));
    const int cus = p.multiProcessorCount;
    uint32_t* out;
    uint64_t* st;
    CK(hipMalloc(&out, sizeof(uint32_t) * 64 * cus * 4 * 3));
    CK(hipMalloc(&st, sizeof(uint64_t) * 4 * cus * 4 * 3));
    run_all<0>(cus, iters, out, st);
    CK(hipFree(out)); CK(hipFree(st));
    return 0;
}
