// Row kernels of the AlphaZero network's forward pass (az_network.py), bf16 in
// HBM, f32 arithmetic.  The activations are [B*62, d] rows with d = 160: torch's
// generic LayerNorm kernel spends ~0.5 ms per call on the C5 batch (8192 x 62
// rows) where the bytes take ~65 us, and the residual adds and the six embedding
// gathers are separate passes.  Here:
//   embed_ln   : x = sum of the six token embeddings; h = LN(x)         (one pass)
//   add_ln     : x += delta; h = LN(x)                                  (one pass)
//   ln         : h = LN(x)
// One row per 32-lane half-wave: lane l holds elements l, l+32, ... (d/32 per
// lane), so every load/store instruction of a half-wave covers 64 contiguous
// bytes.  Mean and variance: f32 two-pass over the registers, shuffle
// reductions inside the half-wave.  LayerNorm as torch: (x - mean) *
// rsqrt(var + eps) * gamma + beta, biased variance.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace dk {
namespace net {

constexpr int LN_MAX_PER_LANE = 16;   // d <= 512

__device__ __forceinline__ float bf2f(uint16_t v) { return __uint_as_float((uint32_t)v << 16); }
__device__ __forceinline__ uint16_t f2bf(float f) {   // round to nearest even (torch's conversion)
    const uint32_t u = __float_as_uint(f);
    if ((u & 0x7F800000u) == 0x7F800000u && (u & 0x7FFFFFu)) return (uint16_t)((u >> 16) | 0x40u);   // NaN
    return (uint16_t)((u + 0x7FFFu + ((u >> 16) & 1u)) >> 16);
}

__device__ __forceinline__ float half_wave_sum(float v) {
#pragma unroll
    for (int o = 16; o >= 1; o >>= 1) v += __shfl_xor(v, o, 32);
    return v;
}

template <int PER>
__device__ __forceinline__ void ln_row(const float (&x)[PER], int d, int lane, const uint16_t* gamma, const uint16_t* beta,
                                       float eps, uint16_t* out) {
    float s = 0.0f;
#pragma unroll
    for (int k = 0; k < PER; ++k) s += x[k];
    const float mean = half_wave_sum(s) / (float)d;
    float q = 0.0f;
#pragma unroll
    for (int k = 0; k < PER; ++k) { const float c = x[k] - mean; q += c * c; }
    const float rstd = rsqrtf(half_wave_sum(q) / (float)d + eps);
#pragma unroll
    for (int k = 0; k < PER; ++k) {
        const int j = lane + 32 * k;
        out[j] = f2bf((x[k] - mean) * rstd * bf2f(gamma[j]) + bf2f(beta[j]));
    }
}

// tokens [B, 311] int32 (encode_state_pi); tables: object, position, player, subposition, team, phase
template <int PER>
__global__ void embed_ln_kernel(const int32_t* __restrict__ tokens, uint32_t B, const uint16_t* __restrict__ e0,
                                const uint16_t* __restrict__ e1, const uint16_t* __restrict__ e2,
                                const uint16_t* __restrict__ e3, const uint16_t* __restrict__ e4,
                                const uint16_t* __restrict__ e5, const uint16_t* gamma, const uint16_t* beta, float eps,
                                uint16_t* __restrict__ x_out, uint16_t* __restrict__ h_out) {
    const int d = 32 * PER;
    const uint32_t row = blockIdx.x * (blockDim.x / 32) + threadIdx.x / 32;
    const int lane = threadIdx.x & 31;
    if (row >= B * 62u) return;
    const uint32_t b = row / 62u, s = row % 62u;
    const int32_t* t = tokens + (size_t)b * 311;
    const uint16_t* rows[6] = {e0 + (size_t)t[s] * d, e1 + (size_t)t[62 + s] * d, e2 + (size_t)t[124 + s] * d,
                               e3 + (size_t)t[186 + s] * d, e4 + (size_t)t[248 + s] * d, e5 + (size_t)t[310] * d};
    float x[PER];
#pragma unroll
    for (int k = 0; k < PER; ++k) {
        const int j = lane + 32 * k;
        // torch sums the six bf16 embeddings left to right with a bf16 rounding after each add
        float acc = bf2f(rows[0][j]);
#pragma unroll
        for (int e = 1; e < 6; ++e) acc = bf2f(f2bf(acc + bf2f(rows[e][j])));
        x[k] = acc;
        x_out[(size_t)row * d + j] = f2bf(acc);
    }
    ln_row<PER>(x, d, lane, gamma, beta, eps, h_out + (size_t)row * d);
}

// x += delta (bf16 add as torch rounds it); h = LN(x)
template <int PER>
__global__ void add_ln_kernel(uint16_t* __restrict__ x_io, const uint16_t* __restrict__ delta, uint32_t rows,
                              const uint16_t* gamma, const uint16_t* beta, float eps, uint16_t* __restrict__ h_out) {
    const int d = 32 * PER;
    const uint32_t row = blockIdx.x * (blockDim.x / 32) + threadIdx.x / 32;
    const int lane = threadIdx.x & 31;
    if (row >= rows) return;
    float x[PER];
#pragma unroll
    for (int k = 0; k < PER; ++k) {
        const size_t j = (size_t)row * d + lane + 32 * k;
        const uint16_t v = delta ? f2bf(bf2f(x_io[j]) + bf2f(delta[j])) : x_io[j];
        if (delta) x_io[j] = v;
        x[k] = bf2f(v);
    }
    ln_row<PER>(x, d, lane, gamma, beta, eps, h_out + (size_t)row * d);
}

}  // namespace net
}  // namespace dk
