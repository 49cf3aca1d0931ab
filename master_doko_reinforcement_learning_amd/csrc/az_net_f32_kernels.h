// Kernels of the networks' f32 forward (az_network.FusedTrunkF32): the reference's precision --
// f32 activations everywhere, GEMM products at least as fine as its matmul precision "medium"
// (az_doko.py:539-541, main.py:508).  At d = 160 / 256 with 4 heads every GEMM runs inside the
// hand-written bf16x3 kernels below (qkv_attn_ln_f32x3, mlp_ln_f32x3 / mlp16_ln_f32x3, the class
// heads); only other shapes fall back to torch GEMMs around these row kernels, the memory-bound
// passes fused:
//   embed_ln_f32 : x = sum of the six token embeddings (left to right, f32); h = LN(x)
//   add_ln_f32   : x += delta; h = LN(x)                 (delta may be NULL: h = LN(x))
//   attn62_f32   : softmax(q k^T / sqrt(hd)) v per (sample, head), q / k / v read from the
//                  fused qkv projection [B*62, 3d], the heads' outputs written [B*62, d]
//   gelu_f32     : y = GELU(y) in place, the exact erf form of nn.GELU()
// One row per 32-lane half-wave in the row kernels: lane l holds float4 groups l, l + 32
// (d / 4 groups), so a half-wave instruction moves up to 512 contiguous bytes.  LayerNorm as
// torch: two-pass mean / biased variance, (x - mean) * rsqrt(var + eps) * gamma + beta.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace dk {
namespace net {

constexpr int LN4_MAX = 4;   // float4 groups per lane: d <= 512

__device__ __forceinline__ float hw_sum(float v) {
#pragma unroll
    for (int o = 16; o >= 1; o >>= 1) v += __shfl_xor(v, o, 32);
    return v;
}

template <int P4>
__device__ __forceinline__ void ln_row_f32(const float4 (&x)[P4], int d, int lane, const float4* gamma4,
                                           const float4* beta4, float eps, float4* out4) {
    const int n4 = d / 4;
    float s = 0.0f;
#pragma unroll
    for (int k = 0; k < P4; ++k)
        if (lane + 32 * k < n4) s += (x[k].x + x[k].y) + (x[k].z + x[k].w);
    const float mean = hw_sum(s) / (float)d;
    float q = 0.0f;
#pragma unroll
    for (int k = 0; k < P4; ++k)
        if (lane + 32 * k < n4) {
            const float a = x[k].x - mean, b = x[k].y - mean, c = x[k].z - mean, e = x[k].w - mean;
            q += (a * a + b * b) + (c * c + e * e);
        }
    const float rstd = rsqrtf(hw_sum(q) / (float)d + eps);
#pragma unroll
    for (int k = 0; k < P4; ++k) {
        const int j = lane + 32 * k;
        if (j < n4) {
            const float4 g = gamma4[j], b = beta4[j];
            out4[j] = make_float4((x[k].x - mean) * rstd * g.x + b.x, (x[k].y - mean) * rstd * g.y + b.y,
                                  (x[k].z - mean) * rstd * g.z + b.z, (x[k].w - mean) * rstd * g.w + b.w);
        }
    }
}

// tokens [B, 311] int32 (encode_state_pi / encode_state_ipi); tables (f32): object, position,
// player, subposition, team, phase (or player to guess)
template <int P4>
__global__ void embed_ln_f32_kernel(const int32_t* __restrict__ tokens, uint32_t B, int d, const float* __restrict__ e0,
                                    const float* __restrict__ e1, const float* __restrict__ e2,
                                    const float* __restrict__ e3, const float* __restrict__ e4,
                                    const float* __restrict__ e5, const float* gamma, const float* beta, float eps,
                                    float* __restrict__ x_out, float* __restrict__ h_out) {
    const uint32_t row = blockIdx.x * (blockDim.x / 32) + threadIdx.x / 32;
    const int lane = threadIdx.x & 31, n4 = d / 4;
    if (row >= B * 62u) return;
    const uint32_t b = row / 62u, s = row % 62u;
    const int32_t* t = tokens + (size_t)b * 311;
    const float4* rows[6] = {(const float4*)(e0 + (size_t)t[s] * d), (const float4*)(e1 + (size_t)t[62 + s] * d),
                             (const float4*)(e2 + (size_t)t[124 + s] * d), (const float4*)(e3 + (size_t)t[186 + s] * d),
                             (const float4*)(e4 + (size_t)t[248 + s] * d), (const float4*)(e5 + (size_t)t[310] * d)};
    float4* xo = (float4*)(x_out + (size_t)row * d);
    float4 x[P4];
#pragma unroll
    for (int k = 0; k < P4; ++k) {
        const int j = lane + 32 * k;
        x[k] = make_float4(0.0f, 0.0f, 0.0f, 0.0f);
        if (j < n4) {
            float4 a = rows[0][j];
#pragma unroll
            for (int e = 1; e < 6; ++e) {   // torch: ((((e0 + e1) + e2) + e3) + e4) + e5
                const float4 v = rows[e][j];
                a.x += v.x; a.y += v.y; a.z += v.z; a.w += v.w;
            }
            x[k] = a;
            xo[j] = a;
        }
    }
    // (h_out NULL: x only -- the d = 160 x-only chain normalises x in its first half)
    if (h_out != nullptr)
        ln_row_f32<P4>(x, d, lane, (const float4*)gamma, (const float4*)beta, eps, (float4*)(h_out + (size_t)row * d));
}

// The embedding sum alone (h_out NULL: the x-only chain normalises x in its first half), one lane
// per float4 of a row: lanes fully used at any d % 4 == 0 (the row-per-half-wave form above left
// 24 of 32 lanes idle in its second group at d = 160) and x stored contiguously across the wave.
// The six token reads of a row are shared by its d / 4 lanes (cache hits).
__global__ void embed_f32_kernel(const int32_t* __restrict__ tokens, uint32_t B, int d, const float* __restrict__ e0,
                                 const float* __restrict__ e1, const float* __restrict__ e2, const float* __restrict__ e3,
                                 const float* __restrict__ e4, const float* __restrict__ e5, float* __restrict__ x_out) {
    const uint32_t n4 = (uint32_t)d / 4u;
    const uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x;
    if (i >= (uint64_t)B * 62u * n4) return;
    const uint32_t row = (uint32_t)(i / n4), j = (uint32_t)(i % n4);
    const uint32_t b = row / 62u, s = row % 62u;
    const int32_t* t = tokens + (size_t)b * 311;
    const int32_t k0 = t[s], k1 = t[62 + s], k2 = t[124 + s], k3 = t[186 + s], k4 = t[248 + s], k5 = t[310];
    float4 a = ((const float4*)(e0 + (size_t)k0 * d))[j];
    const float4 v1 = ((const float4*)(e1 + (size_t)k1 * d))[j], v2 = ((const float4*)(e2 + (size_t)k2 * d))[j],
                 v3 = ((const float4*)(e3 + (size_t)k3 * d))[j], v4 = ((const float4*)(e4 + (size_t)k4 * d))[j],
                 v5 = ((const float4*)(e5 + (size_t)k5 * d))[j];
    // torch: ((((e0 + e1) + e2) + e3) + e4) + e5
    a.x += v1.x; a.y += v1.y; a.z += v1.z; a.w += v1.w;
    a.x += v2.x; a.y += v2.y; a.z += v2.z; a.w += v2.w;
    a.x += v3.x; a.y += v3.y; a.z += v3.z; a.w += v3.w;
    a.x += v4.x; a.y += v4.y; a.z += v4.z; a.w += v4.w;
    a.x += v5.x; a.y += v5.y; a.z += v5.z; a.w += v5.w;
    ((float4*)x_out)[i] = a;
}

template <int P4>
__global__ void add_ln_f32_kernel(float* __restrict__ x_io, const float* __restrict__ delta, uint32_t rows, int d,
                                  const float* gamma, const float* beta, float eps, float* __restrict__ h_out,
                                  const float* __restrict__ bias = nullptr) {
    const uint32_t row = blockIdx.x * (blockDim.x / 32) + threadIdx.x / 32;
    const int lane = threadIdx.x & 31, n4 = d / 4;
    if (row >= rows) return;
    float4* xr = (float4*)(x_io + (size_t)row * d);
    const float4* dr = delta ? (const float4*)(delta + (size_t)row * d) : nullptr;
    float4 x[P4];
#pragma unroll
    for (int k = 0; k < P4; ++k) {
        const int j = lane + 32 * k;
        x[k] = make_float4(0.0f, 0.0f, 0.0f, 0.0f);
        if (j < n4) {
            float4 v = xr[j];
            if (dr) {
                float4 e = dr[j];
                if (bias) {   // the GEMM's bias, added to its output first (torch's F.linear epilogue order)
                    const float4 b = ((const float4*)bias)[j];
                    e.x += b.x; e.y += b.y; e.z += b.z; e.w += b.w;
                }
                v.x += e.x; v.y += e.y; v.z += e.z; v.w += e.w;
                xr[j] = v;
            }
            x[k] = v;
        }
    }
    ln_row_f32<P4>(x, d, lane, (const float4*)gamma, (const float4*)beta, eps, (float4*)(h_out + (size_t)row * d));
}

// GELU(v) = 0.5 v (1 + erf(v / sqrt 2)), the exact form (libm erff); bias (may be NULL): the
// producing GEMM's bias over rows of w4 float4 groups, added first
__global__ void gelu_f32_kernel(float* __restrict__ y, size_t n4, const float* __restrict__ bias = nullptr, uint32_t w4 = 1) {
    const size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n4) return;
    float4 v = ((float4*)y)[i];
    if (bias) {
        const float4 b = ((const float4*)bias)[i % w4];
        v.x += b.x; v.y += b.y; v.z += b.z; v.w += b.w;
    }
    v.x = 0.5f * v.x * (1.0f + erff(v.x * 0.70710678118654752f));
    v.y = 0.5f * v.y * (1.0f + erff(v.y * 0.70710678118654752f));
    v.z = 0.5f * v.z * (1.0f + erff(v.z * 0.70710678118654752f));
    v.w = 0.5f * v.w * (1.0f + erff(v.w * 0.70710678118654752f));
    ((float4*)y)[i] = v;
}

// Attention core in f32: one wave per (sample, head), the query on the lane (62 of 64 lanes).
// The head's K and V rows (62 x HD f32 each) are staged in LDS; every lane reads the same key
// row (an LDS broadcast).  Keys in chunks of 8: the chunk's scores in registers, one rescale of
// the running output per chunk (online softmax with the chunk maximum), exp via exp2f.
template <int HD>
__global__ void __launch_bounds__(64) attn62_f32_kernel(const float* __restrict__ qkv, float* __restrict__ y,
                                                        uint32_t batch, uint32_t heads, float scale) {
    static_assert(HD % 4 == 0, "head dimension: multiple of 4");
    __shared__ float4 ks[62 * (HD / 4)];
    __shared__ float4 vs[62 * (HD / 4)];
    const uint32_t sample = blockIdx.x / heads, head = blockIdx.x % heads;
    const int lane = threadIdx.x;
    const uint32_t d = heads * HD;
    const float* base = qkv + (size_t)sample * 62 * 3 * d;
    // stage K and V of this head
    for (int i = lane; i < 62 * (HD / 4); i += 64) {
        const int t = i / (HD / 4), e4 = i % (HD / 4);
        ks[i] = *(const float4*)(base + (size_t)t * 3 * d + d + head * HD + 4 * e4);
        vs[i] = *(const float4*)(base + (size_t)t * 3 * d + 2 * d + head * HD + 4 * e4);
    }
    const bool ok = lane < 62;
    float4 q[HD / 4];
    {
        const float* qr = base + (size_t)(ok ? lane : 0) * 3 * d + head * HD;
        const float sl = scale * 1.4426950408889634f;   // scores in log2 units: exp(s) = exp2(s log2 e)
#pragma unroll
        for (int e4 = 0; e4 < HD / 4; ++e4) {
            const float4 v = *(const float4*)(qr + 4 * e4);
            q[e4] = make_float4(v.x * sl, v.y * sl, v.z * sl, v.w * sl);
        }
    }
    __syncthreads();
    float4 acc[HD / 4];
#pragma unroll
    for (int e4 = 0; e4 < HD / 4; ++e4) acc[e4] = make_float4(0.0f, 0.0f, 0.0f, 0.0f);
    float m = -INFINITY, l = 0.0f;
    for (int t0 = 0; t0 < 64; t0 += 8) {
        float s[8];
        float cm = -INFINITY;
#pragma unroll
        for (int u = 0; u < 8; ++u) {
            const int t = t0 + u;
            float a = -INFINITY;
            if (t < 62) {
                a = 0.0f;
#pragma unroll
                for (int e4 = 0; e4 < HD / 4; ++e4) {
                    const float4 kv = ks[t * (HD / 4) + e4];
                    a = fmaf(q[e4].x, kv.x, a); a = fmaf(q[e4].y, kv.y, a);
                    a = fmaf(q[e4].z, kv.z, a); a = fmaf(q[e4].w, kv.w, a);
                }
            }
            s[u] = a;
            cm = fmaxf(cm, a);
        }
        const float mn = fmaxf(m, cm);
        const float corr = exp2f(m - mn);   // 0 on the first chunk (m = -inf)
        l *= corr;
#pragma unroll
        for (int e4 = 0; e4 < HD / 4; ++e4) { acc[e4].x *= corr; acc[e4].y *= corr; acc[e4].z *= corr; acc[e4].w *= corr; }
#pragma unroll
        for (int u = 0; u < 8; ++u) {
            const int t = t0 + u;
            if (t < 62) {
                const float p = exp2f(s[u] - mn);
                l += p;
#pragma unroll
                for (int e4 = 0; e4 < HD / 4; ++e4) {
                    const float4 vv = vs[t * (HD / 4) + e4];
                    acc[e4].x = fmaf(p, vv.x, acc[e4].x); acc[e4].y = fmaf(p, vv.y, acc[e4].y);
                    acc[e4].z = fmaf(p, vv.z, acc[e4].z); acc[e4].w = fmaf(p, vv.w, acc[e4].w);
                }
            }
        }
        m = mn;
    }
    if (!ok) return;
    const float inv = 1.0f / l;
    float* yr = y + ((size_t)sample * 62 + lane) * d + head * HD;
#pragma unroll
    for (int e4 = 0; e4 < HD / 4; ++e4)
        *(float4*)(yr + 4 * e4) = make_float4(acc[e4].x * inv, acc[e4].y * inv, acc[e4].z * inv, acc[e4].w * inv);
}

// The same attention core on the f32 matrix cores (v_mfma_f32_32x32x2_f32: f32 products, f32
// accumulation -- no narrowing), one wave per (sample, head):
//   S^T = K Q^T  : A = K (rows = keys), B = Q^T (columns = queries), k = the head dimension in
//                  steps of 2 (lane half hh supplies dimension hh HD/2 + s), scores pre-scaled by
//                  scale * log2 e in Q; lane (i, hh) then holds query i's scores of keys
//                  32b + (g & 3) + 8 (g >> 2) + 4 hh, so the softmax is the lane's own registers
//                  plus one exchange with lane i ^ 32;
//   O^T = V^T P^T: the k order of a step only has to agree between the operands, so step
//                  (b, g) pairs key j = 32b + (g & 3) + 8 (g >> 2) + 4 hh of each lane half: the
//                  probabilities never leave their registers, V^T comes from LDS;
//   y = O / l    : lane (i, hh) holds dimensions 32t + (g & 3) + 8 (g >> 2) + 4 hh of query i.
// Query tiles one at a time (32 queries; the K fragments stay in registers).  Keys 62, 63 score
// -inf; V rows 62, 63 are zero in LDS.
typedef float f32x16_t __attribute__((ext_vector_type(16)));
// waves per SIMD: 3 at HD = 40 (0.447 against 0.470 ms at 8,192 samples, two spilled registers),
// 2 at HD = 64 (3 spills more there and measured slower)
#ifndef DK_ATTNF32_WAVES40
#define DK_ATTNF32_WAVES40 3
#endif
template <int HD>
__global__ void __launch_bounds__(64, HD == 40 ? DK_ATTNF32_WAVES40 : 2) attn62_f32_mfma_kernel(const float* __restrict__ qkv, float* __restrict__ y,
                                                             uint32_t batch, uint32_t heads, float scale,
                                                             const float* __restrict__ bqkv = nullptr) {
    static_assert(HD % 8 == 0 && HD <= 64, "head dimension: a multiple of 8, at most 64");
    constexpr int KS = HD / 2, DT = (HD + 31) / 32;
    constexpr int LDV = (4 * HD) % 64 == 32 ? HD : HD + 8;   // V rows j and j + 4 in disjoint bank halves
    __shared__ float vs[64 * LDV];
    const uint32_t sample = blockIdx.x / heads, head = blockIdx.x % heads;
    const int lane = threadIdx.x, r = lane & 31, hh = lane >> 5;
    const uint32_t d = heads * HD;
    const float* base = qkv + (size_t)sample * 62 * 3 * d;
    // the qkv GEMM's bias (may be NULL; q | k | v segments of 3d) is added as the operands load
    const float4 zero4 = make_float4(0.0f, 0.0f, 0.0f, 0.0f);
    auto badd = [&](float4 v, int off) {
        if (bqkv) { const float4 b = *(const float4*)(bqkv + off); v.x += b.x; v.y += b.y; v.z += b.z; v.w += b.w; }
        return v;
    };
    for (int i = lane; i < 64 * (HD / 4); i += 64) {
        const int t = i / (HD / 4), e4 = i % (HD / 4);
        const float4 v = t < 62 ? badd(*(const float4*)(base + (size_t)t * 3 * d + 2 * d + head * HD + 4 * e4),
                                       2 * (int)d + (int)head * HD + 4 * e4)
                                : zero4;
        *(float4*)&vs[t * LDV + 4 * e4] = v;
    }
    // K fragments of both key tiles: kf[b][s] = K[32b + r][hh KS + s] (step s pairs dimensions s
    // and KS + s: any pairing works if Q uses the same, and this one is two contiguous runs)
    float kf[2][KS];
#pragma unroll
    for (int b = 0; b < 2; ++b) {
        const int j = 32 * b + r;
        const float4* kr = (const float4*)(base + (size_t)(j < 62 ? j : 0) * 3 * d + d + head * HD + hh * KS);
#pragma unroll
        for (int s4 = 0; s4 < KS / 4; ++s4) {
            const float4 v = j < 62 ? badd(kr[s4], (int)d + (int)head * HD + hh * KS + 4 * s4) : zero4;
            kf[b][4 * s4] = v.x; kf[b][4 * s4 + 1] = v.y; kf[b][4 * s4 + 2] = v.z; kf[b][4 * s4 + 3] = v.w;
        }
    }
    __syncthreads();
    const float sl = scale * 1.4426950408889634f;
#pragma unroll 1
    for (int a = 0; a < 2; ++a) {
        const int i = 32 * a + r;                      // this lane's query
        float qf[KS];
        {
            const float4* qr = (const float4*)(base + (size_t)(i < 62 ? i : 0) * 3 * d + head * HD + hh * KS);
#pragma unroll
            for (int s4 = 0; s4 < KS / 4; ++s4) {
                const float4 v = i < 62 ? badd(qr[s4], (int)head * HD + hh * KS + 4 * s4) : zero4;
                qf[4 * s4] = v.x * sl; qf[4 * s4 + 1] = v.y * sl; qf[4 * s4 + 2] = v.z * sl; qf[4 * s4 + 3] = v.w * sl;
            }
        }
        f32x16_t st[2] = {f32x16_t{0}, f32x16_t{0}};
#pragma unroll
        for (int s = 0; s < KS; ++s)
#pragma unroll
            for (int b = 0; b < 2; ++b) st[b] = __builtin_amdgcn_mfma_f32_32x32x2f32(kf[b][s], qf[s], st[b], 0, 0, 0);
        // keys 62, 63 (tile 1, rows 30, 31: g = 14, 15 of the upper half) take no weight
        if (hh) { st[1][14] = -INFINITY; st[1][15] = -INFINITY; }
        float m = -INFINITY;
#pragma unroll
        for (int b = 0; b < 2; ++b)
#pragma unroll
            for (int g = 0; g < 16; ++g) m = fmaxf(m, st[b][g]);
        m = fmaxf(m, __shfl_xor(m, 32));
        float l = 0.0f;
#pragma unroll
        for (int b = 0; b < 2; ++b)
#pragma unroll
            for (int g = 0; g < 16; ++g) {
                const float pv = exp2f(st[b][g] - m);
                st[b][g] = pv;
                l += pv;
            }
        l += __shfl_xor(l, 32);
        f32x16_t ot[DT];
#pragma unroll
        for (int t = 0; t < DT; ++t) ot[t] = f32x16_t{0};
#pragma unroll
        for (int b = 0; b < 2; ++b) {
            // the key tile's V^T fragments, all read before its MFMAs
            float vf[16][DT];
#pragma unroll
            for (int g = 0; g < 16; ++g) {
                const int j = 32 * b + (g & 3) + 8 * (g >> 2) + 4 * hh;
#pragma unroll
                for (int t = 0; t < DT; ++t) {
                    const int e = 32 * t + r;
                    vf[g][t] = e < HD ? vs[j * LDV + e] : 0.0f;
                }
            }
#pragma unroll
            for (int g = 0; g < 16; ++g)
#pragma unroll
                for (int t = 0; t < DT; ++t) ot[t] = __builtin_amdgcn_mfma_f32_32x32x2f32(vf[g][t], st[b][g], ot[t], 0, 0, 0);
        }
        if (i < 62) {
            const float inv = 1.0f / l;
            float* yr = y + ((size_t)sample * 62 + i) * d + head * HD;
#pragma unroll
            for (int t = 0; t < DT; ++t)
#pragma unroll
                for (int q = 0; q < 4; ++q) {
                    const int e = 32 * t + 8 * q + 4 * hh;
                    if (e < HD)
                        *(float4*)(yr + e) = make_float4(ot[t][4 * q] * inv, ot[t][4 * q + 1] * inv, ot[t][4 * q + 2] * inv,
                                                         ot[t][4 * q + 3] * inv);
                }
        }
    }
}

// ---------------------------------------------------------------------------
// The whole MLP half of a block at the reference's precision (round 5), in one pass:
//   a = GELU(h W1^T + b1);  delta = a W2^T;  x += delta + b2;  h' = LN'(x)        (all f32)
// The products are bf16x3: every f32 operand v is split into v_hi = bf16(v) and
// v_lo = bf16(v - v_hi), and each k-step takes three v_mfma_f32_32x32x16_bf16 --
// A_lo B_hi + A_hi B_lo + A_hi B_hi into one f32 accumulator -- so a product carries
// ~16 mantissa bits (the dropped A_lo B_lo is below 2^-16 of it), the accuracy hipBLASLt
// gives f32 GEMMs at matmul precision "medium" on gfx950 (profiles/r04/fp32_gemm_probe.json:
// ~5e-6 relative) and finer than the TF32 products the reference's setting selects on its
// CUDA hardware (az_doko.py:539-541, main.py:508).  The weights come pre-split (w1_hi / w1_lo,
// w2_hi / w2_lo: bf16 copies made once per module, az_network.FusedTrunkF32); activations
// are split in registers.  Accumulation, bias, GELU, residual and LayerNorm stay f32.
// Layout as mlp_ln_kernel: 8 waves x 32 rows; h fragments (hi and lo) of all K = d in
// registers; chunks of NC = 32 hidden units with W1 rows and W2 columns (hi and lo) staged in
// LDS, double-buffered; GEMM1 D1 = W1_c h^T puts a row's hidden units in the lane's registers,
// whose bias + GELU + split ARE the B operand of GEMM2 (D2 = W2_c a^T) without lane movement.
// Unfused (hipBLASLt GEMMs + GELU pass + add / LN pass) the 4d-wide f32 activation went to HBM
// and back three times per block; here a row costs its h and x reads and its x and h' writes.
__device__ __forceinline__ void split_bf16x8(const float (&v)[8], bf16x8_t& hi, bf16x8_t& lo) {
    union { uint32_t u[4]; bf16x8_t v; } a, b;
#pragma unroll
    for (int t = 0; t < 8; t += 2) {
        a.u[t / 2] = pack_bf16x2(v[t], v[t + 1]);
        b.u[t / 2] = pack_bf16x2(v[t] - bf2f((uint16_t)a.u[t / 2]), v[t + 1] - bf2f((uint16_t)(a.u[t / 2] >> 16)));
    }
    hi = a.v;
    lo = b.v;
}

// XIN (round 6, the d = 160 x-only chain): the input is the residual stream x_io itself (h unused),
// normalised here with (gin, bin) and the row statistics its producer wrote (stats_in: mean and
// 1 / sqrt(var + eps_in) per row, the producer's two-pass LayerNorm statistics -- so the h this
// computes equals the h the producer would have written); h_out == nullptr: x only is written;
// stats_out != nullptr: the new x's row statistics (with `eps`) for the next half.  (Reducing over
// the row here instead kept 80 values per lane live beside the split fragments and spilled.)
template <int D, int NC, int WAVES = 4, bool XIN = false>
__global__ void __launch_bounds__(64 * WAVES, D <= 160 ? 8 / WAVES : 1) mlp_ln_f32x3_kernel(const float* __restrict__ h, float* __restrict__ x_io,
                                                                const uint16_t* __restrict__ w1h, const uint16_t* __restrict__ w1l,
                                                                const float* __restrict__ b1,
                                                                const uint16_t* __restrict__ w2h, const uint16_t* __restrict__ w2l,
                                                                const float* __restrict__ b2, uint32_t rows, uint32_t n_hidden,
                                                                const float* __restrict__ gamma, const float* __restrict__ beta,
                                                                float eps, float* __restrict__ h_out,
                                                                const float* __restrict__ gin = nullptr,
                                                                const float* __restrict__ bin = nullptr,
                                                                const float2* __restrict__ stats_in = nullptr,
                                                                float2* __restrict__ stats_out = nullptr) {
    static_assert(D % 32 == 0 && NC == 32, "d: multiple of 32; chunks of 32 hidden units");
    // WAVES x 32 rows per workgroup; the chunks' weights double-buffered (one barrier per chunk)
    // in two LDS arrays: the chunk loop runs in pairs (compute from lds0 while staging into lds1,
    // then the reverse), so that every LDS access names its array and the compiler's LDS-DMA alias
    // tracking lets the W reads of one buffer run while the other buffer's DMA is in flight (one
    // array indexed by the chunk parity made it wait for the DMA before the first MFMA).
    // LDS unpadded, conflict-free for the ds_read_b128 fragment reads (16 lanes of a group on 16
    // distinct bank quads) and laid out so that a lane's DMA source address is one per-lane
    // constant plus a uniform part:
    //   W1 chunk piece-major: piece p (8 k-values) of hidden row i at (p NC + i) x 16 B -- a
    //     fragment read is 32 consecutive pieces; DMA instruction u moves pieces 2u, 2u + 1 of
    //     all 32 rows;
    //   W2 chunk row-major, pieces XOR-swizzled: piece p of output row o at o NC + 8 (p ^ ((o >> 2) & 3)),
    //     so that the rows r, r + 12, ... of a read group hit distinct bank quads.
    // (global_load_lds_dwordx4: the LDS side is 64 consecutive 16-B pieces per wave instruction,
    // any layout is made on the global side.)  Unpadded, a buffer is 40 KiB at d = 160: two
    // workgroups of 4 waves with double-buffered chunks fill the CU's 160 KiB.
    constexpr int T = 64 * WAVES;
    constexpr int KS = D / 16, OT = D / 32, GS = NC / 16;
    constexpr int W1E = NC * D, W2E = D * NC, BUF = 2 * (W1E + W2E);   // one buffer: W1 hi, W1 lo, W2 hi, W2 lo
    constexpr int Q1 = D / 8, Q2 = NC / 8;                              // pieces per row
    constexpr int NP = BUF / 8, NI = (NP + 63) / 64;                    // pieces per buffer, wave instructions
    __shared__ __attribute__((aligned(16))) uint16_t lds0[BUF];
    __shared__ __attribute__((aligned(16))) uint16_t lds1[BUF];
    const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63, r = lane & 31, hh = lane >> 5;
    const uint32_t row = blockIdx.x * (32u * WAVES) + (uint32_t)wave * 32u + (uint32_t)r;
    const bool ok = row < rows;
#ifdef DK_NET_PROF
    // phase clocks of wave 0 (profiling builds): drained stamps, sums in registers, atomics at the end
    unsigned long long f_prev = __builtin_amdgcn_s_memtime(), facc[6] = {0, 0, 0, 0, 0, 0};
    const unsigned long long f_t0 = f_prev, f_r0 = __builtin_amdgcn_s_memrealtime();
#define DK_FSTAMP(k) do { __builtin_amdgcn_s_waitcnt(0); const unsigned long long t_ = __builtin_amdgcn_s_memtime(); facc[k] += t_ - f_prev; f_prev = t_; } while (0)
#else
#define DK_FSTAMP(k) ((void)0)
#endif
#if DK_MLPF32_PRIO == 1
    if (blockIdx.x & 1) __builtin_amdgcn_s_setprio(1);
#elif DK_MLPF32_PRIO == 2
    if ((blockIdx.x >> 8) & 1) __builtin_amdgcn_s_setprio(1);
#endif
    // the row's h, split: lane (r, hh) holds k = 16 kk + 8 hh .. + 7 of row r
    bf16x8_t hfh[KS], hfl[KS];
    auto prologue = [&]() {
    if constexpr (XIN) {
        // the row's x (this lane: k = 16 kk + 8 hh .. + 7), normalised with the producer's row
        // statistics and the consumer's weights, then split (as the h loads below: no reduction)
        const float* xr0 = x_io + (size_t)(ok ? row : 0u) * D + 8 * hh;
        const float2 st = stats_in[ok ? row : 0u];
#pragma unroll
        for (int kk = 0; kk < KS; ++kk) {
            const int c0 = 16 * kk + 8 * hh;
            const float4 xa = *(const float4*)(xr0 + 16 * kk), xb = *(const float4*)(xr0 + 16 * kk + 4);
            const float4 g0 = *(const float4*)(gin + c0), g1 = *(const float4*)(gin + c0 + 4);
            const float4 e0 = *(const float4*)(bin + c0), e1 = *(const float4*)(bin + c0 + 4);
            const float x8[8] = {xa.x, xa.y, xa.z, xa.w, xb.x, xb.y, xb.z, xb.w};
            const float g[8] = {g0.x, g0.y, g0.z, g0.w, g1.x, g1.y, g1.z, g1.w};
            const float be[8] = {e0.x, e0.y, e0.z, e0.w, e1.x, e1.y, e1.z, e1.w};
            float v[8];
#pragma unroll
            for (int j = 0; j < 8; ++j) v[j] = (x8[j] - st.x) * st.y * g[j] + be[j];
            split_bf16x8(v, hfh[kk], hfl[kk]);
            // (materialised here, a k-step at a time: sunk to their first use in the chunk loop,
            // with every load left at the top, they spilled)
            asm volatile("" : "+v"(hfh[kk]), "+v"(hfl[kk]));
        }
    } else {
        const float* hr = h + (size_t)(ok ? row : 0u) * D + 8 * hh;
#pragma unroll
        for (int kk = 0; kk < KS; ++kk) {
            float v[8];
            // (rows past the end compute on row 0 and are never stored: unconditional loads, one wait)
            const float4 a = *(const float4*)(hr + 16 * kk);
            const float4 b = *(const float4*)(hr + 16 * kk + 4);
            v[0] = a.x; v[1] = a.y; v[2] = a.z; v[3] = a.w; v[4] = b.x; v[5] = b.y; v[6] = b.z; v[7] = b.w;
            split_bf16x8(v, hfh[kk], hfl[kk]);
        }
    }
    };
#if !DK_MLPF32_STAGE_FIRST
    prologue();
#endif
    typedef __attribute__((address_space(3))) void lds_void;
    // (a compile-time count of DMA instructions per wave: the loads issued before a stage -- the
    // chunk's biases -- then wait on a counted vmcnt, not on the stage itself)
    static_assert(NP % 64 == 0 && NI % WAVES == 0 && (NC * Q1) % 64 == 0 && (D * Q2) % 64 == 0,
                  "whole wave instructions per buffer and region, the same count per wave");
    // per-lane DMA source offsets (elements): W1 (row lane & 31, piece lane >> 5 of the pair);
    // W2 (row lane >> 2 of the instruction's 16, swizzled piece); uniform parts added per call
    const int dma1 = (lane & 31) * D + 8 * (lane >> 5);
    const int dma2 = (lane >> 2) * (int)n_hidden + 8 * ((lane & 3) ^ ((lane >> 4) & 3));
    constexpr int NIW = NI / WAVES;   // DMA instructions per wave and chunk
    // Four waves, each matrix a wave's share (d = 160: 10 instructions each): wave m stages all of
    // matrix m (W1 hi, W1 lo, W2 hi, W2 lo) through ONE buffer resource, with buffer_load ... lds
    // (MUBUF: vmcnt only).  The FLAT-encoded global_load_lds also counts in lgkmcnt, and while
    // one is in flight the compiler can only wait lgkmcnt(0) for an LDS read, so a W fragment
    // read ahead was waited on together with every read issued after it.  (Four resident
    // resources, one per matrix, pushed the biases' SGPRs into spills.)
    constexpr bool PER_MATRIX = WAVES == 4 && NC * Q1 / 64 == NIW && D * Q2 / 64 == NIW;
    const int wv = __builtin_amdgcn_readfirstlane(wave);
    const bool w1side = wv < 2;
    const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(
        (void*)(wv == 0 ? w1h : wv == 1 ? w1l : wv == 2 ? w2h : w2l), (short)0, (int)(2u * n_hidden * D), 0x00020000);
    const int dmav = 2 * (w1side ? dma1 : dma2);                                  // bytes
    const uint32_t cstride = w1side ? 2u * NC * D : 2u * NC, ustride = w1side ? 32u : 32u * n_hidden;
    auto stage_one = [&](uint32_t c, uint16_t* dst, int ui) {
        if constexpr (PER_MATRIX) {
            __builtin_amdgcn_raw_ptr_buffer_load_lds(rs, (lds_void*)&dst[512 * (wv * NIW + ui)], 16, dmav,
                                                     (int)(c * cstride + (uint32_t)ui * ustride), 0, 0);
        } else {
            const int u = wave + WAVES * ui;   // wave-uniform
            const uint16_t* g;
            if (u < 2 * (NC * Q1 / 64)) {
                const int lo = u >= NC * Q1 / 64, v = lo ? u - NC * Q1 / 64 : u;
                g = (lo ? w1l : w1h) + (size_t)c * NC * D + 16 * v + dma1;
            } else {
                const int u2 = u - 2 * (NC * Q1 / 64), lo = u2 >= D * Q2 / 64, v = lo ? u2 - D * Q2 / 64 : u2;
                g = (lo ? w2l : w2h) + (size_t)(16 * v) * n_hidden + (size_t)c * NC + dma2;
            }
            __builtin_amdgcn_global_load_lds(g, (lds_void*)&dst[512 * u], 16, 0, 0);
        }
    };
#ifndef DK_MLPF32_DMA_STEP
#define DK_MLPF32_DMA_STEP 1
#endif
#ifndef DK_MLPF32_PKGELU
#define DK_MLPF32_PKGELU 0
#endif
#ifndef DK_MLPF32_EARLY_BIAS
#define DK_MLPF32_EARLY_BIAS 0
#endif
#ifndef DK_MLPF32_PRIO
#define DK_MLPF32_PRIO 0
#endif
#ifndef DK_MLPF32_STAGE_FIRST
#define DK_MLPF32_STAGE_FIRST 0
#endif
    constexpr int DMA_PER_STEP = DK_MLPF32_DMA_STEP;
    auto stage = [&](uint32_t c, uint16_t* dst) {
#pragma unroll
        for (int ui = 0; ui < NIW; ++ui) stage_one(c, dst, ui);
    };
    // the lane's W2 swizzle (rows 32 t + r share (row >> 2) & 3)
    const int sw = (r >> 2) & 3;
    f32x16_t acc2[OT];
#pragma unroll
    for (int t = 0; t < OT; ++t) acc2[t] = f32x16_t{0};
    const uint32_t chunks = n_hidden / NC;
    stage(0u, lds0);
#ifdef DK_SOL_NODMA
    stage(0u, lds1);   // (speed-of-light measurement build: every chunk computes on chunk 0's weights)
#endif
#if DK_MLPF32_STAGE_FIRST
    prologue();        // (the first chunk's DMA in flight under the row loads)
#endif
    __builtin_amdgcn_s_waitcnt(0);
    __syncthreads();
    DK_FSTAMP(0);
    float bb[NC];   // (DK_MLPF32_EARLY_BIAS: loaded before the previous chunk's closing wait)
#if DK_MLPF32_EARLY_BIAS
#pragma unroll
    for (int m = 0; m < NC; ++m) bb[m] = b1[m];
#endif
    auto chunk = [&](uint32_t c, const uint16_t* cur, uint16_t* nxt) {
        // GEMM1 accumulates onto the chunk's biases (acc1[4 j + e] = b1[32 c + 8 j + 4 hh + e]),
        // read with uniform addresses (scalar loads: counted by lgkmcnt, so that waiting for them
        // does not wait for the stage's DMA, which vmcnt counts), each lane taking its half
#if !DK_MLPF32_EARLY_BIAS
#pragma unroll
        for (int m = 0; m < NC; ++m) bb[m] = b1[c * NC + m];
#endif
        f32x16_t acc1;
#pragma unroll
        for (int j = 0; j < 4; ++j)
#pragma unroll
            for (int e = 0; e < 4; ++e) acc1[4 * j + e] = hh ? bb[8 * j + 4 + e] : bb[8 * j + e];
        // (unconditional: the last chunk stages itself again into the idle buffer, so that every
        // path issues the same DMA count and the bias wait stays a counted vmcnt)
        // the next chunk's DMA is spread over GEMM1's k-steps, one wave instruction per k-step
        // (issued back to back at the top of the chunk, each cost ~100-185 issue cycles of the
        // wave while its MFMAs waited; MI355X_MICROARCH.md LDS-DMA issue cost)
        const uint32_t cn = c + 1 < chunks ? c + 1 : c;
        // GEMM1: D1 = W1_c h^T + b1 (one 32 x 32 tile), three products per k-step
        const uint16_t* a1 = cur + 8 * (NC * hh + r);
        // W1 fragments read one k-step ahead (the LDS latency under the previous k-step's MFMAs):
        // k-step kk's piece 2 kk + hh of row r
        auto w1f = [&](const uint16_t* base, int kk) { return *(const bf16x8_t*)(base + 16 * NC * kk); };
        bf16x8_t nh = w1f(a1, 0), nl = w1f(a1 + W1E, 0);
#pragma unroll
        for (int kk = 0; kk < KS; ++kk) {
            const bf16x8_t ah = nh, al = nl;
            if (kk + 1 < KS) { nh = w1f(a1, kk + 1); nl = w1f(a1 + W1E, kk + 1); }
            if (PER_MATRIX) __builtin_amdgcn_sched_barrier(0);   // the next reads stay a k-step ahead
#ifndef DK_SOL_NOGEMM1
            acc1 = __builtin_amdgcn_mfma_f32_32x32x16_bf16(al, hfh[kk], acc1, 0, 0, 0);
            acc1 = __builtin_amdgcn_mfma_f32_32x32x16_bf16(ah, hfl[kk], acc1, 0, 0, 0);
            acc1 = __builtin_amdgcn_mfma_f32_32x32x16_bf16(ah, hfh[kk], acc1, 0, 0, 0);
#else
            asm volatile("" :: "v"(ah), "v"(al));
#endif
#ifndef DK_SOL_NODMA
            // (scheduling barriers keep [next fragments' reads][MFMAs][DMA piece] in that order: the
            // DMA writes LDS, and the reads the scheduler would not move above it sat one MFMA
            // before their use)
            __builtin_amdgcn_sched_barrier(0);
            // DMA_PER_STEP pieces per k-step from the first: all issued early in GEMM1, so that their
            // landing latency (~1 us) runs under the rest of the chunk
#pragma unroll
            for (int q = 0; q < DMA_PER_STEP; ++q)
                if (DMA_PER_STEP * kk + q < NIW) stage_one(cn, nxt, DMA_PER_STEP * kk + q);
            if (kk == KS - 1)
#pragma unroll
                for (int ui = DMA_PER_STEP * KS; ui < NIW; ++ui) stage_one(cn, nxt, ui);   // (any rest here)
            __builtin_amdgcn_sched_barrier(0);
#endif
        }
        DK_FSTAMP(1);
        // GELU (f32) -> split B fragments of GEMM2 (k-step s = half: registers 8 s .. 8 s + 7,
        // hidden units 16 s + 4 hh + (g & 3) + 8 ((g >> 2) & 1))
        bf16x8_t afh[GS], afl[GS];
#pragma unroll
        for (int s2 = 0; s2 < GS; ++s2) {
            float g[8];
#pragma unroll
#ifndef DK_SOL_NOGELU
#if DK_MLPF32_PKGELU
            for (int t = 0; t < 8; t += 2) {
                const f32x2_t gg = gelu_poly_pk(f32x2_t{acc1[8 * s2 + t], acc1[8 * s2 + t + 1]});
                g[t] = gg.x;
                g[t + 1] = gg.y;
            }
#else
            for (int t = 0; t < 8; ++t) g[t] = gelu_poly(acc1[8 * s2 + t]);
#endif
#else
            for (int t = 0; t < 8; ++t) g[t] = acc1[8 * s2 + t];   // (speed-of-light measurement build)
#endif
            split_bf16x8(g, afh[s2], afl[s2]);
        }
        DK_FSTAMP(2);
        // GEMM2: D2 += W2_c a^T, OT tiles of 32 output columns, three products per k-step
        const uint16_t* a2h = cur + 2 * W1E + r * NC;
        const uint16_t* a2l = a2h + W2E;
        // W2 fragments read one (k-step, tile) ahead: tile t's row 32 t + r, piece 2 s + hh
        // (swizzled as GEMM1's pieces: rows 32 t + r and r share (row >> 2) & 3)
        auto w2f = [&](const uint16_t* base, int q) {
            return *(const bf16x8_t*)(base + (32 * (q % OT)) * NC + 8 * ((2 * (q / OT) + hh) ^ sw));
        };
        bf16x8_t ph = w2f(a2h, 0), pl = w2f(a2l, 0);
#pragma unroll
        for (int q = 0; q < GS * OT; ++q) {
            const int s2 = q / OT, t = q % OT;
            const bf16x8_t wh = ph, wl = pl;
            if (q + 1 < GS * OT) { ph = w2f(a2h, q + 1); pl = w2f(a2l, q + 1); }
            if (PER_MATRIX) __builtin_amdgcn_sched_barrier(0);   // (a tile ahead)
#ifndef DK_SOL_NOGEMM2
            acc2[t] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(wl, afh[s2], acc2[t], 0, 0, 0);
            acc2[t] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(wh, afl[s2], acc2[t], 0, 0, 0);
            acc2[t] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(wh, afh[s2], acc2[t], 0, 0, 0);
#else
            asm volatile("" :: "v"(wh), "v"(wl), "v"(afh[s2]), "v"(afl[s2]));
#endif
        }
        DK_FSTAMP(3);
#if DK_MLPF32_EARLY_BIAS
#pragma unroll
        for (int m = 0; m < NC; ++m) bb[m] = b1[cn * NC + m];   // (their latency under the wait below)
#endif
        __builtin_amdgcn_s_waitcnt(0);   // this wave's pieces of the next chunk have landed
        __syncthreads();                 // ... and every wave's; every wave is done with `cur`
        DK_FSTAMP(4);
    };
    for (uint32_t c = 0; c < chunks; c += 2) {
        chunk(c, lds0, lds1);
        if (c + 1 < chunks) chunk(c + 1, lds1, lds0);
    }
    // (XIN: the epilogue reads x again instead of the compiler keeping the prologue's x values
    // alive through the chunk loop, which spilled them)
    if constexpr (XIN) asm volatile("" ::: "memory");
    // epilogue: acc2[t][g] = delta of row `row`, column 32 t + 8 (g >> 2) + 4 hh + (g & 3);
    // x += (delta + b2) (the GEMM's bias first: F.linear's epilogue order), then LN
    // (all loads first, the stores under one branch: per-store branches kept every x load
    // behind the previous store)
    float* xr = x_io + (size_t)(ok ? row : 0u) * D;
    float s1 = 0.0f;
#pragma unroll
    for (int t = 0; t < OT; ++t)
#pragma unroll
        for (int q = 0; q < 4; ++q) {
            const int col = 32 * t + 8 * q + 4 * hh;
            const float4 xv = *(const float4*)(xr + col);
            const float4 bv = *(const float4*)(b2 + col);
            const float xn[4] = {xv.x + (acc2[t][4 * q] + bv.x), xv.y + (acc2[t][4 * q + 1] + bv.y),
                                 xv.z + (acc2[t][4 * q + 2] + bv.z), xv.w + (acc2[t][4 * q + 3] + bv.w)};
#pragma unroll
            for (int e = 0; e < 4; ++e) acc2[t][4 * q + e] = xn[e];
            s1 += (xn[0] + xn[1]) + (xn[2] + xn[3]);
        }
    s1 += __shfl_xor(s1, 32);
    const float mean = s1 / (float)D;
    float s2 = 0.0f;
#pragma unroll
    for (int t = 0; t < OT; ++t)
#pragma unroll
        for (int g = 0; g < 16; ++g) {
            const float dv = acc2[t][g] - mean;
            s2 += dv * dv;
        }
    s2 += __shfl_xor(s2, 32);
    const float rstd = rsqrtf(s2 / (float)D + eps);
    float* hr = h_out + (size_t)(ok ? row : 0u) * D;
    const bool wh = !XIN || h_out != nullptr;   // (uniform; XIN with h_out == nullptr: x only)
    if constexpr (XIN) {
        if (stats_out != nullptr && ok && hh == 0) stats_out[row] = make_float2(mean, rstd);
    }
    if (ok && !wh) {
#pragma unroll
        for (int t = 0; t < OT; ++t)
#pragma unroll
            for (int q = 0; q < 4; ++q)
                *(float4*)(xr + 32 * t + 8 * q + 4 * hh) =
                    make_float4(acc2[t][4 * q], acc2[t][4 * q + 1], acc2[t][4 * q + 2], acc2[t][4 * q + 3]);
    }
    if (ok && wh) {
#pragma unroll
        for (int t = 0; t < OT; ++t)
#pragma unroll
            for (int q = 0; q < 4; ++q) {
                const int col = 32 * t + 8 * q + 4 * hh;
                const float4 gv = *(const float4*)(gamma + col), bv = *(const float4*)(beta + col);
                *(float4*)(xr + col) = make_float4(acc2[t][4 * q], acc2[t][4 * q + 1], acc2[t][4 * q + 2], acc2[t][4 * q + 3]);
                *(float4*)(hr + col) = make_float4((acc2[t][4 * q] - mean) * rstd * gv.x + bv.x,
                                                   (acc2[t][4 * q + 1] - mean) * rstd * gv.y + bv.y,
                                                   (acc2[t][4 * q + 2] - mean) * rstd * gv.z + bv.z,
                                                   (acc2[t][4 * q + 3] - mean) * rstd * gv.w + bv.w);
            }
    }
    DK_FSTAMP(5);
#ifdef DK_NET_PROF
    if (lane == 0 && wave == 0) {
        for (int q = 0; q < 6; ++q) atomicAdd(&dk_mlp_prof_acc[q], facc[q]);
        // the shader clock over the workgroup's life: cycles (s_memtime) and 100 MHz ticks
        atomicAdd(&dk_mlp_prof_acc[6], __builtin_amdgcn_s_memtime() - f_t0);
        atomicAdd(&dk_mlp_prof_acc[7], __builtin_amdgcn_s_memrealtime() - f_r0);
    }
#endif
#undef DK_FSTAMP
}

// ---------------------------------------------------------------------------
// The MLP half at d = 256 with 16 rows per wave (v_mfma_f32_16x16x32_bf16): the 32-row form
// holds 128 registers of h fragments and 128 of output accumulators per wave at d = 256, so it
// runs one wave per SIMD, and each weight-DMA piece a wave issues (~100-185 cycles) idles the
// SIMD's MFMA pipe.  At 16 rows a wave holds half of each; eight waves x 16 rows = 128 rows per
// workgroup (the same weight staging per row), two waves per SIMD.
//   GEMM1 (per 32-hidden chunk, two 16 x 16 tiles): D1 = W1_c h^T; lane (n = row, kg) then holds
//     hidden 4 kg + j (tile 0) and 16 + 4 kg + j (tile 1), j < 4: bias + GELU + split in place ARE
//     the B fragment of GEMM2's 32-wide k-step (slot 8 kg + j), given W2's columns in the matching
//     order: within every 32-hidden group, slot q <- hidden (q & 7) < 4 ? 4 (q >> 3) + (q & 7) :
//     16 + 4 (q >> 3) + (q & 7) - 4 (az_network.mlp_split_bf16x3 at d = 256).
//   GEMM2: D2 = W2_c a^T over 16 output tiles of 16 columns.
// LDS as mlp_ln_f32x3_kernel: W1 chunk piece-major (a fragment read: 16 rows x 4 pieces, distinct
// bank quads), W2 chunk rows of 4 pieces with piece p at p ^ ((o & 4) >> 1) (conflict-free for the
// 16 x 16 x 32 A-fragment groups), double-buffered, DMA spread over GEMM1's k-steps.
// XIN: the input is the residual stream itself (h == nullptr), normalised here with the
// LayerNorm (gin, bin, eps_in) that its producer no longer applies; h_out == nullptr: x only is
// written (the next half normalises it) -- two of the four row-sized HBM transfers per half gone.
template <int D, int NC, bool XIN = false>
__global__ void __launch_bounds__(512, 1) mlp16_ln_f32x3_kernel(const float* __restrict__ h, float* __restrict__ x_io,
                                                              const uint16_t* __restrict__ w1h, const uint16_t* __restrict__ w1l,
                                                              const float* __restrict__ b1,
                                                              const uint16_t* __restrict__ w2h, const uint16_t* __restrict__ w2l,
                                                              const float* __restrict__ b2, uint32_t rows, uint32_t n_hidden,
                                                              const float* __restrict__ gamma, const float* __restrict__ beta,
                                                              float eps, float* __restrict__ h_out,
                                                              const float* __restrict__ gin = nullptr,
                                                              const float* __restrict__ bin = nullptr, float eps_in = 0.0f) {
    static_assert(D % 32 == 0 && NC == 32, "d: multiple of 32; chunks of 32 hidden units");
    constexpr int WAVES = 8;
    constexpr int KS = D / 32, OT = D / 16;                             // 32-wide k-steps, 16-column output tiles
    constexpr int W1E = NC * D, W2E = D * NC, BUF = 2 * (W1E + W2E);   // one buffer: W1 hi, W1 lo, W2 hi, W2 lo
    constexpr int Q1 = D / 8, Q2 = NC / 8;                              // 16-B pieces per row
    constexpr int NP = BUF / 8, NI = NP / 64, NIW = NI / WAVES;         // pieces, wave instructions (per wave)
    static_assert(NP % 64 == 0 && NI % WAVES == 0 && (NC * Q1) % 64 == 0 && (D * Q2) % 64 == 0, "whole instructions");
    __shared__ __attribute__((aligned(16))) uint16_t lds0[BUF];
    __shared__ __attribute__((aligned(16))) uint16_t lds1[BUF];
    const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63, n = lane & 15, kg = lane >> 4;
    const uint32_t row = blockIdx.x * (16u * WAVES) + (uint32_t)wave * 16u + (uint32_t)n;
    const bool ok = row < rows;
    // the row's h, split: lane (n, kg) holds k = 32 ks + 8 kg .. + 7 (rows past the end: row 0, never stored)
    bf16x8_t hfh[KS], hfl[KS];
    {
#ifdef DK_SOL_NOIO
        const float* hr = (XIN ? x_io : h) + 8 * kg;   // (measurement build: every row reads row 0, no HBM)
#else
        const float* hr = (XIN ? x_io : h) + (size_t)(ok ? row : 0u) * D + 8 * kg;
#endif
        float4 va[KS], vb[KS];
#pragma unroll
        for (int ks = 0; ks < KS; ++ks) {
            va[ks] = *(const float4*)(hr + 32 * ks);
            vb[ks] = *(const float4*)(hr + 32 * ks + 4);
        }
        float mu = 0.0f, rs = 1.0f;
        if constexpr (XIN) {
            // the row's LayerNorm over its four lanes (n, n + 16, n + 32, n + 48): two-pass
            float s1 = 0.0f;
#pragma unroll
            for (int ks = 0; ks < KS; ++ks) s1 += ((va[ks].x + va[ks].y) + (va[ks].z + va[ks].w)) + ((vb[ks].x + vb[ks].y) + (vb[ks].z + vb[ks].w));
            s1 += __shfl_xor(s1, 16);
            s1 += __shfl_xor(s1, 32);
            mu = s1 / (float)D;
            float s2 = 0.0f;
#pragma unroll
            for (int ks = 0; ks < KS; ++ks) {
                const float a0 = va[ks].x - mu, a1 = va[ks].y - mu, a2 = va[ks].z - mu, a3 = va[ks].w - mu;
                const float c0 = vb[ks].x - mu, c1 = vb[ks].y - mu, c2 = vb[ks].z - mu, c3 = vb[ks].w - mu;
                s2 += ((a0 * a0 + a1 * a1) + (a2 * a2 + a3 * a3)) + ((c0 * c0 + c1 * c1) + (c2 * c2 + c3 * c3));
            }
            s2 += __shfl_xor(s2, 16);
            s2 += __shfl_xor(s2, 32);
            rs = rsqrtf(s2 / (float)D + eps_in);
        }
#pragma unroll
        for (int ks = 0; ks < KS; ++ks) {
            float v[8] = {va[ks].x, va[ks].y, va[ks].z, va[ks].w, vb[ks].x, vb[ks].y, vb[ks].z, vb[ks].w};
            if constexpr (XIN) {
                const int c0 = 32 * ks + 8 * kg;
                const float4 g0 = *(const float4*)(gin + c0), g1 = *(const float4*)(gin + c0 + 4);
                const float4 e0 = *(const float4*)(bin + c0), e1 = *(const float4*)(bin + c0 + 4);
                const float g[8] = {g0.x, g0.y, g0.z, g0.w, g1.x, g1.y, g1.z, g1.w};
                const float be[8] = {e0.x, e0.y, e0.z, e0.w, e1.x, e1.y, e1.z, e1.w};
#pragma unroll
                for (int j = 0; j < 8; ++j) v[j] = (v[j] - mu) * rs * g[j] + be[j];
            }
            split_bf16x8(v, hfh[ks], hfl[ks]);
        }
    }
    typedef __attribute__((address_space(3))) void lds_void;
    // per-lane DMA source offsets (bytes): W1 (row lane & 31, piece lane >> 5 of the instruction's
    // pair); W2 (row lane >> 2 of the instruction's 16, piece lane & 3 swizzled by the row's bit 2)
    const int dma1 = 2 * ((lane & 31) * D + 8 * (lane >> 5));
    const int dma2 = 2 * ((lane >> 2) * (int)n_hidden + 8 * ((lane & 3) ^ (((lane >> 2) & 4) >> 1)));
    // The DMA goes through buffer_load ... lds (MUBUF: vmcnt only).  The FLAT-encoded
    // global_load_lds also counts in lgkmcnt, and while one is in flight the compiler can only
    // wait lgkmcnt(0) for an LDS read: every W fragment read then waited on the reads issued
    // after it, the whole point of reading ahead lost.
    const uint32_t wb1 = 2u * NC * D, wbytes = 2u * n_hidden * D;   // bytes: one chunk of W1, all of W1 / W2
    const __amdgpu_buffer_rsrc_t r1h = __builtin_amdgcn_make_buffer_rsrc((void*)w1h, (short)0, (int)wbytes, 0x00020000);
    const __amdgpu_buffer_rsrc_t r1l = __builtin_amdgcn_make_buffer_rsrc((void*)w1l, (short)0, (int)wbytes, 0x00020000);
    const __amdgpu_buffer_rsrc_t r2h = __builtin_amdgcn_make_buffer_rsrc((void*)w2h, (short)0, (int)wbytes, 0x00020000);
    const __amdgpu_buffer_rsrc_t r2l = __builtin_amdgcn_make_buffer_rsrc((void*)w2l, (short)0, (int)wbytes, 0x00020000);
    const int wv = __builtin_amdgcn_readfirstlane(wave);
    // instruction u = wv + WAVES ui: which matrix it stages depends on ui alone (each matrix is a
    // whole number of WAVES-instruction rounds), so after unrolling every branch below is static
    constexpr int N1 = NC * Q1 / 64, N2 = D * Q2 / 64;
    static_assert(N1 % WAVES == 0 && N2 % WAVES == 0, "matrix boundaries on instruction rounds");
    auto stage_one = [&](uint32_t c, uint16_t* dst, int ui) {
        const int u = wv + WAVES * ui;   // wave-uniform (SGPR)
        if (WAVES * ui < 2 * N1) {
            const bool lo = WAVES * ui >= N1;
            const int v = lo ? u - N1 : u;
            __builtin_amdgcn_raw_ptr_buffer_load_lds(lo ? r1l : r1h, (lds_void*)&dst[512 * u], 16, dma1,
                                                     (int)(c * wb1 + 32u * v), 0, 0);
        } else {
            const bool lo = WAVES * ui >= 2 * N1 + N2;
            const int v = u - 2 * N1 - (lo ? N2 : 0);
            __builtin_amdgcn_raw_ptr_buffer_load_lds(lo ? r2l : r2h, (lds_void*)&dst[512 * u], 16, dma2,
                                                     (int)(32u * v * n_hidden + 2u * c * NC), 0, 0);
        }
    };
    // GEMM1's biases for this lane (hidden 16 tt + 4 kg + j of the chunk), read a chunk ahead
    // during GEMM2, after the chunk's DMA has been issued (vmcnt retires in order)
    float4 bn0 = *(const float4*)(b1 + 4 * kg), bn1 = *(const float4*)(b1 + 16 + 4 * kg);
    f32x4_t acc2[OT];
#pragma unroll
    for (int t = 0; t < OT; ++t) acc2[t] = f32x4_t{0.0f, 0.0f, 0.0f, 0.0f};
    const uint32_t chunks = n_hidden / NC;
#pragma unroll
    for (int ui = 0; ui < NIW; ++ui) stage_one(0u, lds0, ui);
    __builtin_amdgcn_s_waitcnt(0);
    __syncthreads();
    const int sw2 = (n & 4) >> 1;   // W2 piece swizzle of rows 16 t + n
    // the residual rows of the epilogue: loaded in the last chunk, after its GEMM1 (the h
    // fragments' registers are free then), in flight under its GELU and GEMM2
    float4 xpre[OT];
#ifdef DK_SOL_NOIO
    float* xr = x_io;
#else
    float* xr = x_io + (size_t)(ok ? row : 0u) * D;
#endif
    auto chunk = [&](uint32_t c, const uint16_t* cur, uint16_t* nxt, auto last) {
        constexpr bool LAST = decltype(last)::value;
        // GEMM1 onto the chunk's biases
        f32x4_t acc1[2] = {f32x4_t{bn0.x, bn0.y, bn0.z, bn0.w}, f32x4_t{bn1.x, bn1.y, bn1.z, bn1.w}};
        const uint32_t cn = c + 1 < chunks ? c + 1 : c;
        // W1 fragment of tile tt, k-step ks: row 16 tt + n, piece 4 ks + kg (piece-major: (p NC + row) x 8)
        auto w1f = [&](const uint16_t* base, int tt, int ks) {
            return *(const bf16x8_t*)(base + 8 * ((4 * ks + kg) * NC + 16 * tt + n));
        };
        bf16x8_t nh0 = w1f(cur, 0, 0), nl0 = w1f(cur + W1E, 0, 0), nh1 = w1f(cur, 1, 0), nl1 = w1f(cur + W1E, 1, 0);
#pragma unroll
        for (int ks = 0; ks < KS; ++ks) {
            const bf16x8_t ah0 = nh0, al0 = nl0, ah1 = nh1, al1 = nl1;
            if (ks + 1 < KS) {
                nh0 = w1f(cur, 0, ks + 1); nl0 = w1f(cur + W1E, 0, ks + 1);
                nh1 = w1f(cur, 1, ks + 1); nl1 = w1f(cur + W1E, 1, ks + 1);
            }
            __builtin_amdgcn_sched_barrier(0);   // the next k-step's reads stay a whole k-step ahead
#ifndef DK_SOL_NOGEMM1
            acc1[0] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(al0, hfh[ks], acc1[0], 0, 0, 0);
            acc1[1] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(al1, hfh[ks], acc1[1], 0, 0, 0);
            acc1[0] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(ah0, hfl[ks], acc1[0], 0, 0, 0);
            acc1[1] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(ah1, hfl[ks], acc1[1], 0, 0, 0);
            acc1[0] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(ah0, hfh[ks], acc1[0], 0, 0, 0);
            acc1[1] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(ah1, hfh[ks], acc1[1], 0, 0, 0);
#else
            acc1[0][ks & 3] += (float)ah0[0] + (float)al0[1] + (float)ah1[2] + (float)al1[3];
#endif
            // the next chunk's DMA, one piece per k-step (issue cost under the MFMAs)
            __builtin_amdgcn_sched_barrier(0);
#ifndef DK_SOL_NODMA
            if (!LAST) {
                if (ks < NIW) stage_one(cn, nxt, ks);
                if (ks == KS - 1)
#pragma unroll
                    for (int ui = KS; ui < NIW; ++ui) stage_one(cn, nxt, ui);
            }
#endif
            __builtin_amdgcn_sched_barrier(0);
        }
        // GEMM2's W2 fragments ride a ring two tiles deep (tile t: row 16 t + n, piece kg ^ sw2);
        // the first two are read before the GELU so its VALU work covers their latency, and the
        // sched_barriers keep each read two tiles ahead of its MFMAs (left to itself the compiler
        // moved every read next to its use behind an lgkmcnt(0))
        const uint16_t* a2 = cur + 2 * W1E + n * NC + 8 * (kg ^ sw2);
        bf16x8_t rh[3], rl[3];
        rh[0] = *(const bf16x8_t*)a2; rl[0] = *(const bf16x8_t*)(a2 + W2E);
        rh[1] = *(const bf16x8_t*)(a2 + 16 * NC); rl[1] = *(const bf16x8_t*)(a2 + W2E + 16 * NC);
        if (!LAST) {
            bn0 = *(const float4*)(b1 + cn * NC + 4 * kg);
            bn1 = *(const float4*)(b1 + cn * NC + 16 + 4 * kg);
        } else {
#pragma unroll
            for (int t = 0; t < OT; ++t) xpre[t] = *(const float4*)(xr + 16 * t + 4 * kg);
        }
        __builtin_amdgcn_sched_barrier(0);
        // GELU (f32) -> the split B fragment of GEMM2's k-step: slots 0..3 tile 0, 4..7 tile 1
        bf16x8_t afh, afl;
        {
            float g[8];
#pragma unroll
            for (int j = 0; j < 4; ++j) {
                g[j] = gelu_poly(acc1[0][j]);
                g[4 + j] = gelu_poly(acc1[1][j]);
            }
            split_bf16x8(g, afh, afl);
        }
        __builtin_amdgcn_sched_barrier(0);
        // GEMM2: D2 += W2_c a^T
#pragma unroll
        for (int t = 0; t < OT; ++t) {
            if (t + 2 < OT) {
                rh[(t + 2) % 3] = *(const bf16x8_t*)(a2 + 16 * (t + 2) * NC);
                rl[(t + 2) % 3] = *(const bf16x8_t*)(a2 + W2E + 16 * (t + 2) * NC);
            }
            __builtin_amdgcn_sched_barrier(0);
            const bf16x8_t wh = rh[t % 3], wl = rl[t % 3];
#ifndef DK_SOL_NOGEMM2
            acc2[t] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(wl, afh, acc2[t], 0, 0, 0);
            acc2[t] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(wh, afl, acc2[t], 0, 0, 0);
            acc2[t] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(wh, afh, acc2[t], 0, 0, 0);
#else
            acc2[t][0] += (float)wh[0] + (float)wl[1] + (float)afh[2] + (float)afl[3];
#endif
            __builtin_amdgcn_sched_barrier(0);
        }
#ifndef DK_SOL_NOBAR
        if (!LAST) {
            __builtin_amdgcn_s_waitcnt(0);   // this wave's pieces of the next chunk have landed
            __syncthreads();                 // ... and every wave's; every wave is done with `cur`
        }
#endif
    };
    // (an even chunk count, checked on the host: the last chunk, peeled, computes from lds1)
    for (uint32_t c = 0; c + 2 < chunks; c += 2) {
        chunk(c, lds0, lds1, std::false_type{});
        chunk(c + 1, lds1, lds0, std::false_type{});
    }
    chunk(chunks - 2, lds0, lds1, std::false_type{});
    chunk(chunks - 1, lds1, lds0, std::true_type{});
    // epilogue: acc2[t][j] = delta of row `row`, column 16 t + 4 kg + j; x += (delta + b2), then LN
    // over the row's four lanes (n, n + 16, n + 32, n + 48)
    float s1 = 0.0f;
#pragma unroll
    for (int t = 0; t < OT; ++t) {
        const int col = 16 * t + 4 * kg;
        const float4 xv = xpre[t];
        const float4 bv = *(const float4*)(b2 + col);
        acc2[t][0] = xv.x + (acc2[t][0] + bv.x);
        acc2[t][1] = xv.y + (acc2[t][1] + bv.y);
        acc2[t][2] = xv.z + (acc2[t][2] + bv.z);
        acc2[t][3] = xv.w + (acc2[t][3] + bv.w);
        s1 += (acc2[t][0] + acc2[t][1]) + (acc2[t][2] + acc2[t][3]);
    }
    s1 += __shfl_xor(s1, 16);
    s1 += __shfl_xor(s1, 32);
    const float mean = s1 / (float)D;
    float s2 = 0.0f;
#pragma unroll
    for (int t = 0; t < OT; ++t)
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            const float dv = acc2[t][j] - mean;
            s2 += dv * dv;
        }
    s2 += __shfl_xor(s2, 16);
    s2 += __shfl_xor(s2, 32);
    const float rstd = rsqrtf(s2 / (float)D + eps);
    float* hr = h_out + (size_t)(ok ? row : 0u) * D;
    const bool wh = h_out != nullptr;   // (uniform)
#ifdef DK_SOL_NOIO
    if (ok && (rows >> 31)) {
#else
    if (ok) {
#endif
#pragma unroll
        for (int t = 0; t < OT; ++t) {
            const int col = 16 * t + 4 * kg;
            *(float4*)(xr + col) = make_float4(acc2[t][0], acc2[t][1], acc2[t][2], acc2[t][3]);
            if (wh) {
                const float4 gv = *(const float4*)(gamma + col), bv = *(const float4*)(beta + col);
                *(float4*)(hr + col) = make_float4((acc2[t][0] - mean) * rstd * gv.x + bv.x, (acc2[t][1] - mean) * rstd * gv.y + bv.y,
                                                   (acc2[t][2] - mean) * rstd * gv.z + bv.z, (acc2[t][3] - mean) * rstd * gv.w + bv.w);
            }
        }
    }
}

// ---------------------------------------------------------------------------
// The whole attention half of a block at the reference's precision (round 5), one 256-thread
// workgroup per sample (as qkv_attn_ln_kernel at bf16):
//   Q, K, V = W h^T + b            (head w on wave w; bf16x3 products, f32 accumulators)
//   P = softmax(K Q^T * scale)      (bf16x3 products; softmax in f32)
//   y = P V                         (bf16x3 products)
//   delta = y Wp^T;  x += delta + bp;  h' = LN(x)        (bf16x3 products; f32 residual and LN)
// with the folded out / c projection (Block.folded_proj).  Every operand is split into bf16
// hi + lo and each k-step takes three MFMAs (A_lo B_hi + A_hi B_lo + A_hi B_hi), as
// mlp_ln_f32x3_kernel.  The weights come pre-split (wq_hi / wq_lo [3d][d], wp_hi / wp_lo [d][d]).
// Unfused (hipBLASLt qkv GEMM, the f32 attention kernel, the projection GEMM, add + LN), q, k, v
// (12 d bytes per token), y and delta went to HBM and back.
// LDS, one region reused in turn: the sample's h rows (hi, lo) -> the heads' V^T tiles (hi, lo)
// -> y rows (hi, lo) -> the residual rows (f32).
// DT1: compute the second 32-row tile (head dims 32 .. HD - 1) here; without it (HD = 40: the
// tails of Q, K and V come from one shared tile, tail_tiles_x3) acc[1] is left zero.
template <int HD, int D, bool DT1 = true>
__device__ __forceinline__ void head_tiles_x3(const uint16_t* hsh, const uint16_t* hsl, const uint16_t* __restrict__ wh,
                                              const uint16_t* __restrict__ wl, const float* __restrict__ bias,
                                              f32x16_t (&acc)[2][2]) {
    constexpr int LDY = D + 8, NKS = D / 16;
    const int lane = threadIdx.x & 63, r = lane & 31, hh = lane >> 5;
#pragma unroll
    for (int dt = 0; dt < 2; ++dt)
#pragma unroll
        for (int si = 0; si < 2; ++si) acc[dt][si] = f32x16_t{0};
    const size_t o0 = (size_t)r * D, o1 = (size_t)(32 + r < HD ? 32 + r : 0) * D;
    // W fragments PF k-steps ahead in a register ring (HD = 64, two waves per SIMD: two steps;
    // HD = 40 keeps one and its third wave per SIMD)
#ifndef DK_ATTN_PF64
#define DK_ATTN_PF64 2
#endif
    constexpr int PF = HD == 64 ? DK_ATTN_PF64 : 1;
    bf16x8_t ring[PF][2][2];
    auto wfr = [&](int ks, bf16x8_t (&nw)[2][2]) {
        const int k0 = 16 * ks + 8 * hh;
        nw[0][0] = load_frag8(wh + o0 + k0, true);
        nw[0][1] = load_frag8(wl + o0 + k0, true);
        // (rows past HD load row 0, unconditionally: a load under a lane condition made the
        // compiler wait for the next k-step's loads; the rows' outputs are zeroed below)
        if (DT1) {
            nw[1][0] = load_frag8(wh + o1 + k0, true);
            nw[1][1] = load_frag8(wl + o1 + k0, true);
        } else {
            nw[1][0] = nw[0][0];
            nw[1][1] = nw[0][1];
        }
    };
#pragma unroll
    for (int p = 0; p < PF; ++p) wfr(p, ring[p]);
#pragma unroll
    for (int ks = 0; ks < NKS; ++ks) {
        auto& nw = ring[ks % PF];
        const bf16x8_t a0h = nw[0][0], a0l = nw[0][1], a1h = nw[1][0], a1l = nw[1][1];
        if (ks + PF < NKS) wfr(ks + PF, nw);
        // (the next k-step's loads stay at the top: left to the scheduler they sank to the end of
        // the step, reusing the current operands' registers, and the next step waited for them)
        __builtin_amdgcn_sched_barrier(0);
        bf16x8_t bhf[2], blf[2];
#pragma unroll
        for (int si = 0; si < 2; ++si) {
            bhf[si] = *(const bf16x8_t*)&hsh[(32 * si + r) * LDY + 16 * ks + 8 * hh];
            blf[si] = *(const bf16x8_t*)&hsl[(32 * si + r) * LDY + 16 * ks + 8 * hh];
        }
#pragma unroll
        for (int si = 0; si < 2; ++si) {
            acc[0][si] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a0l, bhf[si], acc[0][si], 0, 0, 0);
            acc[0][si] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a0h, blf[si], acc[0][si], 0, 0, 0);
            acc[0][si] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a0h, bhf[si], acc[0][si], 0, 0, 0);
            if (HD > 32 && DT1) {
                acc[1][si] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a1l, bhf[si], acc[1][si], 0, 0, 0);
                acc[1][si] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a1h, blf[si], acc[1][si], 0, 0, 0);
                acc[1][si] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a1h, bhf[si], acc[1][si], 0, 0, 0);
            }
        }
        // (keeps the compiler from hoisting every k-step's W loads to the top: registers)
        __builtin_amdgcn_sched_barrier(0);
    }
#pragma unroll
    for (int dt = 0; dt < 2; ++dt)
#pragma unroll
        for (int g = 0; g < 16; ++g) {
            const int m = 32 * dt + (g & 3) + 8 * (g >> 2) + 4 * hh;
            const bool real = m < HD && (DT1 || dt == 0);   // (for HD = 40: register g < 4 of tile 1)
            const float bv = real ? bias[m] : 0.0f;
            acc[dt][0][g] = real ? acc[dt][0][g] + bv : 0.0f;
            acc[dt][1][g] = real ? acc[dt][1][g] + bv : 0.0f;
        }
}

// HD = 40: the head dims 32..39 of Q, K and V as ONE 32-row tile -- A row r is row 32 + (r & 7)
// of projection r >> 3 (Q, K, V; rows 24..31 repeat Q's and are discarded) -- instead of three
// tiles of which a quarter is real: 60 MFMAs for the three tails instead of 180.  The result:
// tail[si] register g < 4 (+ 4 p) holds projection p's dim 32 + (g & 3) + 4 hh of token 32 si + r
// (the register order of tile 1 of head_tiles_x3), bias included.
template <int HD, int D>
__device__ __forceinline__ void tail_tiles_x3(const uint16_t* hsh, const uint16_t* hsl, const uint16_t* __restrict__ wh,
                                              const uint16_t* __restrict__ wl, const float* __restrict__ bias,
                                              f32x16_t (&tail)[2]) {
    static_assert(HD > 32 && 3 * (HD - 32) <= 32 && (HD - 32) == 8, "three tails of 8 rows in one tile");
    constexpr int LDY = D + 8, NKS = D / 16;
    const int lane = threadIdx.x & 63, r = lane & 31, hh = lane >> 5;
    const int pr = (r >> 3) < 3 ? (r >> 3) : 0;
    const size_t o = (size_t)pr * D * D + (size_t)(32 + (r & 7)) * D;
    tail[0] = f32x16_t{0};
    tail[1] = f32x16_t{0};
    bf16x8_t nh = load_frag8(wh + o + 8 * hh, true), nl = load_frag8(wl + o + 8 * hh, true);
#pragma unroll
    for (int ks = 0; ks < NKS; ++ks) {
        const bf16x8_t ah = nh, al = nl;
        if (ks + 1 < NKS) {
            nh = load_frag8(wh + o + 16 * (ks + 1) + 8 * hh, true);
            nl = load_frag8(wl + o + 16 * (ks + 1) + 8 * hh, true);
        }
        __builtin_amdgcn_sched_barrier(0);
        bf16x8_t bhf[2], blf[2];
#pragma unroll
        for (int si = 0; si < 2; ++si) {
            bhf[si] = *(const bf16x8_t*)&hsh[(32 * si + r) * LDY + 16 * ks + 8 * hh];
            blf[si] = *(const bf16x8_t*)&hsl[(32 * si + r) * LDY + 16 * ks + 8 * hh];
        }
#pragma unroll
        for (int si = 0; si < 2; ++si) {
            tail[si] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(al, bhf[si], tail[si], 0, 0, 0);
            tail[si] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(ah, blf[si], tail[si], 0, 0, 0);
            tail[si] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(ah, bhf[si], tail[si], 0, 0, 0);
        }
        __builtin_amdgcn_sched_barrier(0);
    }
    // bias: register g of projection p = g >> 2 (< 3), dim 32 + (g & 3) + 4 hh; bias points at
    // the head's Q bias, K's and V's are D and 2 D further
#pragma unroll
    for (int g = 0; g < 12; ++g) {
        const float bv = bias[(g >> 2) * D + 32 + (g & 3) + 4 * hh];
        tail[0][g] += bv;
        tail[1][g] += bv;
    }
}

// Q^T / K^T accumulators -> hi / lo fragments of the attention's k-steps (pack_head's order)
template <int HD>
__device__ __forceinline__ void split_head(const f32x16_t (&acc)[2][2], bf16x8_t (&fh)[2][(HD + 15) / 16],
                                           bf16x8_t (&fl)[2][(HD + 15) / 16]) {
#pragma unroll
    for (int si = 0; si < 2; ++si)
#pragma unroll
        for (int kk = 0; kk < (HD + 15) / 16; ++kk) {
            float v[8];
#pragma unroll
            for (int j = 0; j < 8; ++j) v[j] = acc[kk >> 1][si][8 * (kk & 1) + j];
            split_bf16x8(v, fh[si][kk], fl[si][kk]);
        }
}

// XIN (as mlp16_ln_f32x3_kernel): the sample's rows come from x_io (h_in unused) and are
// normalised here with (gin, bin, eps_in); h_out == nullptr: x only is written.  x_out != nullptr:
// the new x goes there and x_io is only read (a branch starting from a shared trunk's x without a
// copy of it).
template <int HD, bool XIN = false>
__global__ void __launch_bounds__(256, HD == 40 ? 3 : 2) qkv_attn_ln_f32x3_kernel(const float* __restrict__ h_in, float* __restrict__ x_io,
                                                                   const uint16_t* __restrict__ wqh, const uint16_t* __restrict__ wql,
                                                                   const float* __restrict__ bqkv,
                                                                   const uint16_t* __restrict__ wph, const uint16_t* __restrict__ wpl,
                                                                   const float* __restrict__ bp, float scale,
                                                                   const float* __restrict__ gamma, const float* __restrict__ beta,
                                                                   float eps, float* __restrict__ h_out,
                                                                   const float* __restrict__ gin = nullptr,
                                                                   const float* __restrict__ bin = nullptr, float eps_in = 0.0f,
                                                                   const float2* __restrict__ stats_in = nullptr,
                                                                   float2* __restrict__ stats_out = nullptr,
                                                                   float* __restrict__ x_out = nullptr) {
    constexpr int S = 62, D = HD * 4, LDY = D + 8, LDT = 64 + 4, KS = (HD + 15) / 16, LDX = D + 4;
    constexpr bool TAIL3 = HD == 40;                       // the three projections' dims 32..39 in one tile
    constexpr bool PERDT = HD == 64;                       // Q / K one 32-dim tile at a time
    constexpr int RH = 2 * 64 * LDY;                       // h rows / y rows: hi then lo (bf16 elements)
    constexpr int RV = 2 * 4 * HD * LDT;                   // the V^T tiles: hi then lo
    constexpr int RX = 2 * 64 * LDX;                       // the residual rows (f32, in bf16 elements)
    constexpr int R = RH > RV ? (RH > RX ? RH : RX) : (RV > RX ? RV : RX);
    __shared__ __attribute__((aligned(16))) uint16_t lds[R];
    const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63, r = lane & 31, hh = lane >> 5;
    const uint32_t b = blockIdx.x;
    uint16_t* hsh = lds;
    uint16_t* hsl = lds + 64 * LDY;
    // the sample's h rows, split; rows 62, 63 zero
    const float* hg = (XIN ? x_io : h_in) + (size_t)b * S * D;
    if constexpr (XIN && D == 160) {
        // XIN at d = 160 (round 6): four threads per row (64 rows), thread q of a row holds its
        // pieces 5 q .. 5 q + 4 (40 values), so the row's LayerNorm reduces over lanes ^1, ^2;
        // every load issued first; rows 62, 63 zero
        constexpr int PPT = D / 8 / 4;                     // pieces per thread
        const int rr = threadIdx.x >> 2, q4 = threadIdx.x & 3;
        const bool ok = rr < S;
        const float* src = hg + (size_t)(ok ? rr : S - 1) * D + 8 * PPT * q4;
        float4 va[PPT], vb[PPT];
#pragma unroll
        for (int i = 0; i < PPT; ++i) { va[i] = *(const float4*)(src + 8 * i); vb[i] = *(const float4*)(src + 8 * i + 4); }
        // the row statistics: the producer's (stats_in), else a two-pass reduction over the 4 lanes
        float mu, rs;
        if (stats_in != nullptr) {   // (uniform)
            const float2 st = stats_in[(size_t)b * S + (ok ? rr : S - 1)];
            mu = st.x; rs = st.y;
        } else {
            float s1 = 0.0f;
#pragma unroll
            for (int i = 0; i < PPT; ++i) s1 += ((va[i].x + va[i].y) + (va[i].z + va[i].w)) + ((vb[i].x + vb[i].y) + (vb[i].z + vb[i].w));
            s1 += __shfl_xor(s1, 1);
            s1 += __shfl_xor(s1, 2);
            mu = s1 / (float)D;
            float s2 = 0.0f;
#pragma unroll
            for (int i = 0; i < PPT; ++i) {
                const float v[8] = {va[i].x, va[i].y, va[i].z, va[i].w, vb[i].x, vb[i].y, vb[i].z, vb[i].w};
#pragma unroll
                for (int j = 0; j < 8; ++j) s2 += (v[j] - mu) * (v[j] - mu);
            }
            s2 += __shfl_xor(s2, 1);
            s2 += __shfl_xor(s2, 2);
            rs = rsqrtf(s2 / (float)D + eps_in);
        }
#pragma unroll
        for (int i = 0; i < PPT; ++i) {
            const int kp = PPT * q4 + i, c0 = 8 * kp;
            const float4 g0 = *(const float4*)(gin + c0), g1 = *(const float4*)(gin + c0 + 4);
            const float4 e0 = *(const float4*)(bin + c0), e1 = *(const float4*)(bin + c0 + 4);
            const float g[8] = {g0.x, g0.y, g0.z, g0.w, g1.x, g1.y, g1.z, g1.w};
            const float be[8] = {e0.x, e0.y, e0.z, e0.w, e1.x, e1.y, e1.z, e1.w};
            const float x8[8] = {va[i].x, va[i].y, va[i].z, va[i].w, vb[i].x, vb[i].y, vb[i].z, vb[i].w};
            float v[8];
#pragma unroll
            for (int j = 0; j < 8; ++j) v[j] = ok ? (x8[j] - mu) * rs * g[j] + be[j] : 0.0f;
            bf16x8_t fh, fl;
            split_bf16x8(v, fh, fl);
            *(bf16x8_t*)&hsh[rr * LDY + c0] = fh;
            *(bf16x8_t*)&hsl[rr * LDY + c0] = fl;
        }
    } else {
        // every load issued before the first split / LDS store (a load -> store loop waited a
        // memory round trip per iteration); rows 62, 63 zero
        constexpr int NPC = 64 * (D / 8) / 256;
        static_assert(64 * (D / 8) % 256 == 0, "whole pieces per thread");
        float4 va[NPC], vb[NPC];
#pragma unroll
        for (int i = 0; i < NPC; ++i) {
            const int p = threadIdx.x + 256 * i, rr = p / (D / 8), kp = p - rr * (D / 8);
            const float* src = hg + (size_t)(rr < S ? rr : S - 1) * D + 8 * kp;
            va[i] = *(const float4*)src;
            vb[i] = *(const float4*)(src + 4);
        }
        // XIN: each row's D / 8 pieces sit on D / 8 consecutive lanes (the same piece index kp for
        // every i): the row's LayerNorm reduces over them, two-pass
        static_assert(!XIN || (D / 8 == 32 && 256 % (D / 8) == 0), "XIN here: a row on one half-wave (d = 160 above)");
        float4 xg0{}, xg1{}, xe0{}, xe1{};
        if constexpr (XIN) {
            const int c0 = 8 * (threadIdx.x & (D / 8 - 1));
            xg0 = *(const float4*)(gin + c0); xg1 = *(const float4*)(gin + c0 + 4);
            xe0 = *(const float4*)(bin + c0); xe1 = *(const float4*)(bin + c0 + 4);
        }
#pragma unroll
        for (int i = 0; i < NPC; ++i) {
            const int p = threadIdx.x + 256 * i, rr = p / (D / 8), kp = p - rr * (D / 8);
            const bool ok = rr < S;
            float v[8] = {va[i].x, va[i].y, va[i].z, va[i].w, vb[i].x, vb[i].y, vb[i].z, vb[i].w};
            if constexpr (XIN) {
                float s1 = ((v[0] + v[1]) + (v[2] + v[3])) + ((v[4] + v[5]) + (v[6] + v[7]));
#pragma unroll
                for (int o = 1; o < D / 8; o <<= 1) s1 += __shfl_xor(s1, o);
                const float mu = s1 / (float)D;
                float s2 = 0.0f;
#pragma unroll
                for (int j = 0; j < 8; ++j) s2 += (v[j] - mu) * (v[j] - mu);
#pragma unroll
                for (int o = 1; o < D / 8; o <<= 1) s2 += __shfl_xor(s2, o);
                const float rs = rsqrtf(s2 / (float)D + eps_in);
                const float g[8] = {xg0.x, xg0.y, xg0.z, xg0.w, xg1.x, xg1.y, xg1.z, xg1.w};
                const float be[8] = {xe0.x, xe0.y, xe0.z, xe0.w, xe1.x, xe1.y, xe1.z, xe1.w};
#pragma unroll
                for (int j = 0; j < 8; ++j) v[j] = (v[j] - mu) * rs * g[j] + be[j];
            }
#pragma unroll
            for (int j = 0; j < 8; ++j) v[j] = ok ? v[j] : 0.0f;
            bf16x8_t fh, fl;
            split_bf16x8(v, fh, fl);
            *(bf16x8_t*)&hsh[rr * LDY + 8 * kp] = fh;
            *(bf16x8_t*)&hsl[rr * LDY + 8 * kp] = fl;
        }
    }
    __syncthreads();
    // Register budget: Q^T and K^T into split fragments, then X = K Q^T and the softmax (Q / K
    // dead), then the V^T projection while only P is live; V^T goes to LDS once every wave is
    // done with the h rows.
    const size_t hq = (size_t)wave * HD * D;
    bf16x8_t pfh[2][4], pfl[2][4];
    float vtail[2][4];                                     // V^T dims 32..39 (HD = 40), kept for the V tile
    {
        // (PERDT: the fragments of one 32-dim tile, two k-steps)
        bf16x8_t qfh[2][PERDT ? 2 : KS], qfl[2][PERDT ? 2 : KS], kfh[2][PERDT ? 2 : KS], kfl[2][PERDT ? 2 : KS];
        {
            f32x16_t acc[2][2];
            if constexpr (TAIL3) {
                // dims 32..39 of Q, K and V from one shared tile, dims 0..31 per projection
                f32x16_t tl[2];
                tail_tiles_x3<HD, D>(hsh, hsl, wqh + hq, wql + hq, bqkv + wave * HD, tl);
#pragma unroll
                for (int si = 0; si < 2; ++si)
#pragma unroll
                    for (int g = 0; g < 4; ++g) vtail[si][g] = tl[si][8 + g];
                head_tiles_x3<HD, D, false>(hsh, hsl, wqh + hq, wql + hq, bqkv + wave * HD, acc);             // Q^T
#pragma unroll
                for (int si = 0; si < 2; ++si)
#pragma unroll
                    for (int g = 0; g < 4; ++g) acc[1][si][g] = tl[si][g];
                split_head<HD>(acc, qfh, qfl);
                head_tiles_x3<HD, D, false>(hsh, hsl, wqh + hq + (size_t)D * D, wql + hq + (size_t)D * D, bqkv + D + wave * HD,
                                            acc);                                                            // K^T
#pragma unroll
                for (int si = 0; si < 2; ++si)
#pragma unroll
                    for (int g = 0; g < 4; ++g) acc[1][si][g] = tl[si][4 + g];
                split_head<HD>(acc, kfh, kfl);
            } else if constexpr (!PERDT) {
                head_tiles_x3<HD, D>(hsh, hsl, wqh + hq, wql + hq, bqkv + wave * HD, acc);                      // Q^T
                split_head<HD>(acc, qfh, qfl);
                head_tiles_x3<HD, D>(hsh, hsl, wqh + hq + (size_t)D * D, wql + hq + (size_t)D * D, bqkv + D + wave * HD, acc);   // K^T
                split_head<HD>(acc, kfh, kfl);
            }
        }
        // X[ti][si] = K_ti Q_si^T, three products per k-step
        f32x16_t x[2][2];
        if constexpr (PERDT) {
            // HD = 64: Q^T and K^T one 32-dim tile at a time, X accumulated over the two (all four
            // heads' fragments at once would not fit two waves per SIMD)
#pragma unroll
            for (int ti = 0; ti < 2; ++ti)
#pragma unroll
                for (int si = 0; si < 2; ++si) x[ti][si] = f32x16_t{0};
#pragma unroll
            for (int dt = 0; dt < 2; ++dt) {
                const size_t ro = hq + (size_t)32 * dt * D;
                f32x16_t acc[2][2];
                head_tiles_x3<HD, D, false>(hsh, hsl, wqh + ro, wql + ro, bqkv + wave * HD + 32 * dt, acc);              // Q^T dims 32 dt ..
                split_head<32>(acc, qfh, qfl);
                head_tiles_x3<HD, D, false>(hsh, hsl, wqh + ro + (size_t)D * D, wql + ro + (size_t)D * D,
                                            bqkv + D + wave * HD + 32 * dt, acc);                                        // K^T
                split_head<32>(acc, kfh, kfl);
#pragma unroll
                for (int ti = 0; ti < 2; ++ti)
#pragma unroll
                    for (int si = 0; si < 2; ++si)
#pragma unroll
                        for (int kk = 0; kk < 2; ++kk) {
                            x[ti][si] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(kfl[ti][kk], qfh[si][kk], x[ti][si], 0, 0, 0);
                            x[ti][si] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(kfh[ti][kk], qfl[si][kk], x[ti][si], 0, 0, 0);
                            x[ti][si] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(kfh[ti][kk], qfh[si][kk], x[ti][si], 0, 0, 0);
                        }
            }
        } else {
#pragma unroll
        for (int ti = 0; ti < 2; ++ti)
#pragma unroll
            for (int si = 0; si < 2; ++si) {
                f32x16_t acc = {0};
#pragma unroll
                for (int kk = 0; kk < KS; ++kk) {
                    acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(kfl[ti][kk], qfh[si][kk], acc, 0, 0, 0);
                    acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(kfh[ti][kk], qfl[si][kk], acc, 0, 0, 0);
                    acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(kfh[ti][kk], qfh[si][kk], acc, 0, 0, 0);
                }
                x[ti][si] = acc;
            }
        }
        // softmax over the keys t of every query column s (f32), P split
#pragma unroll
        for (int si = 0; si < 2; ++si) {
            float m = -INFINITY;
#pragma unroll
            for (int ti = 0; ti < 2; ++ti)
#pragma unroll
                for (int g = 0; g < 16; ++g) {
                    const int t = 32 * ti + (g & 3) + 8 * (g >> 2) + 4 * hh;
                    x[ti][si][g] *= scale;
                    if (t < S) m = fmaxf(m, x[ti][si][g]);
                }
            m = fmaxf(m, __shfl_xor(m, 32));
            float l = 0.0f;
#pragma unroll
            for (int ti = 0; ti < 2; ++ti)
#pragma unroll
                for (int g = 0; g < 16; ++g) {
                    const int t = 32 * ti + (g & 3) + 8 * (g >> 2) + 4 * hh;
                    const float pv = t < S ? expf(x[ti][si][g] - m) : 0.0f;
                    x[ti][si][g] = pv;
                    l += pv;
                }
            l += __shfl_xor(l, 32);
            const float inv = 1.0f / l;
#pragma unroll
            for (int q = 0; q < 4; ++q) {
                float v[8];
#pragma unroll
                for (int jj = 0; jj < 8; ++jj) v[jj] = x[q >> 1][si][8 * (q & 1) + jj] * inv;
                split_bf16x8(v, pfh[si][q], pfl[si][q]);
            }
        }
    }
    f32x16_t vacc[2][2];
    head_tiles_x3<HD, D, !TAIL3>(hsh, hsl, wqh + hq + (size_t)2 * D * D, wql + hq + (size_t)2 * D * D, bqkv + 2 * D + wave * HD,
                                 vacc);                                                                   // V^T
    if constexpr (TAIL3) {
#pragma unroll
        for (int si = 0; si < 2; ++si)
#pragma unroll
            for (int g = 0; g < 4; ++g) vacc[1][si][g] = vtail[si][g];
    }
    __syncthreads();   // every wave is done with the h rows
    uint16_t* vth = lds + wave * HD * LDT;
    uint16_t* vtl = lds + 4 * HD * LDT + wave * HD * LDT;
#pragma unroll
    for (int dt = 0; dt < 2; ++dt)
#pragma unroll
        for (int g = 0; g < 16; ++g) {
            const int m = 32 * dt + (g & 3) + 8 * (g >> 2) + 4 * hh;
            if (m < HD) {
#pragma unroll
                for (int si = 0; si < 2; ++si) {
                    const float v = vacc[dt][si][g];
                    const uint16_t hi = f2bf(v);
                    vth[m * LDT + 32 * si + r] = hi;
                    vtl[m * LDT + 32 * si + r] = f2bf(v - bf2f(hi));
                }
            }
        }
    __syncthreads();   // V^T tiles complete
    // O[si][et] = P_si V_et, three products per k-step; y kept in registers until the V^T tiles
    // are dead
    f32x16_t yo[2][2];
#pragma unroll
    for (int et = 0; et < 2; ++et) {
        const int e = 32 * et + r, er = e < HD ? e : HD - 1;
        bf16x8_t vfh[4], vfl[4];
        if (32 * et < HD) {
#pragma unroll
            for (int q = 0; q < 4; ++q) {
                const int t0 = 16 * q + 4 * hh;
                union { uint2 u[2]; bf16x8_t v; } fh, fl;
                fh.u[0] = *(const uint2*)&vth[er * LDT + t0]; fh.u[1] = *(const uint2*)&vth[er * LDT + t0 + 8];
                fl.u[0] = *(const uint2*)&vtl[er * LDT + t0]; fl.u[1] = *(const uint2*)&vtl[er * LDT + t0 + 8];
                vfh[q] = fh.v; vfl[q] = fl.v;
            }
        }
#pragma unroll
        for (int si = 0; si < 2; ++si) {
            f32x16_t acc = {0};
            if (32 * et < HD) {
#pragma unroll
                for (int q = 0; q < 4; ++q) {
                    acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(pfl[si][q], vfh[q], acc, 0, 0, 0);
                    acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(pfh[si][q], vfl[q], acc, 0, 0, 0);
                    acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(pfh[si][q], vfh[q], acc, 0, 0, 0);
                }
            }
            yo[si][et] = acc;
        }
    }
    __syncthreads();   // every wave is done with the V^T tiles
    // y rows (hi, lo) into LDS: y[s][wave HD + e]; rows 62, 63 stay zero (A operand padding)
    uint16_t* ysh = lds;
    uint16_t* ysl = lds + 64 * LDY;
#pragma unroll
    for (int si = 0; si < 2; ++si)
#pragma unroll
        for (int et = 0; et < 2; ++et) {
            const int e = 32 * et + r;
            if (e < HD) {
#pragma unroll
                for (int g = 0; g < 16; ++g) {
                    const int sidx = 32 * si + (g & 3) + 8 * (g >> 2) + 4 * hh;
                    const float v = sidx < S ? yo[si][et][g] : 0.0f;
                    const uint16_t hi = f2bf(v);
                    ysh[sidx * LDY + wave * HD + e] = hi;
                    ysl[sidx * LDY + wave * HD + e] = f2bf(v - bf2f(hi));
                }
            }
        }
    __syncthreads();   // y complete
    // delta = y Wp^T (v_mfma_f32_16x16x32_bf16; the wave's column tiles wave + 4 j over all 64 rows)
    constexpr int NT = D / 16, KP = D / 32, NJ = (NT + 3) / 4;
    const int rl = lane & 15, kg = lane >> 4;
    f32x4_t acc[4][NJ];
#pragma unroll
    for (int m = 0; m < 4; ++m)
#pragma unroll
        for (int j = 0; j < NJ; ++j) acc[m][j] = f32x4_t{0.0f, 0.0f, 0.0f, 0.0f};
    // Wp fragments one k-step ahead, issued at the top of the step (each loaded and consumed in
    // place had every (k-step, tile) wait a full L2 round trip); tiles past NT load tile 0, unused
    bf16x8_t pcur[NJ][2], pnxt[NJ][2];
    auto wpf = [&](int ks, bf16x8_t (&dst)[NJ][2]) {
#pragma unroll
        for (int j = 0; j < NJ; ++j) {
            const int t = wave + 4 * j;
            const size_t wo = (size_t)(16 * (t < NT ? t : 0) + rl) * D + 32 * ks + 8 * kg;
            dst[j][0] = load_frag8(wph + wo, true);
            dst[j][1] = load_frag8(wpl + wo, true);
        }
    };
    wpf(0, pcur);
#pragma unroll
    for (int ks = 0; ks < KP; ++ks) {
        if (ks + 1 < KP) wpf(ks + 1, pnxt);
        __builtin_amdgcn_sched_barrier(0);
        bf16x8_t ah[4], al[4];
#pragma unroll
        for (int m = 0; m < 4; ++m) {
            ah[m] = *(const bf16x8_t*)&ysh[(16 * m + rl) * LDY + 32 * ks + 8 * kg];
            al[m] = *(const bf16x8_t*)&ysl[(16 * m + rl) * LDY + 32 * ks + 8 * kg];
        }
#pragma unroll
        for (int j = 0; j < NJ; ++j) {
            const int t = wave + 4 * j;
            if (t < NT) {
                const bf16x8_t bh = pcur[j][0], bl = pcur[j][1];
#pragma unroll
                for (int m = 0; m < 4; ++m) {
                    acc[m][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(al[m], bh, acc[m][j], 0, 0, 0);
                    acc[m][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(ah[m], bl, acc[m][j], 0, 0, 0);
                    acc[m][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(ah[m], bh, acc[m][j], 0, 0, 0);
                }
            }
        }
        __builtin_amdgcn_sched_barrier(0);
#pragma unroll
        for (int j = 0; j < NJ; ++j) {
            pcur[j][0] = pnxt[j][0];
            pcur[j][1] = pnxt[j][1];
        }
    }
    __syncthreads();   // every wave is done with the y rows
    // the residual rows (f32) into LDS, x' = x + (delta + bp) in place
    float* xs = reinterpret_cast<float*>(lds);
    const float* xg = x_io + (size_t)b * S * D;
    {
        // all residual loads first (clamped to the last piece), then the LDS stores
        constexpr int NX = (S * (D / 4) + 255) / 256;
        float4 v[NX];
#pragma unroll
        for (int i = 0; i < NX; ++i) {
            const int p = threadIdx.x + 256 * i;
            v[i] = *(const float4*)(xg + 4 * (p < S * (D / 4) ? p : S * (D / 4) - 1));
        }
#pragma unroll
        for (int i = 0; i < NX; ++i) {
            const int p = threadIdx.x + 256 * i, rr = p / (D / 4), kp = p - rr * (D / 4);
            if (p < S * (D / 4)) *(float4*)&xs[rr * LDX + 4 * kp] = v[i];
        }
    }
    __syncthreads();
#pragma unroll
    for (int j = 0; j < NJ; ++j) {
        const int t = wave + 4 * j;
        if (t < NT) {
            const int col = 16 * t + rl;
            const float bias = bp[col];
#pragma unroll
            for (int m = 0; m < 4; ++m)
#pragma unroll
                for (int v = 0; v < 4; ++v) {
                    const int row = 16 * m + 4 * kg + v;
                    if (row < S) xs[row * LDX + col] += acc[m][j][v] + bias;
                }
        }
    }
    __syncthreads();
    // LayerNorm: 4 threads per row, two-pass mean / biased variance; x' and h' written as float4
    {
        constexpr int LP = D / 16;     // float4 pieces per thread
        const int row = threadIdx.x >> 2, q = threadIdx.x & 3;
        float4 xv[LP];
        float s1 = 0.0f;
#pragma unroll
        for (int i = 0; i < LP; ++i) {
            xv[i] = *(const float4*)&xs[row * LDX + 4 * (q + 4 * i)];
            s1 += (xv[i].x + xv[i].y) + (xv[i].z + xv[i].w);
        }
        s1 += __shfl_xor(s1, 1);
        s1 += __shfl_xor(s1, 2);
        const float mean = s1 / (float)D;
        float s2 = 0.0f;
#pragma unroll
        for (int i = 0; i < LP; ++i) {
            const float a = xv[i].x - mean, c = xv[i].y - mean, e = xv[i].z - mean, f = xv[i].w - mean;
            s2 += (a * a + c * c) + (e * e + f * f);
        }
        s2 += __shfl_xor(s2, 1);
        s2 += __shfl_xor(s2, 2);
        const float rstd = rsqrtf(s2 / (float)D + eps);
        if (row < S) {
            const size_t o = ((size_t)b * S + row) * D;
            if (stats_out != nullptr && q == 0) stats_out[(size_t)b * S + row] = make_float2(mean, rstd);
            const bool wh = h_out != nullptr;   // (uniform)
#pragma unroll
            for (int i = 0; i < LP; ++i) {
                const int c0 = 4 * (q + 4 * i);
                *(float4*)((x_out != nullptr ? x_out : x_io) + o + c0) = xv[i];
                if (wh) {
                    const float4 g = *(const float4*)(gamma + c0), be = *(const float4*)(beta + c0);
                    *(float4*)(h_out + o + c0) = make_float4((xv[i].x - mean) * rstd * g.x + be.x, (xv[i].y - mean) * rstd * g.y + be.y,
                                                             (xv[i].z - mean) * rstd * g.z + be.z, (xv[i].w - mean) * rstd * g.w + be.w);
                }
            }
        }
    }
}


// ---------------------------------------------------------------------------
// The heads at the reference's precision (round 5): PerClassAttentionMLPHead
// (az_doko.py:28-56), f32 activations, bf16x3 MFMA products (as mlp_ln_f32x3_kernel).
// 8 f32 values -> the hi / lo fragments of one k-step
__device__ __forceinline__ void split_f32x8(const float* p, bool ok, bf16x8_t& hi, bf16x8_t& lo) {
    float v[8];
    if (ok) {
        const float4 a = *(const float4*)p, c = *(const float4*)(p + 4);
        v[0] = a.x; v[1] = a.y; v[2] = a.z; v[3] = a.w; v[4] = c.x; v[5] = c.y; v[6] = c.z; v[7] = c.w;
    } else {
#pragma unroll
        for (int j = 0; j < 8; ++j) v[j] = 0.0f;
    }
    split_bf16x8(v, hi, lo);
}

// The pooling and each class's LayerNorm, one 256-thread workgroup per sample (the f32 form of
// class_pool_ln_kernel):
//   scores^T = X Q^T * scale   (the token in the registers, the class on the lane)
//   P = softmax over the 62 tokens (f32)
//   A = P X                    (X^T fragments gathered from the f32 rows in LDS)
//   out[c][b][:] = LN(A[c]) * w[c] + b[c]   (class-major [C, B, d]: the class MLP's operand)
// LDS: the sample's x rows (f32, rows padded to d + 8: the two half-waves of a gather 4 rows apart
// land on disjoint bank halves), then the pooled rows.
template <int D>
__global__ void __launch_bounds__(256, 2) class_pool_ln_f32x3_kernel(const float* __restrict__ xin, uint32_t batch,
                                                                     const float* __restrict__ queries, uint32_t classes,
                                                                     float scale, const float* __restrict__ lnw,
                                                                     const float* __restrict__ lnb, float eps,
                                                                     float* __restrict__ out) {
    constexpr int S = 62, LDX = D + 8, KD = D / 16, DT = D / 32, LP = D / 32;
    static_assert(D % 32 == 0, "d: a multiple of 32");
    __shared__ __attribute__((aligned(16))) float xs[64 * LDX];
    const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63, r = lane & 31, hh = lane >> 5;
    const uint32_t b = blockIdx.x;
    const int C = (int)classes;
    const float* xg = xin + (size_t)b * S * D;
    {
        // every load issued before the first LDS store (a load -> store loop waited a memory round
        // trip per iteration); rows 62, 63 zero
        constexpr int N4 = 64 * (D / 4) / 256;
        static_assert(64 * (D / 4) % 256 == 0, "whole float4s per thread");
        float4 v[N4];
#pragma unroll
        for (int i = 0; i < N4; ++i) {
            const int p = threadIdx.x + 256 * i, t = p / (D / 4), d0 = 4 * (p - t * (D / 4));
            v[i] = *(const float4*)(xg + (size_t)(t < S ? t : S - 1) * D + d0);
        }
#pragma unroll
        for (int i = 0; i < N4; ++i) {
            const int p = threadIdx.x + 256 * i, t = p / (D / 4), d0 = 4 * (p - t * (D / 4));
            *(float4*)&xs[t * LDX + d0] = t < S ? v[i] : make_float4(0.f, 0.f, 0.f, 0.f);
        }
    }
    __syncthreads();
    const int CT = C > 32 ? 2 : 1, WPC = 4 / CT;       // class tiles, waves per class tile
    const int ct = wave % CT, part = wave / CT;
    const int cls = 32 * ct + r;
    const float* qrow = queries + (size_t)(cls < C ? cls : 0) * D + 8 * hh;
    f32x16_t sc[2];
    sc[0] = f32x16_t{0};
    sc[1] = f32x16_t{0};
    // the query pieces one k-step ahead (loaded in the step that used them, each step waited an
    // L2 round trip)
    float4 qa = *(const float4*)qrow, qb = *(const float4*)(qrow + 4);
#pragma unroll
    for (int ks = 0; ks < KD; ++ks) {
        float qv[8] = {qa.x, qa.y, qa.z, qa.w, qb.x, qb.y, qb.z, qb.w};
        if (ks + 1 < KD) {
            qa = *(const float4*)(qrow + 16 * (ks + 1));
            qb = *(const float4*)(qrow + 16 * (ks + 1) + 4);
        }
#pragma unroll
        for (int j = 0; j < 8; ++j) qv[j] = cls < C ? qv[j] : 0.0f;
        bf16x8_t qh, ql;
        split_bf16x8(qv, qh, ql);
#pragma unroll
        for (int mt = 0; mt < 2; ++mt) {
            bf16x8_t xh, xl;
            split_f32x8(&xs[(32 * mt + r) * LDX + 16 * ks + 8 * hh], true, xh, xl);
            sc[mt] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(xl, qh, sc[mt], 0, 0, 0);
            sc[mt] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(xh, ql, sc[mt], 0, 0, 0);
            sc[mt] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(xh, qh, sc[mt], 0, 0, 0);
        }
    }
    // softmax over the tokens t < 62 of the lane's class (torch: exp(v - max) / sum)
    bf16x8_t pfh[4], pfl[4];
    {
        float mx = -INFINITY;
#pragma unroll
        for (int mt = 0; mt < 2; ++mt)
#pragma unroll
            for (int g = 0; g < 16; ++g) {
                const int t = 32 * mt + (g & 3) + 8 * (g >> 2) + 4 * hh;
                sc[mt][g] *= scale;
                if (t < S) mx = fmaxf(mx, sc[mt][g]);
            }
        mx = fmaxf(mx, __shfl_xor(mx, 32));
        float l = 0.0f;
#pragma unroll
        for (int mt = 0; mt < 2; ++mt)
#pragma unroll
            for (int g = 0; g < 16; ++g) {
                const int t = 32 * mt + (g & 3) + 8 * (g >> 2) + 4 * hh;
                const float e = t < S ? expf(sc[mt][g] - mx) : 0.0f;
                sc[mt][g] = e;
                l += e;
            }
        l += __shfl_xor(l, 32);
#pragma unroll
        for (int q = 0; q < 4; ++q) {
            float v[8];
#pragma unroll
            for (int j = 0; j < 8; ++j) v[j] = sc[q >> 1][8 * (q & 1) + j] / l;
            split_bf16x8(v, pfh[q], pfl[q]);
        }
    }
    // A = P X for the wave's d tiles t = part, part + WPC, ...: the B fragment of k-step q holds
    // the tokens 16 q + 4 hh + {0..3, 8..11} of dimension 32 t + r (P's register order)
    constexpr int MAXT = (DT + 1) / 2;
    f32x16_t acc[MAXT];
#pragma unroll
    for (int i = 0; i < MAXT; ++i) {
        const int t = part + WPC * i;
        acc[i] = f32x16_t{0};
        if (t < DT) {
#pragma unroll
            for (int q = 0; q < 4; ++q) {
                const int t0 = 16 * q + 4 * hh;
                const float* col = &xs[t0 * LDX + 32 * t + r];
                float v[8];
#pragma unroll
                for (int j = 0; j < 4; ++j) {
                    v[j] = col[j * LDX];
                    v[4 + j] = col[(8 + j) * LDX];
                }
                bf16x8_t fh, fl;
                split_bf16x8(v, fh, fl);
                acc[i] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(pfl[q], fh, acc[i], 0, 0, 0);
                acc[i] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(pfh[q], fl, acc[i], 0, 0, 0);
                acc[i] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(pfh[q], fh, acc[i], 0, 0, 0);
            }
        }
    }
    __syncthreads();   // every wave's reads of the x rows done: the pooled rows replace them
#pragma unroll
    for (int i = 0; i < MAXT; ++i) {
        const int t = part + WPC * i;
        if (t < DT) {
#pragma unroll
            for (int g = 0; g < 16; ++g) {
                const int c = 32 * ct + (g & 3) + 8 * (g >> 2) + 4 * hh;
                if (c < C) xs[c * LDX + 32 * t + r] = acc[i][g];
            }
        }
    }
    __syncthreads();
    // LayerNorm of each class row (F.layer_norm without affine, then * w[c] + b[c]): 4 threads per row
    {
        const int c = threadIdx.x >> 2, q = threadIdx.x & 3;
        float4 xv[2 * LP];
        float s1 = 0.0f;
#pragma unroll
        for (int i = 0; i < 2 * LP; ++i) {
            xv[i] = *(const float4*)&xs[c * LDX + 4 * (q + 4 * i)];
            s1 += (xv[i].x + xv[i].y) + (xv[i].z + xv[i].w);
        }
        s1 += __shfl_xor(s1, 1);
        s1 += __shfl_xor(s1, 2);
        const float mean = s1 / (float)D;
        float s2 = 0.0f;
#pragma unroll
        for (int i = 0; i < 2 * LP; ++i) {
            const float a = xv[i].x - mean, e = xv[i].y - mean, f = xv[i].z - mean, g = xv[i].w - mean;
            s2 += (a * a + e * e) + (f * f + g * g);
        }
        s2 += __shfl_xor(s2, 1);
        s2 += __shfl_xor(s2, 2);
        const float rstd = rsqrtf(s2 / (float)D + eps);
        if (c < C) {
            const size_t o = ((size_t)c * batch + b) * D;
#pragma unroll
            for (int i = 0; i < 2 * LP; ++i) {
                const int c0 = 4 * (q + 4 * i);
                const float4 gv = *(const float4*)(lnw + (size_t)c * D + c0), bv = *(const float4*)(lnb + (size_t)c * D + c0);
                *(float4*)(out + o + c0) = make_float4((xv[i].x - mean) * rstd * gv.x + bv.x, (xv[i].y - mean) * rstd * gv.y + bv.y,
                                                       (xv[i].z - mean) * rstd * gv.z + bv.z, (xv[i].w - mean) * rstd * gv.w + bv.w);
            }
        }
    }
}

// The same pooling + class LayerNorm for a few classes (C <= 8: the AlphaZero value head's 4), in
// f32 FMAs: a 32-class MFMA tile would be 7/8 padding there, and its four waves each recomputed the
// whole score tile.  One 256-thread workgroup per sample:
//   x rows -> LDS (f32, rows padded to d + 1 words: the score phase reads a column, one row per
//   lane, on distinct banks), the queries -> LDS;
//   scores: lane t of wave w holds token t of class w (+ 4), q . x_t in k order, * scale
//   (torch: einsum, then * scale); softmax over the wave's 62 tokens (max, exp, sum, divide);
//   attended[c][k] = sum over t of p[c][t] x[t][k] (t ascending), one (c, k) per lane;
//   LayerNorm of each class row (two-pass, biased variance) * w[c] + b[c], class-major output.
template <int D>
__global__ void __launch_bounds__(256) class_pool_small_ln_f32_kernel(const float* __restrict__ xin, uint32_t batch,
                                                                      const float* __restrict__ queries, uint32_t classes,
                                                                      float scale, const float* __restrict__ lnw,
                                                                      const float* __restrict__ lnb, float eps,
                                                                      float* __restrict__ out) {
    constexpr int S = 62, LDX = D + 1, CM = 8;
    static_assert(D % 4 == 0, "whole float4 pieces per row");
    __shared__ float xs[S * LDX];
    __shared__ float qs[CM * D];      // the queries, then the attended rows
    __shared__ float ps[CM * 64];     // softmax weights [c][t]
    const int tid = threadIdx.x, wave = tid >> 6, t = tid & 63, C = (int)classes;
    const uint32_t b = blockIdx.x;
    const float4* xg = (const float4*)(xin + (size_t)b * S * D);
    {
        constexpr int N4 = S * D / 4, PER = (N4 + 255) / 256;
        float4 v[PER];
#pragma unroll
        for (int i = 0; i < PER; ++i) {
            const int p = tid + 256 * i;
            v[i] = xg[p < N4 ? p : N4 - 1];   // (every load issued before the stores)
        }
#pragma unroll
        for (int i = 0; i < PER; ++i) {
            const int p = tid + 256 * i;
            if (p < N4) {
                const int row = (4 * p) / D, k = 4 * p - row * D;
                float* dst = &xs[row * LDX + k];
                dst[0] = v[i].x; dst[1] = v[i].y; dst[2] = v[i].z; dst[3] = v[i].w;
            }
        }
        for (int p = tid; p < C * D; p += 256) qs[p] = queries[p];
    }
    __syncthreads();
    for (int c = wave; c < C; c += 4) {
        float sc = 0.0f;
        if (t < S) {
            const float* xr = &xs[t * LDX];
            const float* qr = &qs[c * D];
#pragma unroll 8
            for (int k = 0; k < D; ++k) sc = fmaf(qr[k], xr[k], sc);
        }
        sc *= scale;
        float m = t < S ? sc : -INFINITY;
#pragma unroll
        for (int o = 32; o >= 1; o >>= 1) m = fmaxf(m, __shfl_xor(m, o));
        const float e = t < S ? expf(sc - m) : 0.0f;
        float l = e;
#pragma unroll
        for (int o = 32; o >= 1; o >>= 1) l += __shfl_xor(l, o);
        ps[c * 64 + t] = e / l;
    }
    __syncthreads();
    // (the queries are read: their LDS takes the attended rows)
    float av[(CM * D + 255) / 256];
#pragma unroll
    for (int i = 0; i < (CM * D + 255) / 256; ++i) {
        const int o = tid + 256 * i;
        av[i] = 0.0f;
        if (o < C * D) {
            const int c = o / D, k = o - c * D;
            float a = 0.0f;
            for (int s2 = 0; s2 < S; ++s2) a = fmaf(ps[c * 64 + s2], xs[s2 * LDX + k], a);
            av[i] = a;
        }
    }
    __syncthreads();
#pragma unroll
    for (int i = 0; i < (CM * D + 255) / 256; ++i) {
        const int o = tid + 256 * i;
        if (o < C * D) qs[o] = av[i];
    }
    __syncthreads();
    constexpr int KP = (D + 63) / 64;   // a row's values per lane
    for (int c = wave; c < C; c += 4) {
        float v[KP];
        float s1 = 0.0f;
#pragma unroll
        for (int j = 0; j < KP; ++j) {
            const int k = t + 64 * j;
            v[j] = k < D ? qs[c * D + k] : 0.0f;
            s1 += v[j];
        }
#pragma unroll
        for (int o = 32; o >= 1; o >>= 1) s1 += __shfl_xor(s1, o);
        const float mean = s1 / (float)D;
        float s2 = 0.0f;
#pragma unroll
        for (int j = 0; j < KP; ++j) {
            const int k = t + 64 * j;
            const float dv = k < D ? v[j] - mean : 0.0f;
            s2 += dv * dv;
        }
#pragma unroll
        for (int o = 32; o >= 1; o >>= 1) s2 += __shfl_xor(s2, o);
        const float rstd = rsqrtf(s2 / (float)D + eps);
        float* orow = out + ((size_t)c * batch + b) * D;
#pragma unroll
        for (int j = 0; j < KP; ++j) {
            const int k = t + 64 * j;
            if (k < D) orow[k] = (v[j] - mean) * rstd * lnw[(size_t)c * D + k] + lnb[(size_t)c * D + k];
        }
    }
}

// Each class's MLP, out[b][c] = w2[c] . GELU(W1[c] a[c][b] + b1[c]) + b2[c] (the exact erf GELU
// of nn.GELU), grid (row blocks of 128, classes), 4 waves x 32 rows: the row's pooled vector split
// in registers, W1[c] hi / lo fragments straight from L2 one k-step ahead (a class's W1 is 2 d^2
// bf16 pieces, read by every workgroup of the class), the hidden units reduced into the output
// without leaving the registers.  Replaces the class-batched GEMM, the bias + GELU pass and the
// w2 product + sum over d of ClassHead.forward.
template <int D>
__global__ void __launch_bounds__(256, 2) class_mlp_f32x3_kernel(const float* __restrict__ ac, uint32_t batch, uint32_t classes,
                                                                 const uint16_t* __restrict__ w1h, const uint16_t* __restrict__ w1l,
                                                                 const float* __restrict__ b1, const float* __restrict__ w2,
                                                                 const float* __restrict__ b2, float* __restrict__ out) {
    constexpr int KS = D / 16, OT = D / 32;
    const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63, r = lane & 31, hh = lane >> 5;
    const uint32_t c = blockIdx.y;
    const uint32_t row = blockIdx.x * 128u + (uint32_t)wave * 32u + (uint32_t)r;
    const bool ok = row < batch;
    bf16x8_t afh[KS], afl[KS];
    const float* ar = ac + ((size_t)c * batch + (ok ? row : 0u)) * D + 8 * hh;
    // (unconditional loads -- rows past the batch read row 0 and are never stored: a load under
    // the row condition waited for each load in turn)
#pragma unroll
    for (int kk = 0; kk < KS; ++kk) split_f32x8(ar + 16 * kk, true, afh[kk], afl[kk]);
    const uint16_t* wh = w1h + (size_t)c * D * D + (size_t)r * D + 8 * hh;
    const uint16_t* wl = w1l + (size_t)c * D * D + (size_t)r * D + 8 * hh;
    const float* b1c = b1 + (size_t)c * D;
    const float* w2c = w2 + (size_t)c * D;
    float part = 0.0f;
    // W fragments one k-step ahead, across the output tiles too
    bf16x8_t nh = load_frag8(wh, true), nl = load_frag8(wl, true);
#pragma unroll 1
    for (int ot = 0; ot < OT; ++ot) {
        f32x16_t acc = f32x16_t{0};
#pragma unroll
        for (int ks = 0; ks < KS; ++ks) {
            const bf16x8_t ah = nh, al = nl;
            if (ks + 1 < KS || ot + 1 < OT) {
                const int o2 = ks + 1 < KS ? 32 * ot * D + 16 * (ks + 1) : 32 * (ot + 1) * D;
                nh = load_frag8(wh + o2, true);
                nl = load_frag8(wl + o2, true);
            }
            __builtin_amdgcn_sched_barrier(0);   // (the next step's loads stay ahead of this step's MFMAs)
            acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(al, afh[ks], acc, 0, 0, 0);
            acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(ah, afl[ks], acc, 0, 0, 0);
            acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(ah, afh[ks], acc, 0, 0, 0);
            __builtin_amdgcn_sched_barrier(0);
        }
#pragma unroll
        for (int g = 0; g < 16; ++g) {
            const int i = 32 * ot + (g & 3) + 8 * (g >> 2) + 4 * hh;
            const float v = acc[g] + b1c[i];
            part += 0.5f * v * (1.0f + erff(v * 0.70710678118654752f)) * w2c[i];
        }
    }
    part += __shfl_xor(part, 32);
    if (ok && hh == 0) out[(size_t)row * classes + c] = part + b2[c];
}

// The bf16 network's class MLPs in one launch (the bf16 form of class_mlp_f32x3_kernel):
// out[b][c] = bf16(w2[c] . GELU(W1[c] a[c][b] + b1[c]) + b2[c]), bf16 operands, one product per
// k-step, f32 accumulation, the exact erf GELU in f32 -- replacing the class-batched bmm, the bias
// and GELU passes and the w2 product + sum of ClassHead.forward (each rounding to bf16).
template <int D>
__global__ void __launch_bounds__(256, 2) class_mlp_bf16_kernel(const uint16_t* __restrict__ ac, uint32_t batch, uint32_t classes,
                                                                const uint16_t* __restrict__ w1, const uint16_t* __restrict__ b1,
                                                                const uint16_t* __restrict__ w2, const uint16_t* __restrict__ b2,
                                                                uint16_t* __restrict__ out) {
    constexpr int KS = D / 16, OT = D / 32;
    const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63, r = lane & 31, hh = lane >> 5;
    const uint32_t c = blockIdx.y;
    const uint32_t row = blockIdx.x * 128u + (uint32_t)wave * 32u + (uint32_t)r;
    const bool ok = row < batch;
    // (unconditional loads: rows past the batch read row 0 and are never stored)
    bf16x8_t af[KS];
    const uint16_t* ar = ac + ((size_t)c * batch + (ok ? row : 0u)) * D + 8 * hh;
#pragma unroll
    for (int kk = 0; kk < KS; ++kk) af[kk] = *(const bf16x8_t*)(ar + 16 * kk);
    const uint16_t* wr = w1 + (size_t)c * D * D + (size_t)r * D + 8 * hh;
    const uint16_t* b1c = b1 + (size_t)c * D;
    const uint16_t* w2c = w2 + (size_t)c * D;
    float part = 0.0f;
    bf16x8_t nw = *(const bf16x8_t*)wr;
#pragma unroll 1
    for (int ot = 0; ot < OT; ++ot) {
        f32x16_t acc = f32x16_t{0};
#pragma unroll
        for (int ks = 0; ks < KS; ++ks) {
            const bf16x8_t a = nw;
            if (ks + 1 < KS || ot + 1 < OT) {
                const int o2 = ks + 1 < KS ? 32 * ot * D + 16 * (ks + 1) : 32 * (ot + 1) * D;
                nw = *(const bf16x8_t*)(wr + o2);
            }
            __builtin_amdgcn_sched_barrier(0);
            acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, af[ks], acc, 0, 0, 0);
            __builtin_amdgcn_sched_barrier(0);
        }
#pragma unroll
        for (int g = 0; g < 16; ++g) {
            const int i = 32 * ot + (g & 3) + 8 * (g >> 2) + 4 * hh;
            const float v = acc[g] + bf2f(b1c[i]);
            part += 0.5f * v * (1.0f + erff(v * 0.70710678118654752f)) * bf2f(w2c[i]);
        }
    }
    part += __shfl_xor(part, 32);
    if (ok && hh == 0) out[(size_t)row * classes + c] = f2bf(part + bf2f(b2[c]));
}

}  // namespace net
}  // namespace dk
