// Row kernels of the AlphaZero network's forward pass (az_network.py), bf16 in
// HBM, f32 arithmetic.  The activations are [B*62, d] rows with d = 160: torch's
// generic LayerNorm kernel spends ~0.5 ms per call on the C5 batch (8192 x 62
// rows) where the bytes take ~65 us, and the residual adds and the six embedding
// gathers are separate passes.  Here:
//   embed_ln   : x = sum of the six token embeddings; h = LN(x)         (one pass)
//   add_ln     : x += delta; h = LN(x)                                  (one pass)
//   ln         : h = LN(x)
// One row per 32-lane half-wave: lane l holds bf16 pairs l, l+32, ..., so every
// load/store instruction of a half-wave covers up to 128 contiguous bytes.  Mean and variance: f32 two-pass over the registers, shuffle
// reductions inside the half-wave.  LayerNorm as torch: (x - mean) *
// rsqrt(var + eps) * gamma + beta, biased variance.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <type_traits>

namespace dk {
namespace net {

constexpr int LN_MAX_PER_LANE = 8;    // bf16 pairs per lane: d <= 512

__device__ __forceinline__ float bf2f(uint16_t v) { return __uint_as_float((uint32_t)v << 16); }
// f32 -> bf16, round to nearest even (torch's conversion): gfx950's v_cvt_pk_bf16_f32, one
// instruction for two values (the integer form took six per value); NaN stays NaN
__device__ __forceinline__ uint32_t pack_bf16x2(float lo, float hi) {
    typedef __bf16 bf16x2_t __attribute__((ext_vector_type(2)));
    union { bf16x2_t v; uint32_t u; } r;
    r.v = bf16x2_t{(__bf16)lo, (__bf16)hi};
    return r.u;
}
__device__ __forceinline__ uint16_t f2bf(float f) {
    union { __bf16 b; uint16_t u; } r;
    r.b = (__bf16)f;
    return r.u;
}

__device__ __forceinline__ float half_wave_sum(float v) {
#pragma unroll
    for (int o = 16; o >= 1; o >>= 1) v += __shfl_xor(v, o, 32);
    return v;
}

// A row as bf16 pairs: lane l holds pairs l, l + 32, ... (PER pairs, the last
// ones masked when d/2 is not a multiple of 32), so every load / store of a
// half-wave moves up to 128 contiguous bytes.
template <int PER>
__device__ __forceinline__ void ln_row(const float (&x)[2 * PER], int d, int lane, const uint32_t* gamma2,
                                       const uint32_t* beta2, float eps, uint32_t* out2) {
    const int np = d / 2;
    float s = 0.0f;
#pragma unroll
    for (int k = 0; k < PER; ++k)
        if (lane + 32 * k < np) s += x[2 * k] + x[2 * k + 1];
    const float mean = half_wave_sum(s) / (float)d;
    float q = 0.0f;
#pragma unroll
    for (int k = 0; k < PER; ++k)
        if (lane + 32 * k < np) {
            const float c0 = x[2 * k] - mean, c1 = x[2 * k + 1] - mean;
            q += c0 * c0 + c1 * c1;
        }
    const float rstd = rsqrtf(half_wave_sum(q) / (float)d + eps);
#pragma unroll
    for (int k = 0; k < PER; ++k) {
        const int j = lane + 32 * k;
        if (j < np) {
            const uint32_t g = gamma2[j], b = beta2[j];
            const float y0 = (x[2 * k] - mean) * rstd * bf2f((uint16_t)g) + bf2f((uint16_t)b);
            const float y1 = (x[2 * k + 1] - mean) * rstd * bf2f((uint16_t)(g >> 16)) + bf2f((uint16_t)(b >> 16));
            out2[j] = pack_bf16x2(y0, y1);
        }
    }
}

// tokens [B, 311] int32 (encode_state_pi); tables: object, position, player, subposition, team, phase
template <int PER>
__global__ void embed_ln_kernel(const int32_t* __restrict__ tokens, uint32_t B, int d, const uint16_t* __restrict__ e0,
                                const uint16_t* __restrict__ e1, const uint16_t* __restrict__ e2,
                                const uint16_t* __restrict__ e3, const uint16_t* __restrict__ e4,
                                const uint16_t* __restrict__ e5, const uint16_t* gamma, const uint16_t* beta, float eps,
                                uint16_t* __restrict__ x_out, uint16_t* __restrict__ h_out) {
    const uint32_t row = blockIdx.x * (blockDim.x / 32) + threadIdx.x / 32;
    const int lane = threadIdx.x & 31, np = d / 2;
    if (row >= B * 62u) return;
    const uint32_t b = row / 62u, s = row % 62u;
    const int32_t* t = tokens + (size_t)b * 311;
    const uint32_t* rows[6] = {(const uint32_t*)(e0 + (size_t)t[s] * d), (const uint32_t*)(e1 + (size_t)t[62 + s] * d),
                               (const uint32_t*)(e2 + (size_t)t[124 + s] * d), (const uint32_t*)(e3 + (size_t)t[186 + s] * d),
                               (const uint32_t*)(e4 + (size_t)t[248 + s] * d), (const uint32_t*)(e5 + (size_t)t[310] * d)};
    uint32_t* xo = (uint32_t*)(x_out + (size_t)row * d);
    float x[2 * PER];
#pragma unroll
    for (int k = 0; k < PER; ++k) {
        const int j = lane + 32 * k;
        x[2 * k] = x[2 * k + 1] = 0.0f;
        if (j < np) {
            // torch sums the six bf16 embeddings left to right with a bf16 rounding after each add
            uint32_t v = rows[0][j];
            float a0 = bf2f((uint16_t)v), a1 = bf2f((uint16_t)(v >> 16));
#pragma unroll
            for (int e = 1; e < 6; ++e) {
                v = rows[e][j];
                a0 = bf2f(f2bf(a0 + bf2f((uint16_t)v)));
                a1 = bf2f(f2bf(a1 + bf2f((uint16_t)(v >> 16))));
            }
            x[2 * k] = a0; x[2 * k + 1] = a1;
            xo[j] = pack_bf16x2(a0, a1);
        }
    }
    ln_row<PER>(x, d, lane, (const uint32_t*)gamma, (const uint32_t*)beta, eps, (uint32_t*)(h_out + (size_t)row * d));
}

// x += delta (bf16 add as torch rounds it); h = LN(x).  A half-wave handles ADD_LN_ROWS
// consecutive rows and issues all of their loads before any arithmetic, so each wave
// keeps ADD_LN_ROWS times more bytes in flight (and the grid has that many fewer waves).
constexpr int ADD_LN_ROWS = 4;
template <int PER>
__global__ void add_ln_kernel(uint16_t* __restrict__ x_io, const uint16_t* __restrict__ delta, uint32_t rows, int d,
                              const uint16_t* gamma, const uint16_t* beta, float eps, uint16_t* __restrict__ h_out) {
    const uint32_t row0 = (blockIdx.x * (blockDim.x / 32) + threadIdx.x / 32) * ADD_LN_ROWS;
    const int lane = threadIdx.x & 31, np = d / 2;
    if (row0 >= rows) return;
    uint32_t xv[ADD_LN_ROWS][PER], dv[ADD_LN_ROWS][PER];
#pragma unroll
    for (int q = 0; q < ADD_LN_ROWS; ++q)
#pragma unroll
        for (int k = 0; k < PER; ++k) {
            const int j = lane + 32 * k;
            const bool ok = row0 + q < rows && j < np;
            const size_t at = (size_t)(row0 + q) * (d / 2) + j;
            xv[q][k] = ok ? ((const uint32_t*)x_io)[at] : 0u;
            dv[q][k] = (ok && delta) ? ((const uint32_t*)delta)[at] : 0u;
        }
#pragma unroll
    for (int q = 0; q < ADD_LN_ROWS; ++q) {
        if (row0 + q >= rows) break;
        uint32_t* xr = (uint32_t*)(x_io + (size_t)(row0 + q) * d);
        float x[2 * PER];
#pragma unroll
        for (int k = 0; k < PER; ++k) {
            const int j = lane + 32 * k;
            uint32_t v = xv[q][k];
            if (delta) {
                const uint32_t e = dv[q][k];
                v = (uint32_t)f2bf(bf2f((uint16_t)v) + bf2f((uint16_t)e)) |
                    ((uint32_t)f2bf(bf2f((uint16_t)(v >> 16)) + bf2f((uint16_t)(e >> 16))) << 16);
                if (j < np) xr[j] = v;
            }
            x[2 * k] = bf2f((uint16_t)v); x[2 * k + 1] = bf2f((uint16_t)(v >> 16));
        }
        ln_row<PER>(x, d, lane, (const uint32_t*)gamma, (const uint32_t*)beta, eps,
                    (uint32_t*)(h_out + (size_t)(row0 + q) * d));
    }
}

// ---------------------------------------------------------------------------
// Self-attention core of a block for the networks' shape: 62 tokens, H heads of
// dimension HD (AlphaZero: 4 x 40, d = 160; IMPI: 4 x 64, d = 256), reading q, k, v
// straight out of the fused qkv projection [B*62, 3d] and writing the heads' outputs
// into [B*62, d] (no permute / transpose copies).  One wave per (sample, head), bf16
// MFMA v_mfma_f32_32x32x16_bf16 (tokens padded to 64, head dimension to 16 KS):
//   X  = K Q^T   (2 x 2 tiles of 32 x 32, KS k-steps over the head dimension):
//        X[t][s] has the query s on the lane, the keys t in the registers;
//   P  = softmax over t per column s (registers + one cross-half shuffle),
//        normalised, packed to bf16 in place (the accumulator-as-operand idiom:
//        registers 8q..8q+7 of a tile are k-step q, element j of lane half h is
//        key 16q + 8(j>>2) + 4h + (j&3));
//   O  = P V     (P^T fragments as the A operand, V^T staged in LDS as [e][t] so
//        a lane's 8 keys are two 8-byte reads; 2 x 2 tiles, 4 k-steps):
//        O[s][e] has e on the lane: each register is one 64-byte row segment.
typedef __bf16 bf16x8_t __attribute__((ext_vector_type(8)));
typedef float f32x16_t __attribute__((ext_vector_type(16)));

__device__ __forceinline__ bf16x8_t load_frag8(const uint16_t* p, bool ok) {
    union { uint4 u; bf16x8_t v; } r;
    r.u = ok ? *(const uint4*)p : make_uint4(0u, 0u, 0u, 0u);
    return r.v;
}

template <int HD, class Put>
__device__ __forceinline__ void attn62_core(const bf16x8_t (&qf)[2][(HD + 15) / 16], const bf16x8_t (&kf)[2][(HD + 15) / 16],
                                            const uint16_t* vt, float scale, bool valid, Put put);

// One (sample, head) of the attention core, the body shared by attn62_kernel and attn_ln_kernel:
// `base` = the sample's qkv rows, `vt` the wave's LDS V^T tile (HD x (64 + 4) bf16), put(s, e, v) receives output
// element (token s < 62, head dim e < HD).  Every wave of the workgroup must call it (barrier).
template <int HD, int H, class Put>
__device__ __forceinline__ void attn62_head(const uint16_t* __restrict__ base, uint32_t hd, bool valid, uint16_t* vt,
                                            float scale, Put put) {
    static_assert(HD % 8 == 0 && HD <= 64, "head dimension: a multiple of 8, at most 64");
    constexpr int S = 62, D = HD * H, LDT = 64 + 4;   // LDS row stride (keys) in bf16
    constexpr int PC = HD / 8;                        // 16-byte pieces per key row of V
    constexpr int KS = (HD + 15) / 16;                // k-steps over the head dimension
    const int lane = threadIdx.x & 63, r = lane & 31, h = lane >> 5;
    // V^T into LDS as [e][t]: the 62 x HD tile is read as 62 * HD / 8 16-byte pieces (8
    // dims of one key each, HD / 8 per lane) and scattered transposed; zero padding for
    // t >= 62 (lanes of the second output tile with e >= HD read row HD - 1 and put nothing)
    {
#pragma unroll
        for (int i = 0; i < PC; ++i) {
            const int v = lane + 64 * i;          // piece v: key v / PC, dims 8 (v % PC) .. +8
            const int t = v / PC, e0 = 8 * (v % PC);
            const bool ok = valid && v < S * PC;
            union { uint4 u; uint16_t s[8]; } pc;
            pc.u = ok ? *(const uint4*)(base + (size_t)t * (3 * D) + 2 * D + hd * HD + e0) : make_uint4(0u, 0u, 0u, 0u);
#pragma unroll
            for (int m = 0; m < 8; ++m) vt[(e0 + m) * LDT + t] = pc.s[m];
        }
    }
    // Q and K fragments: tile i covers tokens 32i + r, k-step kk covers dims 16kk + 8h + j
    bf16x8_t qf[2][KS], kf[2][KS];
#pragma unroll
    for (int i = 0; i < 2; ++i) {
        const int tok = 32 * i + r;
#pragma unroll
        for (int kk = 0; kk < KS; ++kk) {
            const int e0 = 16 * kk + 8 * h;
            const bool ok = valid && tok < S && e0 < HD;
            const uint16_t* row = base + (size_t)(ok ? tok : 0) * (3 * D) + hd * HD + (ok ? e0 : 0);
            qf[i][kk] = load_frag8(row, ok);
            kf[i][kk] = load_frag8(row + D, ok);
        }
    }
    attn62_core<HD>(qf, kf, vt, scale, valid, put);
}

// The attention core from the Q / K fragments on: qf[i][kk], kf[i][kk] = tokens 32 i + r,
// k-step kk over the head dimension (any order of the dimensions, the same in both);
// vt = the wave's V^T tile [e][t] in LDS, written by the caller.  Every wave of the
// workgroup must call it (barrier).
template <int HD, class Put>
__device__ __forceinline__ void attn62_core(const bf16x8_t (&qf)[2][(HD + 15) / 16], const bf16x8_t (&kf)[2][(HD + 15) / 16],
                                            const uint16_t* vt, float scale, bool valid, Put put) {
    constexpr int S = 62, LDT = 64 + 4, KS = (HD + 15) / 16;
    const int lane = threadIdx.x & 63, r = lane & 31, h = lane >> 5;
    // X[ti][si] = K_ti Q_si^T
    f32x16_t x[2][2];
#pragma unroll
    for (int ti = 0; ti < 2; ++ti)
#pragma unroll
        for (int si = 0; si < 2; ++si) {
            f32x16_t acc = {0};
#pragma unroll
            for (int kk = 0; kk < KS; ++kk) acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(kf[ti][kk], qf[si][kk], acc, 0, 0, 0);
            x[ti][si] = acc;
        }
    // softmax over the keys t of every query column s; P packed to bf16 fragments
    bf16x8_t pf[2][4];
#pragma unroll
    for (int si = 0; si < 2; ++si) {
        float m = -INFINITY;
#pragma unroll
        for (int ti = 0; ti < 2; ++ti)
#pragma unroll
            for (int g = 0; g < 16; ++g) {
                const int t = 32 * ti + (g & 3) + 8 * (g >> 2) + 4 * h;
                if (t < S) m = fmaxf(m, x[ti][si][g]);
            }
        m = fmaxf(m, __shfl_xor(m, 32));
        float l = 0.0f;
#pragma unroll
        for (int ti = 0; ti < 2; ++ti)
#pragma unroll
            for (int g = 0; g < 16; ++g) {
                const int t = 32 * ti + (g & 3) + 8 * (g >> 2) + 4 * h;
                const float pv = t < S ? __expf((x[ti][si][g] - m) * scale) : 0.0f;
                x[ti][si][g] = pv;
                l += pv;
            }
        l += __shfl_xor(l, 32);
        const float inv = 1.0f / l;
#pragma unroll
        for (int q = 0; q < 4; ++q) {
            union { uint32_t u[4]; bf16x8_t v; } pk;
#pragma unroll
            for (int j = 0; j < 4; ++j)
                pk.u[j] = pack_bf16x2(x[q >> 1][si][8 * (q & 1) + 2 * j] * inv, x[q >> 1][si][8 * (q & 1) + 2 * j + 1] * inv);
            pf[si][q] = pk.v;
        }
    }
    __syncthreads();   // V^T in LDS (every wave of the block reaches this)
    // O[si][et] = P_si V_et
#pragma unroll
    for (int et = 0; et < 2; ++et) {
        bf16x8_t vf[4];
        const int e = 32 * et + r, er = e < HD ? e : HD - 1;
        if (32 * et >= HD) break;
#pragma unroll
        for (int q = 0; q < 4; ++q) {
            const int t0 = 16 * q + 4 * h;   // keys t0..t0+3 and t0+8..t0+11 (within tile q >> 1)
            union { uint2 u[2]; bf16x8_t v; } f;
            f.u[0] = *(const uint2*)&vt[er * LDT + t0];
            f.u[1] = *(const uint2*)&vt[er * LDT + t0 + 8];
            vf[q] = f.v;
        }
#pragma unroll
        for (int si = 0; si < 2; ++si) {
            f32x16_t acc = {0};
#pragma unroll
            for (int q = 0; q < 4; ++q) acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(pf[si][q], vf[q], acc, 0, 0, 0);
            if (valid && e < HD) {
#pragma unroll
                for (int g = 0; g < 16; ++g) {
                    const int s = 32 * si + (g & 3) + 8 * (g >> 2) + 4 * h;
                    if (s < S) put(s, e, acc[g]);
                }
            }
        }
    }
}

template <int HD, int H>
__global__ void __launch_bounds__(256) attn62_kernel(const uint16_t* __restrict__ qkv, uint16_t* __restrict__ y,
                                                     uint32_t batch, float scale) {
    constexpr int S = 62, D = HD * H, LDT = 64 + 4;
    __shared__ uint16_t vt_all[4][HD * LDT];
    const int wave = threadIdx.x >> 6;
    const uint32_t bh = blockIdx.x * 4u + (uint32_t)wave;
    const bool valid = bh < batch * (uint32_t)H;
    const uint32_t b = valid ? bh / H : 0u, hd = valid ? bh % H : 0u;
    attn62_head<HD, H>(qkv + (size_t)b * S * (3 * D), hd, valid, vt_all[wave], scale,
                       [&](int s, int e, float v) { y[((size_t)b * S + s) * D + hd * HD + e] = f2bf(v); });
}

// ---------------------------------------------------------------------------
// The attention half of a transformer block after the qkv projection, in one pass per sample:
//   y = MHA core (attn62_head, one wave per head; y stays in LDS)
//   delta = y Wp^T + bp   (the folded out_proj / c_proj GEMM, 16 rows per wave,
//                          v_mfma_f32_16x16x32_bf16, Wp fragments read through the caches)
//   x += delta;  h = LN(x)  (the residual add and ln_2, as add_ln)
// Unfused, y and delta each went to HBM and back (2 x 4 d bytes per token) in three launches.
// The sample's residual rows and both outputs move as coalesced 16-byte pieces of its 62
// contiguous rows.  Numerics as the unfused path: y rounded to bf16 (the attention output),
// delta + bias rounded to bf16 (the GEMM's output), x + delta rounded, LN of the rounded row.
typedef float f32x4_t __attribute__((ext_vector_type(4)));
// The block's tail after attention, shared by attn_ln_kernel and qkv_attn_ln_kernel: ys = the
// sample's y rows (64 x LDY, rows 62 and 63 zero), lds_a = free LDS for the residual rows.
// Call after a barrier that completes ys.
template <int HD>
__device__ __forceinline__ void proj_res_ln(const uint16_t* ys, uint16_t* lds_a, uint16_t* __restrict__ x_io,
                                            const uint16_t* __restrict__ wp, const uint16_t* __restrict__ bp, uint32_t b,
                                            const uint16_t* __restrict__ gamma, const uint16_t* __restrict__ beta, float eps,
                                            uint16_t* __restrict__ h_out) {
    constexpr int S = 62, D = HD * 4, LDY = D + 8, NT = D / 16, KS = D / 32;
    constexpr int NJ = (NT + 3) / 4;          // column tiles per wave: w, w + 4, w + 8, ...
    constexpr int XP = (S * (D / 8) + 255) / 256, LP = D / 32;   // 16-B pieces per thread: residual load, LN row
    static_assert(D % 32 == 0, "d: a multiple of 32");
    const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
    // the sample's residual rows: issued before the GEMM, stored to LDS after it
    uint16_t* xs = lds_a;
    const uint16_t* xg = x_io + (size_t)b * S * D;
    uint4 xr[XP];
#pragma unroll
    for (int i = 0; i < XP; ++i) {
        const int p = threadIdx.x + 256 * i;
        xr[i] = p < S * (D / 8) ? *(const uint4*)(xg + 8 * p) : make_uint4(0u, 0u, 0u, 0u);
    }
    // delta = y Wp^T, the wave's column tiles T = wave + 4 j over all 64 rows (each Wp
    // fragment read once per workgroup and used for 4 row tiles): A = y rows (lane: row rl,
    // k 8 kg .. +7), B[k][n] = Wp[n][k]
    const int rl = lane & 15, kg = lane >> 4;
    f32x4_t acc[4][NJ];
#pragma unroll
    for (int m = 0; m < 4; ++m)
#pragma unroll
        for (int j = 0; j < NJ; ++j) acc[m][j] = f32x4_t{0.0f, 0.0f, 0.0f, 0.0f};
    // Wp fragments one k-step ahead (a two-deep register ring): loaded inside the k-step that
    // used them, each L2 round trip sat between its load and its four MFMAs, KS x NJ times in a
    // row (the phase clocks of profiles/r04/net/attn_prof.log: the tail was the longest phase)
    auto wfrag = [&](int ks, int j) {
        const int t = wave + 4 * j;
        return load_frag8(wp + (size_t)(16 * (t < NT ? t : 0) + rl) * D + 32 * ks + 8 * kg, t < NT);
    };
    bf16x8_t wr[2][NJ];
#pragma unroll
    for (int j = 0; j < NJ; ++j) wr[0][j] = wfrag(0, j);
#pragma unroll
    for (int ks = 0; ks < KS; ++ks) {
        if (ks + 1 < KS) {
#pragma unroll
            for (int j = 0; j < NJ; ++j) wr[(ks + 1) & 1][j] = wfrag(ks + 1, j);
        }
        bf16x8_t a[4];
#pragma unroll
        for (int m = 0; m < 4; ++m) a[m] = *(const bf16x8_t*)&ys[(16 * m + rl) * LDY + 32 * ks + 8 * kg];
#pragma unroll
        for (int j = 0; j < NJ; ++j) {
            const int t = wave + 4 * j;
            if (t < NT) {
#pragma unroll
                for (int m = 0; m < 4; ++m) acc[m][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[m], wr[ks & 1][j], acc[m][j], 0, 0, 0);
            }
        }
    }
#pragma unroll
    for (int i = 0; i < XP; ++i) {
        const int p = threadIdx.x + 256 * i;
        if (p < S * (D / 8)) {
            const int rr = p / (D / 8), kp = p - rr * (D / 8);
            *(uint4*)&xs[rr * LDY + 8 * kp] = xr[i];
        }
    }
    __syncthreads();   // residual rows in xs
    // x' = x + bf16(delta + bias), rounded like the unfused add; in place in xs
#pragma unroll
    for (int j = 0; j < NJ; ++j) {
        const int t = wave + 4 * j;
        if (t < NT) {
            const int col = 16 * t + rl;
            const float bias = bf2f(bp[col]);
#pragma unroll
            for (int m = 0; m < 4; ++m)
#pragma unroll
                for (int v = 0; v < 4; ++v) {
                    const int row = 16 * m + 4 * kg + v;
                    const float delta = bf2f(f2bf(acc[m][j][v] + bias));
                    xs[row * LDY + col] = f2bf(bf2f(xs[row * LDY + col]) + delta);
                }
        }
    }
    __syncthreads();   // x' complete
    // LayerNorm: 4 threads per row, 16-B pieces q + 4 i; two-pass mean / variance
    {
        const int row = threadIdx.x >> 2, q = threadIdx.x & 3;
        float xv[LP][8];
        float s1 = 0.0f;
#pragma unroll
        for (int i = 0; i < LP; ++i) {
            union { uint4 u; uint16_t s[8]; } pc;
            pc.u = *(const uint4*)&xs[row * LDY + 8 * (q + 4 * i)];
#pragma unroll
            for (int e = 0; e < 8; ++e) {
                xv[i][e] = bf2f(pc.s[e]);
                s1 += xv[i][e];
            }
        }
        s1 += __shfl_xor(s1, 1);
        s1 += __shfl_xor(s1, 2);
        const float mean = s1 / (float)D;
        float s2 = 0.0f;
#pragma unroll
        for (int i = 0; i < LP; ++i)
#pragma unroll
            for (int e = 0; e < 8; ++e) {
                const float dv = xv[i][e] - mean;
                s2 += dv * dv;
            }
        s2 += __shfl_xor(s2, 1);
        s2 += __shfl_xor(s2, 2);
        const float rstd = rsqrtf(s2 / (float)D + eps);
        if (row < S) {
            const size_t o = ((size_t)b * S + row) * D;
#pragma unroll
            for (int i = 0; i < LP; ++i) {
                const int c0 = 8 * (q + 4 * i);
                union { uint4 u; uint16_t s[8]; uint32_t w[4]; } gv, bv, xo, ho;
                gv.u = *(const uint4*)(gamma + c0);
                bv.u = *(const uint4*)(beta + c0);
#pragma unroll
                for (int e = 0; e < 8; e += 2) {
                    xo.w[e / 2] = pack_bf16x2(xv[i][e], xv[i][e + 1]);
                    ho.w[e / 2] = pack_bf16x2((xv[i][e] - mean) * rstd * bf2f(gv.s[e]) + bf2f(bv.s[e]),
                                              (xv[i][e + 1] - mean) * rstd * bf2f(gv.s[e + 1]) + bf2f(bv.s[e + 1]));
                }
                *(uint4*)(x_io + o + c0) = xo.u;
                *(uint4*)(h_out + o + c0) = ho.u;
            }
        }
    }
}

template <int HD, int H>
__global__ void __launch_bounds__(256, 2) attn_ln_kernel(const uint16_t* __restrict__ qkv, uint16_t* __restrict__ x_io,
                                                         const uint16_t* __restrict__ wp, const uint16_t* __restrict__ bp,
                                                         uint32_t batch, float scale, const uint16_t* __restrict__ gamma,
                                                         const uint16_t* __restrict__ beta, float eps,
                                                         uint16_t* __restrict__ h_out) {
    static_assert(H == 4, "one wave per head, four waves per workgroup");
    constexpr int S = 62, D = HD * H, LDT = 64 + 4, LDY = D + 8;
    // LDS: the heads' V^T tiles, reused for the residual rows once attention is done (43 KB at
    // d = 160, 69 KB at d = 256), and the attention output rows
    constexpr int VT = 4 * HD * LDT, XS = 64 * LDY;
    __shared__ __attribute__((aligned(16))) uint16_t lds_a[VT > XS ? VT : XS];
    __shared__ __attribute__((aligned(16))) uint16_t ys[64 * LDY];
    const int wave = threadIdx.x >> 6;
    const uint32_t b = blockIdx.x;                                   // one sample per workgroup
    (void)batch;
    for (int i = threadIdx.x; i < 2 * D; i += 256) ys[(S + i / D) * LDY + i % D] = 0;   // A operand padding rows
    attn62_head<HD, H>(qkv + (size_t)b * S * (3 * D), (uint32_t)wave, true, lds_a + wave * HD * LDT, scale,
                       [&](int s, int e, float v) { ys[s * LDY + wave * HD + e] = f2bf(v); });
    __syncthreads();   // y complete in ys; the V^T tiles are dead
    proj_res_ln<HD>(ys, lds_a, x_io, wp, bp, b, gamma, beta, eps, h_out);
}

// ---------------------------------------------------------------------------
// The whole attention half of a block from h = ln_1(x), in one pass per sample: the qkv
// projection runs inside the workgroup, so q, k and v (3 x 2 d bytes per token) never go
// to HBM.  Wave w = head w computes its head's rows of Q^T, K^T and V^T = W h^T + b on
// v_mfma_f32_32x32x16_bf16 (A = Wqkv rows of the head, padded to 64 with zero rows; B = the
// sample's h rows from LDS):
//   V^T accumulators go straight to the wave's LDS V^T tile [e][t];
//   Q^T / K^T accumulators become the attention's fragments without moving between lanes:
//   lane (r, hh) holds token 32 si + r, dims 32 dt + (g & 3) + 8 (g >> 2) + 4 hh, and
//   registers g = 8 half .. 8 half + 7 of tile dt are k-step 2 dt + half of X = K Q^T.  The
//   contraction pairs equal (hh, j) of both operands, so Q and K only have to use the same
//   dimension order (k-steps of padding dimensions only are skipped).
// Then the attention core (attn62_core) and the tail as attn_ln_kernel.  LDS: the h rows and
// then y share one tile, the V^T tiles and then the residual rows another.
#ifndef DK_QKV_GS
#define DK_QKV_GS 2
#endif
#ifndef DK_QKV_WPE
#define DK_QKV_WPE 3
#endif
#ifndef DK_QKV_TAIL
#define DK_QKV_TAIL 0   // 1: HD = 40 Q / K / V dims 32..39 from one shared tile (head_tail_tile): 0.350 vs 0.343 ms, not kept
#endif
#ifndef DK_QKV_PF
#define DK_QKV_PF -1   // -1: per head size (below)
#endif
// DT1 = false: only the first 32-row tile (head dims 0..31); acc[1] stays zero (HD = 40: the
// dims 32..39 of Q, K and V come from one shared tile, head_tail_tile)
template <int HD, int D, bool DT1 = true>
__device__ __forceinline__ void head_tiles(const uint16_t* hs, const uint16_t* __restrict__ w,
                                           const uint16_t* __restrict__ bias, f32x16_t (&acc)[2][2]) {
    constexpr int LDY = D + 8;
    const int lane = threadIdx.x & 63, r = lane & 31, hh = lane >> 5;
#pragma unroll
    for (int dt = 0; dt < 2; ++dt)
#pragma unroll
        for (int si = 0; si < 2; ++si) acc[dt][si] = f32x16_t{0};
    // k order: groups of GS = 4 k-steps (64 k; a tail group of 2 at d = 160); in a group lane
    // half hh covers 8 GS consecutive k, 8 per k-step, so a lane reads 16 GS contiguous bytes
    // of its W row in GS back-to-back loads (the line is fetched once, then hit).  One 16-B
    // piece per row half per k-step instead thrashed L1 across k-steps: each 128-B line came
    // from L2 four times.  The h fragments (B operand, LDS) use the same order.
    const uint16_t* w0 = w + (size_t)r * D;
    const uint16_t* w1 = w + (size_t)(32 + r < HD ? 32 + r : 0) * D;
    const bool ok1 = 32 + r < HD;
    auto group = [&](auto gs_c, int k0) {
        constexpr int GS = decltype(gs_c)::value;
        const int kb = k0 + hh * 8 * GS;
        bf16x8_t wa[2][GS];
#pragma unroll
        for (int st = 0; st < GS; ++st) {
            wa[0][st] = load_frag8(w0 + kb + 8 * st, true);
            wa[1][st] = DT1 ? load_frag8(w1 + kb + 8 * st, ok1) : wa[0][st];
        }
#pragma unroll
        for (int st = 0; st < GS; ++st) {
            bf16x8_t hb[2];
#pragma unroll
            for (int si = 0; si < 2; ++si) hb[si] = *(const bf16x8_t*)&hs[(32 * si + r) * LDY + kb + 8 * st];
#pragma unroll
            for (int dt = 0; dt < (DT1 ? 2 : 1); ++dt)
#pragma unroll
                for (int si = 0; si < 2; ++si)
                    acc[dt][si] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(wa[dt][st], hb[si], acc[dt][si], 0, 0, 0);
        }
    };
    // d = 256 (two waves per SIMD): W fragments PF k-steps ahead in a register ring; a
    // scheduling barrier per k-step keeps the compiler from hoisting every load to the top
    // (0.77 -> 0.73 ms at 8192 samples).  d = 160 keeps its third wave per SIMD instead
    // (the ring spills there, and one k-step ahead was no faster: tools/attn_bench.py).
    constexpr int PF = DK_QKV_PF >= 0 ? DK_QKV_PF : (HD == 64 ? 2 : 0);
    if constexpr (PF > 0) {
    constexpr int NKS = D / 16;
    bf16x8_t ring[PF][2];
#pragma unroll
    for (int p = 0; p < PF; ++p) {
        ring[p][0] = load_frag8(w0 + 16 * p + 8 * hh, true);
        ring[p][1] = load_frag8(w1 + 16 * p + 8 * hh, ok1);
    }
#pragma unroll
    for (int ks = 0; ks < NKS; ++ks) {
        const bf16x8_t a0 = ring[ks % PF][0], a1 = ring[ks % PF][1];
        if (ks + PF < NKS) {
            ring[ks % PF][0] = load_frag8(w0 + 16 * (ks + PF) + 8 * hh, true);
            ring[ks % PF][1] = load_frag8(w1 + 16 * (ks + PF) + 8 * hh, ok1);
        }
        bf16x8_t hb[2];
#pragma unroll
        for (int si = 0; si < 2; ++si) hb[si] = *(const bf16x8_t*)&hs[(32 * si + r) * LDY + 16 * ks + 8 * hh];
#pragma unroll
        for (int si = 0; si < 2; ++si) {
            acc[0][si] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a0, hb[si], acc[0][si], 0, 0, 0);
            acc[1][si] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a1, hb[si], acc[1][si], 0, 0, 0);
        }
        __builtin_amdgcn_sched_barrier(0);
    }
    } else {
    constexpr int G = DK_QKV_GS, NG = D / (16 * G), TAIL = (D % (16 * G)) / 16;
#pragma unroll 1
    for (int gi = 0; gi < NG; ++gi) group(std::integral_constant<int, G>{}, 16 * G * gi);
    if constexpr (TAIL > 0) group(std::integral_constant<int, TAIL>{}, 16 * G * NG);
    }
#pragma unroll
    for (int dt = 0; dt < 2; ++dt)
#pragma unroll
        for (int g = 0; g < 16; ++g) {
            const int m = 32 * dt + (g & 3) + 8 * (g >> 2) + 4 * hh;
            const float bv = m < HD && (DT1 || dt == 0) ? bf2f(bias[m]) : 0.0f;
            acc[dt][0][g] += bv;
            acc[dt][1][g] += bv;
        }
}

// HD = 40: the head dims 32..39 of Q, K and V as ONE 32-row tile -- A row r is row 32 + (r & 7)
// of projection r >> 3 (Q, K, V; rows 24..31 repeat Q's and are discarded) -- instead of three
// tiles that are three quarters padding (20 MFMAs for the three tails instead of 60).  Register
// g < 4 (+ 4 p) of tail[si] holds projection p's dim 32 + (g & 3) + 4 hh of token 32 si + r, bias
// included (the register order of tile 1 of head_tiles).  w: the head's Q rows; K's and V's are
// D * D elements further, the biases D further.
template <int HD, int D>
__device__ __forceinline__ void head_tail_tile(const uint16_t* hs, const uint16_t* __restrict__ w,
                                               const uint16_t* __restrict__ bias, f32x16_t (&tail)[2]) {
    static_assert(HD == 40, "three tails of 8 rows in one tile");
    constexpr int LDY = D + 8, NKS = D / 16;
    const int lane = threadIdx.x & 63, r = lane & 31, hh = lane >> 5;
    const int pr = (r >> 3) < 3 ? (r >> 3) : 0;
    const uint16_t* wr = w + (size_t)pr * D * D + (size_t)(32 + (r & 7)) * D + 8 * hh;
    tail[0] = f32x16_t{0};
    tail[1] = f32x16_t{0};
    bf16x8_t nw = load_frag8(wr, true);
#pragma unroll
    for (int ks = 0; ks < NKS; ++ks) {
        const bf16x8_t a = nw;
        if (ks + 1 < NKS) nw = load_frag8(wr + 16 * (ks + 1), true);
        __builtin_amdgcn_sched_barrier(0);
#pragma unroll
        for (int si = 0; si < 2; ++si) {
            const bf16x8_t hb = *(const bf16x8_t*)&hs[(32 * si + r) * LDY + 16 * ks + 8 * hh];
            tail[si] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, hb, tail[si], 0, 0, 0);
        }
        __builtin_amdgcn_sched_barrier(0);
    }
#pragma unroll
    for (int g = 0; g < 12; ++g) {
        const float bv = bf2f(bias[(g >> 2) * D + 32 + (g & 3) + 4 * hh]);
        tail[0][g] += bv;
        tail[1][g] += bv;
    }
}

template <int HD>
__device__ __forceinline__ void pack_head(const f32x16_t (&acc)[2][2], bf16x8_t (&f)[2][(HD + 15) / 16]) {
#pragma unroll
    for (int si = 0; si < 2; ++si)
#pragma unroll
        for (int kk = 0; kk < (HD + 15) / 16; ++kk) {
            union { uint32_t u[4]; bf16x8_t v; } pk;
#pragma unroll
            for (int j = 0; j < 4; ++j)
                pk.u[j] = pack_bf16x2(acc[kk >> 1][si][8 * (kk & 1) + 2 * j], acc[kk >> 1][si][8 * (kk & 1) + 2 * j + 1]);
            f[si][kk] = pk.v;
        }
}

// Phase clocks of qkv_attn_ln_kernel (profiling builds, -DDK_NET_PROF): wave 0 of each
// workgroup stamps the shader clock after each phase; dk_net_prof_read sums them.
#ifdef DK_NET_PROF
__device__ unsigned long long dk_net_prof_acc[8];
__device__ unsigned long long dk_mlp_prof_acc[16];   // mlp_ln_kernel: [wave 0 | wave 4][phase]
#define DK_NSTAMP(k) do { const unsigned long long t_ = __builtin_amdgcn_s_memtime(); \
    if (threadIdx.x == 0) atomicAdd(&dk_net_prof_acc[k], t_ - t_prev); t_prev = t_; } while (0)
#else
#define DK_NSTAMP(k) ((void)0)
#endif
template <int HD>
__global__ void __launch_bounds__(256, HD == 40 ? DK_QKV_WPE : 2) qkv_attn_ln_kernel(const uint16_t* __restrict__ h_in, uint16_t* __restrict__ x_io,
                                                             const uint16_t* __restrict__ wqkv, const uint16_t* __restrict__ bqkv,
                                                             const uint16_t* __restrict__ wp, const uint16_t* __restrict__ bp,
                                                             uint32_t batch, float scale, const uint16_t* __restrict__ gamma,
                                                             const uint16_t* __restrict__ beta, float eps,
                                                             uint16_t* __restrict__ h_out) {
    constexpr int S = 62, D = HD * 4, LDT = 64 + 4, LDY = D + 8, KS = (HD + 15) / 16;
    constexpr int VT = 4 * HD * LDT, XS = 64 * LDY;
    __shared__ __attribute__((aligned(16))) uint16_t lds_a[VT > XS ? VT : XS];   // V^T tiles, then residual rows
    __shared__ __attribute__((aligned(16))) uint16_t ys[64 * LDY];               // h rows, then y rows
    const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
    const uint32_t b = blockIdx.x;                                                // one sample per workgroup
    (void)batch;
#ifdef DK_NET_PROF
    unsigned long long t_prev = __builtin_amdgcn_s_memtime();
#endif
    const uint16_t* hg = h_in + (size_t)b * S * D;
    {
        // every load issued before the first LDS store (a load -> store loop waited a memory
        // round trip per iteration); rows 62, 63 zero
        constexpr int NPC = 64 * (D / 8) / 256;
        static_assert(64 * (D / 8) % 256 == 0, "whole pieces per thread");
        // (the thread index through an opaque copy: the compiler otherwise kept index terms of
        // this prologue alive for the epilogue's LDS writes and spilled them)
        int tid = (int)threadIdx.x;
        asm volatile("" : "+v"(tid));
        uint4 v[NPC];
#pragma unroll
        for (int i = 0; i < NPC; ++i) {
            const int p = tid + 256 * i, rr = p / (D / 8), kp = p - rr * (D / 8);
            v[i] = *(const uint4*)(hg + (size_t)(rr < S ? rr : S - 1) * D + 8 * kp);
        }
#pragma unroll
        for (int i = 0; i < NPC; ++i) {
            const int p = tid + 256 * i, rr = p / (D / 8), kp = p - rr * (D / 8);
            *(uint4*)&ys[rr * LDY + 8 * kp] = rr < S ? v[i] : make_uint4(0u, 0u, 0u, 0u);
        }
    }
    __syncthreads();
    DK_NSTAMP(0);
    const int hh = lane >> 5, r = lane & 31;
    const uint16_t* wh = wqkv + (size_t)wave * HD * D;   // the head's q rows; k, v rows d and 2 d further
    const uint16_t* bh = bqkv + wave * HD;
    uint16_t* vt = lds_a + wave * HD * LDT;
    bf16x8_t qf[2][KS], kf[2][KS];
    if constexpr (HD == 40 && DK_QKV_TAIL) {
        // dims 32..39 of V, K and Q from one shared tile (head_tail_tile), dims 0..31 per projection
        f32x16_t tl[2];
        head_tail_tile<HD, D>(ys, wh, bh, tl);
        f32x16_t acc[2][2];
        head_tiles<HD, D, false>(ys, wh + (size_t)2 * D * D, bh + 2 * D, acc);    // V^T -> [e][t]
#pragma unroll
        for (int g = 0; g < 16; ++g) {
            const int m = (g & 3) + 8 * (g >> 2) + 4 * hh;
            vt[m * LDT + r] = f2bf(acc[0][0][g]);
            vt[m * LDT + 32 + r] = f2bf(acc[0][1][g]);
        }
#pragma unroll
        for (int g = 0; g < 4; ++g) {
            const int m = 32 + g + 4 * hh;
            vt[m * LDT + r] = f2bf(tl[0][8 + g]);
            vt[m * LDT + 32 + r] = f2bf(tl[1][8 + g]);
        }
        DK_NSTAMP(1);
        head_tiles<HD, D, false>(ys, wh + (size_t)D * D, bh + D, acc);            // K^T
#pragma unroll
        for (int si = 0; si < 2; ++si)
#pragma unroll
            for (int g = 0; g < 4; ++g) acc[1][si][g] = tl[si][4 + g];
        pack_head<HD>(acc, kf);
        DK_NSTAMP(2);
        head_tiles<HD, D, false>(ys, wh, bh, acc);                                // Q^T
#pragma unroll
        for (int si = 0; si < 2; ++si)
#pragma unroll
            for (int g = 0; g < 4; ++g) acc[1][si][g] = tl[si][g];
        pack_head<HD>(acc, qf);
        DK_NSTAMP(3);
    } else {
        f32x16_t acc[2][2];
        head_tiles<HD, D>(ys, wh + (size_t)2 * D * D, bh + 2 * D, acc);    // V^T -> [e][t]
#pragma unroll
        for (int dt = 0; dt < 2; ++dt)
#pragma unroll
            for (int g = 0; g < 16; ++g) {
                const int m = 32 * dt + (g & 3) + 8 * (g >> 2) + 4 * hh;
                if (m < HD) {
                    vt[m * LDT + r] = f2bf(acc[dt][0][g]);
                    vt[m * LDT + 32 + r] = f2bf(acc[dt][1][g]);
                }
            }
        DK_NSTAMP(1);
        head_tiles<HD, D>(ys, wh + (size_t)D * D, bh + D, acc);            // K^T
        pack_head<HD>(acc, kf);
        DK_NSTAMP(2);
        head_tiles<HD, D>(ys, wh, bh, acc);                                // Q^T
        pack_head<HD>(acc, qf);
        DK_NSTAMP(3);
    }
    // attn62_core's barrier also ends every wave's reads of the h rows: y may then overwrite them
    attn62_core<HD>(qf, kf, vt, scale, true, [&](int s, int e, float v) { ys[s * LDY + wave * HD + e] = f2bf(v); });
    DK_NSTAMP(4);
    __syncthreads();   // y complete (rows 62, 63 still the zero h padding); the V^T tiles are dead
    DK_NSTAMP(5);
    proj_res_ln<HD>(ys, lds_a, x_io, wp, bp, b, gamma, beta, eps, h_out);
    DK_NSTAMP(6);
}

// ---------------------------------------------------------------------------
// PerClassAttentionMLPHead's pooling and its classes' LayerNorms (az_doko.py:42-50 and the
// nn.LayerNorm that opens each class MLP), one 256-thread workgroup per sample:
//   scores^T = X Q^T        (v_mfma_f32_32x32x16_bf16; the token in the registers, the class
//                            on the lane; rounded to bf16, times scale, rounded: the bf16 torch ops)
//   P = softmax over the 62 tokens (registers + one cross-half shuffle), packed in place as
//       the A operand of
//   A = P X                 (X^T staged in LDS as [d][t], as V^T in the attention core)
//   out[c][b][:] = LN(A[c]) * w[c] + b[c]   (written class-major: the [C, B, d] operand of the
//                                           classes' batched MLP GEMM, no transpose copy)
// Class tiles of 32 (C <= 64): with one class tile the four waves split the d tiles, with two
// each pair does.  LDS: the x rows (then the pooled rows) and x^T.
template <int D>
__global__ void __launch_bounds__(256, 2) class_pool_ln_kernel(const uint16_t* __restrict__ xin, uint32_t batch,
                                                               const uint16_t* __restrict__ queries, uint32_t classes,
                                                               float scale, const uint16_t* __restrict__ lnw,
                                                               const uint16_t* __restrict__ lnb, float eps,
                                                               uint16_t* __restrict__ out) {
    constexpr int S = 62, LDX = D + 8, LDT = 64 + 4, KD = D / 16, DT = D / 32, LP = D / 32;
    static_assert(D % 32 == 0, "d: a multiple of 32");
    __shared__ __attribute__((aligned(16))) uint16_t xs[64 * LDX];   // x rows, then the pooled rows
    __shared__ __attribute__((aligned(16))) uint16_t xt[D * LDT];    // x^T [d][t]
    const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63, r = lane & 31, hh = lane >> 5;
    const uint32_t b = blockIdx.x;                                   // one sample per workgroup
    const int C = (int)classes;
    const uint16_t* xg = xin + (size_t)b * S * D;
    {
        // every load issued before the first LDS store; rows 62, 63 zero
        constexpr int NPC = 64 * (D / 8) / 256;
        static_assert(64 * (D / 8) % 256 == 0, "whole pieces per thread");
        uint4 v[NPC];
#pragma unroll
        for (int i = 0; i < NPC; ++i) {
            const int p = threadIdx.x + 256 * i, t = p / (D / 8), d0 = 8 * (p - t * (D / 8));
            v[i] = *(const uint4*)(xg + (size_t)(t < S ? t : S - 1) * D + d0);
        }
#pragma unroll
        for (int i = 0; i < NPC; ++i) {
            const int p = threadIdx.x + 256 * i, t = p / (D / 8), d0 = 8 * (p - t * (D / 8));
            *(uint4*)&xs[t * LDX + d0] = t < S ? v[i] : make_uint4(0u, 0u, 0u, 0u);
        }
    }
    __syncthreads();
    // x^T from the rows in LDS: thread (d, t0) gathers 8 tokens of one dimension (2-B reads, a
    // half-wave on 32 consecutive dimensions of a row) and writes them as two 8-B pieces.  The
    // direct 2-B scatter of the loaded pieces put 16 lanes on two banks (67 % of LDS cycles
    // were bank conflicts, profiles/r04/net/pmc_c5net.json).
    for (int p = threadIdx.x; p < D * 8; p += 256) {
        const int dd = p % D, t0 = 8 * (p / D);
        union { uint2 u[2]; uint16_t s[8]; } v;
#pragma unroll
        for (int m = 0; m < 8; ++m) v.s[m] = xs[(t0 + m) * LDX + dd];
        uint2* o = (uint2*)&xt[dd * LDT + t0];   // (rows of 136 B: 8-B aligned)
        o[0] = v.u[0];
        o[1] = v.u[1];
    }
    __syncthreads();
    const int CT = C > 32 ? 2 : 1, WPC = 4 / CT;       // class tiles, waves per class tile
    const int ct = wave % CT, part = wave / CT;
    const int cls = 32 * ct + r;
    f32x16_t sc[2];
    sc[0] = f32x16_t{0};
    sc[1] = f32x16_t{0};
    // the query fragments one k-step ahead (an L2 round trip per step otherwise)
    const uint16_t* qrow = queries + (size_t)(cls < C ? cls : 0) * D + 8 * hh;
    uint4 qn = *(const uint4*)qrow;
#pragma unroll
    for (int ks = 0; ks < KD; ++ks) {
        const uint4 qu = qn;
        if (ks + 1 < KD) qn = *(const uint4*)(qrow + 16 * (ks + 1));
        union { uint4 u; bf16x8_t v; } qcv;
        qcv.u = cls < C ? qu : make_uint4(0u, 0u, 0u, 0u);
        const bf16x8_t qf = qcv.v;
#pragma unroll
        for (int mt = 0; mt < 2; ++mt) {
            const bf16x8_t xa = *(const bf16x8_t*)&xs[(32 * mt + r) * LDX + 16 * ks + 8 * hh];
            sc[mt] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(xa, qf, sc[mt], 0, 0, 0);
        }
    }
    // softmax over the tokens t < 62 of the lane's class
    bf16x8_t pf[4];
    {
        float mx = -INFINITY;
#pragma unroll
        for (int mt = 0; mt < 2; ++mt)
#pragma unroll
            for (int g = 0; g < 16; ++g) {
                const int t = 32 * mt + (g & 3) + 8 * (g >> 2) + 4 * hh;
                const float v = bf2f(f2bf(bf2f(f2bf(sc[mt][g])) * scale));
                sc[mt][g] = v;
                if (t < S) mx = fmaxf(mx, v);
            }
        mx = fmaxf(mx, __shfl_xor(mx, 32));
        float l = 0.0f;
#pragma unroll
        for (int mt = 0; mt < 2; ++mt)
#pragma unroll
            for (int g = 0; g < 16; ++g) {
                const int t = 32 * mt + (g & 3) + 8 * (g >> 2) + 4 * hh;
                const float e = t < S ? __expf(sc[mt][g] - mx) : 0.0f;
                sc[mt][g] = e;
                l += e;
            }
        l += __shfl_xor(l, 32);
        const float inv = 1.0f / l;
#pragma unroll
        for (int q = 0; q < 4; ++q) {
            union { uint32_t u[4]; bf16x8_t v; } pk;
#pragma unroll
            for (int j = 0; j < 4; ++j)
                pk.u[j] = pack_bf16x2(sc[q >> 1][8 * (q & 1) + 2 * j] * inv, sc[q >> 1][8 * (q & 1) + 2 * j + 1] * inv);
            pf[q] = pk.v;
        }
    }
    // A = P X for the wave's d tiles t = part, part + WPC, ...
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
                union { uint2 u[2]; bf16x8_t v; } f;
                f.u[0] = *(const uint2*)&xt[(32 * t + r) * LDT + t0];
                f.u[1] = *(const uint2*)&xt[(32 * t + r) * LDT + t0 + 8];
                acc[i] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(pf[q], f.v, acc[i], 0, 0, 0);
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
                if (c < C) xs[c * LDX + 32 * t + r] = f2bf(acc[i][g]);
            }
        }
    }
    __syncthreads();
    // LayerNorm of each class row with the class's affine: 4 threads per row
    {
        const int c = threadIdx.x >> 2, q = threadIdx.x & 3;
        float xv[LP][8];
        float s1 = 0.0f;
#pragma unroll
        for (int i = 0; i < LP; ++i) {
            union { uint4 u; uint16_t s[8]; } pc;
            pc.u = *(const uint4*)&xs[c * LDX + 8 * (q + 4 * i)];
#pragma unroll
            for (int e = 0; e < 8; ++e) {
                xv[i][e] = bf2f(pc.s[e]);
                s1 += xv[i][e];
            }
        }
        s1 += __shfl_xor(s1, 1);
        s1 += __shfl_xor(s1, 2);
        const float mean = s1 / (float)D;
        float s2 = 0.0f;
#pragma unroll
        for (int i = 0; i < LP; ++i)
#pragma unroll
            for (int e = 0; e < 8; ++e) {
                const float dv = xv[i][e] - mean;
                s2 += dv * dv;
            }
        s2 += __shfl_xor(s2, 1);
        s2 += __shfl_xor(s2, 2);
        const float rstd = rsqrtf(s2 / (float)D + eps);
        if (c < C) {
            const size_t o = ((size_t)c * batch + b) * D;
#pragma unroll
            for (int i = 0; i < LP; ++i) {
                const int c0 = 8 * (q + 4 * i);
                union { uint4 u; uint16_t s[8]; uint32_t w[4]; } gv, bv, ho;
                gv.u = *(const uint4*)(lnw + (size_t)c * D + c0);
                bv.u = *(const uint4*)(lnb + (size_t)c * D + c0);
#pragma unroll
                for (int e = 0; e < 8; e += 2)
                    ho.w[e / 2] = pack_bf16x2((xv[i][e] - mean) * rstd * bf2f(gv.s[e]) + bf2f(bv.s[e]),
                                              (xv[i][e + 1] - mean) * rstd * bf2f(gv.s[e + 1]) + bf2f(bv.s[e + 1]));
                *(uint4*)(out + o + c0) = ho.u;
            }
        }
    }
}

// ---------------------------------------------------------------------------
// The MLP's first layer with its activation: y = GELU(x W^T + b), exact (erf) GELU as
// the reference's nn.GELU(), for the networks' small K (= d: 160 AlphaZero, 256 IMPI).
// hipBLASLt runs this GEMM at 160-320 TFLOP/s and the separate GELU pass re-reads and
// re-writes the 4d-wide activation; here the activation is written once.
//   workgroup: 4 waves x RT row tiles of 32 rows; a wave's x fragments (all K) stay in
//   registers for the whole N loop;
//   N loop: 64-column chunks of W staged in LDS (double-buffered, shared by the 4
//   waves); per k-step RT x 2 tiles of v_mfma_f32_32x32x16_bf16 computing D^T = W x^T,
//   so a lane holds one row and, per register quad, 4 consecutive columns;
//   epilogue: bias + GELU on the f32 accumulators, 4 columns packed into one 8-byte store.
// GELU(v) = v Phi(v) = 0.5 v (1 + erf(v / sqrt 2)).  erf by Abramowitz & Stegun 7.1.26
// (|error| <= 1.5e-7, here about 3e-7 with the hardware rcp / exp2): 1 - erf(z) =
// (a1 t + ... + a5 t^5) exp(-z^2), t = 1 / (1 + p z), z >= 0.  That is the size of f32's own
// rounding of 1 + erf near -1 (6e-8) and far below the bf16 output's resolution; the
// library erff costs several times as many instructions and bounded this kernel.
__device__ __forceinline__ float gelu_erf(float v) {
    const float z = fabsf(v) * 0.70710678118654752f;
    const float t = __builtin_amdgcn_rcpf(fmaf(0.3275911f, z, 1.0f));
    float p = fmaf(1.061405429f, t, -1.453152027f);
    p = fmaf(p, t, 1.421413741f);
    p = fmaf(p, t, -0.284496736f);
    p = fmaf(p, t, 0.254829592f);
    const float e = __builtin_amdgcn_exp2f(-z * z * 1.4426950408889634f);
    const float c = p * t * e;                       // erfc(z) = 1 - erf(z)
    const float phi = v >= 0.0f ? 1.0f - 0.5f * c : 0.5f * c;
    return v * phi;
}

// the same on a pair, so that the FMAs / multiplies issue as packed f32 (v_pk_fma_f32)
typedef float f32x2_t __attribute__((ext_vector_type(2)));
__device__ __forceinline__ f32x2_t gelu_erf2(f32x2_t v) {
    const f32x2_t z = __builtin_elementwise_abs(v) * 0.70710678118654752f;
    const f32x2_t d = __builtin_elementwise_fma(f32x2_t{0.3275911f, 0.3275911f}, z, f32x2_t{1.0f, 1.0f});
    const f32x2_t t = {__builtin_amdgcn_rcpf(d.x), __builtin_amdgcn_rcpf(d.y)};
    f32x2_t p = __builtin_elementwise_fma(f32x2_t{1.061405429f, 1.061405429f}, t, f32x2_t{-1.453152027f, -1.453152027f});
    p = __builtin_elementwise_fma(p, t, f32x2_t{1.421413741f, 1.421413741f});
    p = __builtin_elementwise_fma(p, t, f32x2_t{-0.284496736f, -0.284496736f});
    p = __builtin_elementwise_fma(p, t, f32x2_t{0.254829592f, 0.254829592f});
    const f32x2_t a = -z * z * 1.4426950408889634f;
    const f32x2_t e = {__builtin_amdgcn_exp2f(a.x), __builtin_amdgcn_exp2f(a.y)};
    const f32x2_t c = p * t * e;
    const f32x2_t half_c = 0.5f * c;
    const f32x2_t phi = {v.x >= 0.0f ? 1.0f - half_c.x : half_c.x, v.y >= 0.0f ? 1.0f - half_c.y : half_c.y};
    return v * phi;
}

template <int K>
__global__ void __launch_bounds__(256, 2) fc_gelu_kernel(const uint16_t* __restrict__ x, const uint16_t* __restrict__ w,
                                                         const uint16_t* __restrict__ bias, uint16_t* __restrict__ y,
                                                         uint32_t rows, uint32_t n) {
    static_assert(K % 16 == 0, "K: a multiple of 16");
    // K = 160: 64-column chunks, 2 row tiles per wave; K = 256: 32-column chunks, 1 row tile
    // (registers and LDS for two workgroups per CU)
    constexpr int KS = K / 16, NC = K <= 160 ? 64 : 32, CT = NC / 32, LDW = K + 8, RT = K <= 160 ? 2 : 1, LDT = NC + 8;
    __shared__ uint16_t ws[2][NC * LDW];
    __shared__ uint16_t tile[4][32 * RT * LDT];   // per-wave output staging
    const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63, r = lane & 31, h = lane >> 5;
    const uint32_t row0 = blockIdx.x * (128u * RT) + (uint32_t)wave * (32u * RT);
    bf16x8_t af[RT][KS];
#pragma unroll
    for (int i = 0; i < RT; ++i) {
        const uint32_t row = row0 + 32u * i + (uint32_t)r;
        const bool ok = row < rows;
        const uint16_t* xr = x + (size_t)(ok ? row : 0u) * K + 8 * h;
#pragma unroll
        for (int kk = 0; kk < KS; ++kk) af[i][kk] = load_frag8(xr + 16 * kk, ok);
    }
    auto stage = [&](uint32_t c, int buf) {
        const uint16_t* src = w + (size_t)c * NC * K;
        for (int v = threadIdx.x; v < NC * (K / 8); v += 256) {
            const int col = v / (K / 8), k8 = v - col * (K / 8);
            *(uint4*)&ws[buf][col * LDW + 8 * k8] = *(const uint4*)(src + (size_t)col * K + 8 * k8);
        }
    };
    const uint32_t chunks = n / NC;
    stage(0, 0);
    __syncthreads();
    for (uint32_t c = 0; c < chunks; ++c) {
        const int buf = (int)(c & 1u);
        if (c + 1 < chunks) stage(c + 1, buf ^ 1);
        f32x16_t acc[RT][CT];
#pragma unroll
        for (int i = 0; i < RT; ++i)
#pragma unroll
            for (int j = 0; j < CT; ++j) acc[i][j] = f32x16_t{0};
#pragma unroll
        for (int kk = 0; kk < KS; ++kk) {
            bf16x8_t bfr[CT];
#pragma unroll
            for (int j = 0; j < CT; ++j) bfr[j] = *(const bf16x8_t*)&ws[buf][(32 * j + r) * LDW + 16 * kk + 8 * h];
#pragma unroll
            for (int i = 0; i < RT; ++i)
#pragma unroll
                for (int j = 0; j < CT; ++j) acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(bfr[j], af[i][kk], acc[i][j], 0, 0, 0);
        }
        // acc[i][j][g]: row row0 + 32 i + r, column c*NC + 32 j + (g & 3) + 8 (g >> 2) + 4 h.
        // bias + GELU, 4 columns packed per 8-byte LDS write into the wave's [32 RT][NC] tile,
        // then written out as whole row segments of NC columns (NC / 8 lanes per row)
        uint16_t* tw = tile[wave];
#pragma unroll
        for (int j = 0; j < CT; ++j) {
#pragma unroll
            for (int q = 0; q < 4; ++q) {
                const int cl = 32 * j + 8 * q + 4 * h;
                const uint2 bb = *(const uint2*)(bias + c * NC + cl);
                const float b0 = bf2f((uint16_t)bb.x), b1 = bf2f((uint16_t)(bb.x >> 16));
                const float b2 = bf2f((uint16_t)bb.y), b3 = bf2f((uint16_t)(bb.y >> 16));
#pragma unroll
                for (int i = 0; i < RT; ++i) {
                    const f32x2_t g01 = gelu_erf2(f32x2_t{acc[i][j][4 * q + 0] + b0, acc[i][j][4 * q + 1] + b1});
                    const f32x2_t g23 = gelu_erf2(f32x2_t{acc[i][j][4 * q + 2] + b2, acc[i][j][4 * q + 3] + b3});
                    uint2 o;
                    o.x = pack_bf16x2(g01.x, g01.y);
                    o.y = pack_bf16x2(g23.x, g23.y);
                    *(uint2*)&tw[(32 * i + r) * LDT + cl] = o;
                }
            }
        }
        __builtin_amdgcn_s_waitcnt(0xC07F);   // this wave's LDS writes done (lgkmcnt(0))
#pragma unroll
        for (int p = 0; p < RT * NC / 16; ++p) {
            const int v = 64 * p + lane, rl = v / (NC / 8), sg = v % (NC / 8);
            const uint32_t row = row0 + (uint32_t)rl;
            const uint4 o = *(const uint4*)&tw[rl * LDT + 8 * sg];
            if (row < rows) *(uint4*)(y + (size_t)row * n + c * NC + 8 * sg) = o;
        }
        // LDS-only barrier: the next chunk's W is in LDS and this chunk's reads of the other
        // buffer are done; the output stores stay in flight (__syncthreads would wait for them)
        asm volatile("" ::: "memory");
        __builtin_amdgcn_s_waitcnt(0xC07F);   // lgkmcnt(0), vmcnt / expcnt untouched
        __builtin_amdgcn_s_barrier();
        asm volatile("" ::: "memory");
    }
}

// ---------------------------------------------------------------------------
// The whole MLP half of a transformer block in one pass (d = 160, the AlphaZero network, in
// chunks of NC = 64 hidden units; d = 256, the IMPI network, NC = 32 to fit the registers):
//   a = GELU(h W1^T + b1)          (4d hidden units, NC at a time, never leaving the CU)
//   delta = a W2^T + b2            (accumulated over the hidden chunks in registers)
//   x += delta;  h' = LN'(x)       (the residual add and the NEXT LayerNorm, as add_ln)
// Unfused, the block's MLP wrote and re-read the 4d-wide activation (1,280 B per row each
// way) and the 2d-byte delta; here a row costs its h and x reads and its x and h' writes.
//   workgroup: 8 waves x 32 rows; a wave's h fragments (all of K = d) stay in registers;
//   chunk loop over the hidden units: W1 rows [NC x d] and W2 columns [d x NC] of the chunk
//   staged in LDS (double-buffered, shared by the 8 waves);
//   GEMM1: D1 = W1_c h^T, NC / 32 tiles of 32 hidden units x 32 rows (v_mfma_f32_32x32x16_bf16);
//   the bias + GELU'd accumulators ARE the B operand of GEMM2 without moving between lanes:
//   MFMA sums over k, so the k order only has to agree between A and B.  Lane (r, hh)
//   holds hidden units 32j + (g & 3) + 8 (g >> 2) + 4 hh of its row; k-step s = 2j + half
//   takes its registers g = 8 half .. 8 half + 7, and the W2 fragment of the same k-step
//   reads the matching hidden units (two runs of 4) from the LDS copy of W2;
//   GEMM2: D2 = W2_c a^T, d / 32 tiles of 32 output columns x 32 rows, NC / 16 k-steps per chunk;
//   epilogue: delta rounded to bf16 (torch's proj output), x + delta rounded to bf16, the
//   row's mean / variance over the two half-wave lanes that hold it, h' = LN'(x).
// GELU for the fused MLP: the same A&S 7.1.26 erf, rearranged for packed f32 (no selects):
// GELU(v) = 0.5 v (1 + erf(v / sqrt2)) = 0.5 (v + |v|) - 0.5 |v| erfc(|v| / sqrt2), erf being odd.
__device__ __forceinline__ f32x2_t gelu_erf2_pk(f32x2_t v) {
    const f32x2_t a = __builtin_elementwise_abs(v);
    const f32x2_t z = a * 0.70710678118654752f;
    const f32x2_t d = __builtin_elementwise_fma(f32x2_t{0.3275911f, 0.3275911f}, z, f32x2_t{1.0f, 1.0f});
    const f32x2_t t = {__builtin_amdgcn_rcpf(d.x), __builtin_amdgcn_rcpf(d.y)};
    f32x2_t p = __builtin_elementwise_fma(f32x2_t{1.061405429f, 1.061405429f}, t, f32x2_t{-1.453152027f, -1.453152027f});
    p = __builtin_elementwise_fma(p, t, f32x2_t{1.421413741f, 1.421413741f});
    p = __builtin_elementwise_fma(p, t, f32x2_t{-0.284496736f, -0.284496736f});
    p = __builtin_elementwise_fma(p, t, f32x2_t{0.254829592f, 0.254829592f});
    const f32x2_t q = z * (z * -1.4426950408889634f);
    const f32x2_t e = {__builtin_amdgcn_exp2f(q.x), __builtin_amdgcn_exp2f(q.y)};
    const f32x2_t c = (p * t) * e;                                   // erfc(|v| / sqrt2)
    const f32x2_t ha = a * 0.5f;
    return __builtin_elementwise_fma(-ha, c, __builtin_elementwise_fma(v, f32x2_t{0.5f, 0.5f}, ha));
}

// GELU with erfc from one exp2 and no reciprocal (round 4): with a = min(|v|, 5.5),
// log2 erfc(a / sqrt2) ~= a (c0 + c1 a + ... + c5 a^5) (least squares on [0, 5.5] weighted by
// 0.5 a erfc, the GELU error it causes), GELU(v) = max(v, 0) - 0.5 |v| erfc(|v| / sqrt2).
// Beyond |v| = 5.5 the erfc term (< 1.1e-7 there, falling faster than |v| grows) is dropped:
// GELU = max(v, 0), one select, so the error cannot grow with |v|.
// |error| <= 2.9e-7 over all f32 v (f32 evaluation in the kernel's fma order against the f64 erf
// form on [-1e4, 1e4], tests/test_cpu_gelu_poly.py); a third of the bf16 rounding flips of the
// A&S 7.1.26 form above.  9 VALU + 1 transcendental per value against 13 + 2 (the abs values
// are source modifiers).
#ifndef DK_GELU_POLY
#define DK_GELU_POLY 1
#endif
__device__ __forceinline__ float gelu_poly(float v) {
    const float a = fminf(fabsf(v), 5.5f);
    float q = 3.236920019844547e-05f;
    q = fmaf(q, a, -0.0007541869999840856f);
    q = fmaf(q, a, 0.008001405745744705f);
    q = fmaf(q, a, -0.05324144661426544f);
    q = fmaf(q, a, -0.45893436670303345f);
    q = fmaf(q, a, -1.1511378288269043f);
    // 0.5 erfc = exp2(a P(a) - 1): the halving rides in the last fma, not in a multiply of |v|
    const float e = __builtin_amdgcn_exp2f(fmaf(q, a, -1.0f));
    return fmaf(-fabsf(v), fabsf(v) > 5.5f ? 0.0f : e, fmaxf(v, 0.0f));
}

// gelu_poly on a pair, its fma chain on packed f32 (v_pk_fma_f32: two lanes' values per
// instruction), the same operations per element: bit-identical to two gelu_poly calls.
__device__ __forceinline__ f32x2_t gelu_poly_pk(f32x2_t v) {
    const float a0 = fminf(fabsf(v.x), 5.5f), a1 = fminf(fabsf(v.y), 5.5f);
    const f32x2_t a = {a0, a1};
    f32x2_t q = {3.236920019844547e-05f, 3.236920019844547e-05f};
    q = __builtin_elementwise_fma(q, a, f32x2_t{-0.0007541869999840856f, -0.0007541869999840856f});
    q = __builtin_elementwise_fma(q, a, f32x2_t{0.008001405745744705f, 0.008001405745744705f});
    q = __builtin_elementwise_fma(q, a, f32x2_t{-0.05324144661426544f, -0.05324144661426544f});
    q = __builtin_elementwise_fma(q, a, f32x2_t{-0.45893436670303345f, -0.45893436670303345f});
    q = __builtin_elementwise_fma(q, a, f32x2_t{-1.1511378288269043f, -1.1511378288269043f});
    q = __builtin_elementwise_fma(q, a, f32x2_t{-1.0f, -1.0f});
    const f32x2_t e = {fabsf(v.x) > 5.5f ? 0.0f : __builtin_amdgcn_exp2f(q.x), fabsf(v.y) > 5.5f ? 0.0f : __builtin_amdgcn_exp2f(q.y)};
    const f32x2_t m = {fmaxf(v.x, 0.0f), fmaxf(v.y, 0.0f)};
    const f32x2_t na = {-fabsf(v.x), -fabsf(v.y)};
    return __builtin_elementwise_fma(na, e, m);
}

// f32 pair -> two bf16 (round to nearest even, NaN kept), one v_cvt_pk_bf16_f32
constexpr uint32_t MLP_MAX_HIDDEN = 1024;
#ifndef DK_MLP_SKEW
#define DK_MLP_SKEW 1
#endif
#ifndef DK_MLP_W2PAD
#define DK_MLP_W2PAD 4
#endif
#ifndef DK_MLP_P1
#define DK_MLP_P1 1
#endif
#ifndef DK_MLP_P2
#define DK_MLP_P2 1
#endif
// DK_MLP_PIN: the W fragment rings two deep and pinned by scheduling barriers at d <= 160
// (left to itself the compiler issued each read one MFMA before its use; -1.5 % at C5's MLP,
// profiles/r05/bf16_mlp_pin_ab/; d = 256 has no registers for it)
#ifndef DK_MLP_PIN
#define DK_MLP_PIN 1
#endif
#ifndef DK_MLP_WAVES160
#define DK_MLP_WAVES160 8
#endif
#ifndef DK_MLP_NC160
#define DK_MLP_NC160 64
#endif
#ifndef DK_MLP_WAVES256
#define DK_MLP_WAVES256 8
#endif
#ifndef DK_MLP_MINB
#define DK_MLP_MINB 2
#endif
// Epilogue stores 16 B per lane (DK_MLP_WIDE_STORE): lane (r, hh) holds columns
// 32 t + 8 q + 4 hh .. + 3 of row r, 8 B per (t, q).  For the q pair (2m, 2m + 1) one
// v_permlane32_swap per word trades the half-wave's pieces -- the lower lane gives its q = 2m + 1
// piece for the upper lane's q = 2m piece -- so the lower lane holds columns 16 m .. + 7 and the
// upper 16 m + 8 .. + 15: ten 16-B stores per row and tensor instead of twenty 8-B ones (the
// epilogue's store issue, not its bytes, is what it costs).
#ifndef DK_MLP_WIDE_STORE
#define DK_MLP_WIDE_STORE 1
#endif
template <int OT>
__device__ __forceinline__ void mlp_store_row16(const uint2 (&v)[OT][4], uint16_t* row, int hh, bool ok) {
#pragma unroll
    for (int t = 0; t < OT; ++t)
#pragma unroll
        for (int m = 0; m < 2; ++m) {
            const auto a = __builtin_amdgcn_permlane32_swap(v[t][2 * m].x, v[t][2 * m + 1].x, false, false);
            const auto b = __builtin_amdgcn_permlane32_swap(v[t][2 * m].y, v[t][2 * m + 1].y, false, false);
            // lower lanes: (own q = 2m piece, partner's q = 2m piece); upper: (partner's 2m + 1, own 2m + 1)
            if (ok) *(uint4*)(row + 32 * t + 16 * m + 8 * hh) = make_uint4(a[0], b[0], a[1], b[1]);
        }
}

template <int D, int NC, int WAVES = 8>
__global__ void __launch_bounds__(64 * WAVES, WAVES == 8 ? 1 : DK_MLP_MINB) mlp_ln_kernel(const uint16_t* __restrict__ h, uint16_t* __restrict__ x_io,
                                                        const uint16_t* __restrict__ w1, const uint16_t* __restrict__ b1,
                                                        const uint16_t* __restrict__ w2, const uint16_t* __restrict__ b2,
                                                        uint32_t rows, uint32_t n_hidden, const uint16_t* __restrict__ gamma,
                                                        const uint16_t* __restrict__ beta, float eps,
                                                        uint16_t* __restrict__ h_out) {
    static_assert(D % 32 == 0 && NC % 32 == 0, "d and the chunk: multiples of 32");
    // W2 rows padded by 4 elements: a 2-dword-odd row stride puts the 32 rows of a W2
    // fragment read (ds_read_b64) in 32 distinct bank pairs (+8 was 2-way conflicted)
    constexpr int KS = D / 16, OT = D / 32, LDW1 = D + 8, LDW2 = NC + DK_MLP_W2PAD, HT = NC / 32, GS = NC / 16;
    // LDS: the chunk's W1 / W2, in NB buffers: 3 when the waves 4..7 run half a chunk behind
    // (below), 2 otherwise
    constexpr int T = 64 * WAVES;                    // threads of the workgroup
    constexpr bool SKEW = DK_MLP_SKEW && D <= 160 && WAVES == 8;   // d = 256 has no registers to spare
    constexpr bool WIDE = DK_MLP_WIDE_STORE && D <= 160;           // (d = 256: spills)
    constexpr bool PIN = DK_MLP_PIN && D <= 160;
    constexpr int NB = SKEW ? 3 : 2;
    constexpr int W1E = NC * LDW1, W2E = D * LDW2;
    __shared__ __attribute__((aligned(16))) uint16_t lds[NB * (W1E + W2E)];
    __shared__ float b1s[MLP_MAX_HIDDEN];           // the hidden units' biases
    const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63, r = lane & 31, hh = lane >> 5;
    const uint32_t row = blockIdx.x * (32u * WAVES) + (uint32_t)wave * 32u + (uint32_t)r;
#ifdef DK_NET_PROF
    // phase sums in registers, one atomic per phase at the end (mid-kernel atomics would sit in
    // vmcnt in front of the very loads being timed)
    unsigned long long m_prev = __builtin_amdgcn_s_memtime(), macc[6] = {0, 0, 0, 0, 0, 0};
#define DK_MSTAMP(k) do { const unsigned long long t_ = __builtin_amdgcn_s_memtime(); macc[k] += t_ - m_prev; m_prev = t_; } while (0)
#else
#define DK_MSTAMP(k) ((void)0)
#endif
    const bool ok = row < rows;
    bf16x8_t hf[KS];
    {
        const uint16_t* hr = h + (size_t)(ok ? row : 0u) * D + 8 * hh;
#pragma unroll
        for (int kk = 0; kk < KS; ++kk) hf[kk] = load_frag8(hr + 16 * kk, ok);
    }
    // the chunk's weights: W1 rows c*NC .. +NC (D elements each) and columns c*NC .. +NC of every
    // W2 row, as 16-byte pieces; the next chunk's pieces are loaded into registers before this
    // chunk's GEMMs and written to the other LDS buffer after them (their latency hidden)
    // The pieces live in named registers (pa0..2, pb0..2), each piece index a literal: an array
    // indexed in a loop is an alloca that the compiler promoted to LDS here, which serialised
    // every global load behind its LDS store.
    constexpr int P1 = NC * (D / 8), P2 = D * (NC / 8);
    static_assert(P1 <= 5 * T && P2 <= 5 * T, "at most five pieces per thread and matrix");
    uint4 pa0{}, pa1{}, pa2{}, pa3{}, pa4{}, pb0{}, pb1{}, pb2{}, pb3{}, pb4{};
#define DK_MLP_LD(U, R1, R2, c)                                                                                \
    {                                                                                                          \
        const int v = threadIdx.x + T * (U);                                                                    \
        if (v < P1) { const int i = v / (D / 8), p = v - i * (D / 8); R1 = *(const uint4*)(w1 + ((size_t)(c) * NC + i) * D + 8 * p); } \
        if (v < P2) { const int o = v / (NC / 8), p = v - o * (NC / 8); R2 = *(const uint4*)(w2 + (size_t)o * n_hidden + (size_t)(c) * NC + 8 * p); } \
    }
#define DK_MLP_ST(U, R1, R2, buf)                                                                              \
    {                                                                                                          \
        const int v = threadIdx.x + T * (U);                                                                    \
        if (v < P1) { const int i = v / (D / 8), p = v - i * (D / 8); *(uint4*)&lds[(buf) * W1E + i * LDW1 + 8 * p] = R1; } \
        if (v < P2) { const int o = v / (NC / 8), p = v - o * (NC / 8); uint2* d_ = (uint2*)&lds[NB * W1E + (buf) * W2E + o * LDW2 + 8 * p]; \
                      d_[0] = make_uint2(R2.x, R2.y); d_[1] = make_uint2(R2.z, R2.w); } \
    }
#define DK_MLP_LOAD_CHUNK(c) { DK_MLP_LD(0, pa0, pb0, c) DK_MLP_LD(1, pa1, pb1, c) DK_MLP_LD(2, pa2, pb2, c)          \
    if constexpr (3 * T < P1 || 3 * T < P2) DK_MLP_LD(3, pa3, pb3, c)                                          \
    if constexpr (4 * T < P1 || 4 * T < P2) DK_MLP_LD(4, pa4, pb4, c) }
#define DK_MLP_STORE_CHUNK(buf) { DK_MLP_ST(0, pa0, pb0, buf) DK_MLP_ST(1, pa1, pb1, buf) DK_MLP_ST(2, pa2, pb2, buf) \
    if constexpr (3 * T < P1 || 3 * T < P2) DK_MLP_ST(3, pa3, pb3, buf)                                        \
    if constexpr (4 * T < P1 || 4 * T < P2) DK_MLP_ST(4, pa4, pb4, buf) }
    f32x16_t acc2[OT];
#pragma unroll
    for (int t = 0; t < OT; ++t) acc2[t] = f32x16_t{0};
    const uint32_t chunks = n_hidden / NC;
    for (uint32_t i = threadIdx.x; i < n_hidden; i += T) b1s[i] = bf2f(b1[i]);
    DK_MLP_LOAD_CHUNK(0u)
    DK_MLP_STORE_CHUNK(0)
    __syncthreads();
    // the residual rows' column groups of this lane (epilogue), loaded during the last chunk
    constexpr bool PREFETCH_X = D <= 160;
    uint2 xv[OT][4];
    // Per chunk: GEMM1 (MFMA), bias + GELU (VALU), GEMM2 (MFMA).  With one barrier per chunk
    // every wave runs the same phase at the same time, and the two waves of a SIMD (waves w
    // and w + 4) contend for the MFMA pipe and then for the VALU.  So (DK_MLP_SKEW) waves
    // 4..7 run half a chunk behind: in chunk interval c they finish chunk c - 1 (GELU + GEMM2)
    // and then run GEMM1 of chunk c, while waves 0..3 run GEMM1 then GELU + GEMM2 of chunk c:
    // one wave's GELU meets the other's MFMAs.  The lagging waves read chunk c - 1's W2 while
    // chunk c + 1 is staged, hence three LDS buffers.
    f32x16_t acc1[HT];
    auto gemm1 = [&](uint32_t c) {
        const int buf = (int)(c % NB);
#pragma unroll
        for (int j = 0; j < HT; ++j) acc1[j] = f32x16_t{0};
        // software-pipelined P1 k-steps deep: the W1 fragments of k-step kk + P1 are read from
        // LDS while the MFMAs of k-step kk run (an LDS read under load outlasts two MFMAs)
        constexpr int P1D = PIN ? 2 : DK_MLP_P1;
        bf16x8_t ring[P1D][HT];
#pragma unroll
        for (int kk = 0; kk < P1D && kk < KS; ++kk)
#pragma unroll
            for (int j = 0; j < HT; ++j)
                ring[kk][j] = *(const bf16x8_t*)&lds[(buf) * W1E + (32 * j + r) * LDW1 + 16 * kk + 8 * hh];
#pragma unroll
        for (int kk = 0; kk < KS; ++kk) {
            bf16x8_t cur[HT];
#pragma unroll
            for (int j = 0; j < HT; ++j) cur[j] = ring[kk % P1D][j];
            if (kk + P1D < KS) {
#pragma unroll
                for (int j = 0; j < HT; ++j)
                    ring[kk % P1D][j] = *(const bf16x8_t*)&lds[(buf) * W1E + (32 * j + r) * LDW1 + 16 * (kk + P1D) + 8 * hh];
            }
            if (PIN) __builtin_amdgcn_sched_barrier(0);   // (the ring's reads stay P1D k-steps ahead)
#pragma unroll
            for (int j = 0; j < HT; ++j) acc1[j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(cur[j], hf[kk], acc1[j], 0, 0, 0);
            if (PIN) __builtin_amdgcn_sched_barrier(0);
        }
    };
    auto prefetch_x = [&]() {
        if constexpr (PREFETCH_X) {
            // after the last GEMM1 the h fragments are dead: the residual x of the epilogue is
            // loaded now, in flight during the last GELU and GEMM2 (d = 160; d = 256 has no
            // registers to spare)
            const uint16_t* xr = x_io + (size_t)(ok ? row : 0u) * D;
#pragma unroll
            for (int t = 0; t < OT; ++t)
#pragma unroll
                for (int q = 0; q < 4; ++q) xv[t][q] = ok ? *(const uint2*)(xr + 32 * t + 8 * q + 4 * hh) : make_uint2(0u, 0u);
        }
    };
    auto gelu_gemm2 = [&](uint32_t c) {
        const int buf = (int)(c % NB);
        // bias + GELU -> bf16 B fragments of GEMM2 (k-step s = 2 j + half: registers 8 half .. +7)
        bf16x8_t af[GS];
#pragma unroll
        for (int s = 0; s < GS; ++s) {
            const int j = s >> 1, half = s & 1, h0 = 32 * j + 16 * half + 4 * hh;
            const float4 bl = *(const float4*)&b1s[c * NC + h0], bh = *(const float4*)&b1s[c * NC + h0 + 8];
            const float bb[8] = {bl.x, bl.y, bl.z, bl.w, bh.x, bh.y, bh.z, bh.w};
            union { uint32_t u[4]; bf16x8_t v; } pk;
#pragma unroll
            for (int t = 0; t < 8; t += 2) {
#if DK_GELU_POLY
                pk.u[t / 2] = pack_bf16x2(gelu_poly(acc1[j][8 * half + t] + bb[t]), gelu_poly(acc1[j][8 * half + t + 1] + bb[t + 1]));
#else
                const f32x2_t g = gelu_erf2_pk(f32x2_t{acc1[j][8 * half + t] + bb[t], acc1[j][8 * half + t + 1] + bb[t + 1]});
                pk.u[t / 2] = pack_bf16x2(g.x, g.y);
#endif
            }
            af[s] = pk.v;
        }
        // GEMM2, pipelined one output tile deep (the W2 fragment of the next tile read during this one)
        auto w2frag = [&](int s, int t) {
            const int h0 = 32 * (s >> 1) + 16 * (s & 1) + 4 * hh;
            const uint16_t* wr = &lds[NB * W1E + (buf) * W2E + (32 * t + r) * LDW2 + h0];
            union { uint2 u[2]; bf16x8_t v; } a;
            a.u[0] = *(const uint2*)wr;
            a.u[1] = *(const uint2*)(wr + 8);
            return a.v;
        };
        constexpr int P2D = PIN ? 2 : DK_MLP_P2;   // W2 fragments read P2D MFMAs ahead
        bf16x8_t ring2[P2D];
#pragma unroll
        for (int q = 0; q < P2D && q < GS * OT; ++q) ring2[q] = w2frag(q / OT, q % OT);
#pragma unroll
        for (int q = 0; q < GS * OT; ++q) {
            const int s = q / OT, t = q % OT;
            const bf16x8_t cur = ring2[q % P2D];
            if (q + P2D < GS * OT) ring2[q % P2D] = w2frag((q + P2D) / OT, (q + P2D) % OT);
            if (PIN) __builtin_amdgcn_sched_barrier(0);
            acc2[t] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(cur, af[s], acc2[t], 0, 0, 0);
            if (PIN) __builtin_amdgcn_sched_barrier(0);
        }
    };
    // one code path for all waves: iteration c = [GELU + GEMM2 of chunk c - 1][GEMM1 of chunk c];
    // waves 0..3 (SKEW) stage the next chunk and meet the barrier between the two halves,
    // waves 4..7 after them, so the groups run half an iteration apart
    const bool early = SKEW && wave < 4;   // wave-uniform
    auto sync = [&]() {
        // LDS-only barrier: the next chunk is staged and the reads of the buffer it overwrites are done
        asm volatile("" ::: "memory");
        __builtin_amdgcn_s_waitcnt(0xC07F);   // lgkmcnt(0)
        __builtin_amdgcn_s_barrier();
        asm volatile("" ::: "memory");
    };
    auto iteration = [&](uint32_t c, auto last) {
        constexpr bool L = decltype(last)::value;
        if constexpr (!L) DK_MLP_LOAD_CHUNK(c + 1)
        if constexpr (!SKEW) {   // d = 256: chunk c whole (acc1 dead between iterations)
            gemm1(c);
            if constexpr (L) prefetch_x();
            gelu_gemm2(c);
            if constexpr (!L) {
                DK_MLP_STORE_CHUNK((c + 1) % NB)
                sync();
            }
            return;
        }
        if (c > 0) gelu_gemm2(c - 1);
        DK_MSTAMP(1);
        if constexpr (!L) {
            if (early) {
                DK_MLP_STORE_CHUNK((c + 1) % NB)
                DK_MSTAMP(2);
                sync();
                DK_MSTAMP(3);
            }
        }
        gemm1(c);
        if constexpr (L) prefetch_x();
        DK_MSTAMP(4);
        if constexpr (!L) {
            if (!early) {
                DK_MLP_STORE_CHUNK((c + 1) % NB)
                DK_MSTAMP(2);
                sync();
                DK_MSTAMP(3);
            }
        }
    };
    DK_MSTAMP(0);
    for (uint32_t c = 0; c + 1 < chunks; ++c) iteration(c, std::false_type{});
    iteration(chunks - 1, std::true_type{});
    if constexpr (SKEW) gelu_gemm2(chunks - 1);

    // epilogue: acc2[t][g] = delta of row `row`, column 32 t + 8 (g >> 2) + 4 hh + (g & 3)
    uint16_t* xr = x_io + (size_t)(ok ? row : 0u) * D;
    if constexpr (!PREFETCH_X) {
#pragma unroll
        for (int t = 0; t < OT; ++t)
#pragma unroll
            for (int q = 0; q < 4; ++q) xv[t][q] = ok ? *(const uint2*)(xr + 32 * t + 8 * q + 4 * hh) : make_uint2(0u, 0u);
    }
    float s1 = 0.0f;
#pragma unroll
    for (int t = 0; t < OT; ++t)
#pragma unroll
        for (int q = 0; q < 4; ++q) {
            const int col = 32 * t + 8 * q + 4 * hh;
            const uint2 bv = *(const uint2*)(b2 + col);
            const uint16_t xs[4] = {(uint16_t)xv[t][q].x, (uint16_t)(xv[t][q].x >> 16), (uint16_t)xv[t][q].y,
                                    (uint16_t)(xv[t][q].y >> 16)};
            const uint16_t bs[4] = {(uint16_t)bv.x, (uint16_t)(bv.x >> 16), (uint16_t)bv.y, (uint16_t)(bv.y >> 16)};
            float xn[4];
#pragma unroll
            for (int e = 0; e < 4; e += 2) {
                // delta rounded to bf16 (the unfused proj GEMM's output), then x + delta rounded
                const uint32_t dl = pack_bf16x2(acc2[t][4 * q + e] + bf2f(bs[e]), acc2[t][4 * q + e + 1] + bf2f(bs[e + 1]));
                const uint32_t xo = pack_bf16x2(bf2f(xs[e]) + bf2f((uint16_t)dl), bf2f(xs[e + 1]) + bf2f((uint16_t)(dl >> 16)));
                xn[e] = bf2f((uint16_t)xo);
                xn[e + 1] = bf2f((uint16_t)(xo >> 16));
            }
#pragma unroll
            for (int e = 0; e < 4; ++e) {
                acc2[t][4 * q + e] = xn[e];
                s1 += xn[e];
            }
            if constexpr (WIDE) xv[t][q] = make_uint2(pack_bf16x2(xn[0], xn[1]), pack_bf16x2(xn[2], xn[3]));   // (x read above)
            else if (ok) *(uint2*)(xr + col) = make_uint2(pack_bf16x2(xn[0], xn[1]), pack_bf16x2(xn[2], xn[3]));
        }
    if constexpr (WIDE) mlp_store_row16<OT>(xv, xr, hh, ok);
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
    uint16_t* hr = h_out + (size_t)(ok ? row : 0u) * D;
#pragma unroll
    for (int t = 0; t < OT; ++t)
#pragma unroll
        for (int q = 0; q < 4; ++q) {
            const int col = 32 * t + 8 * q + 4 * hh;
            const uint2 gv = *(const uint2*)(gamma + col), bv = *(const uint2*)(beta + col);
            const uint16_t gs[4] = {(uint16_t)gv.x, (uint16_t)(gv.x >> 16), (uint16_t)gv.y, (uint16_t)(gv.y >> 16)};
            const uint16_t bs[4] = {(uint16_t)bv.x, (uint16_t)(bv.x >> 16), (uint16_t)bv.y, (uint16_t)(bv.y >> 16)};
            float o[4];
#pragma unroll
            for (int e = 0; e < 4; ++e) o[e] = (acc2[t][4 * q + e] - mean) * rstd * bf2f(gs[e]) + bf2f(bs[e]);
            if constexpr (WIDE) xv[t][q] = make_uint2(pack_bf16x2(o[0], o[1]), pack_bf16x2(o[2], o[3]));
            else if (ok) *(uint2*)(hr + col) = make_uint2(pack_bf16x2(o[0], o[1]), pack_bf16x2(o[2], o[3]));
        }
    if constexpr (WIDE) mlp_store_row16<OT>(xv, hr, hh, ok);
    DK_MSTAMP(5);
#ifdef DK_NET_PROF
    if (lane == 0 && (wave == 0 || wave == 4))
        for (int k = 0; k < 6; ++k) atomicAdd(&dk_mlp_prof_acc[(wave ? 8 : 0) + k], macc[k]);
#endif
}
#undef DK_MSTAMP
#undef DK_MLP_LD
#undef DK_MLP_ST
#undef DK_MLP_LOAD_CHUNK
#undef DK_MLP_STORE_CHUNK

}  // namespace net
}  // namespace dk
