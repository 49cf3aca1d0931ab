// Shared primitives of the gfx950 engine.  Everything is DK_HD (host+device)
// so the exact same code can also be compiled by g++ into the CPU-side test
// harness (tests/native) — that build is test infrastructure only; the
// product library runs this code on the GPU exclusively.
#pragma once
#include <stdint.h>

#if defined(__HIPCC__)
#include <hip/hip_runtime.h>
#define DK_HD __host__ __device__ __forceinline__
#define DK_DEV __device__ __forceinline__
#else
#define DK_HD inline
#define DK_DEV inline
#endif

namespace dk {

DK_HD int popc64(uint64_t x) { return __builtin_popcountll(x); }
DK_HD int popc32(uint32_t x) { return __builtin_popcount(x); }
DK_HD int ctz32(uint32_t x) { return x ? __builtin_ctz(x) : 32; }
DK_HD int ctz64(uint64_t x) { return __builtin_ctzll(x); }
DK_HD int clz32(uint32_t x) { return x == 0 ? 32 : __builtin_clz(x); }
DK_HD int clz64(uint64_t x) { return x == 0 ? 64 : __builtin_clzll(x); }

// true if any active lane of the wave has p (host builds: p itself)
DK_HD bool wave_any(bool p) {
#if defined(__HIP_DEVICE_COMPILE__)
    return __builtin_amdgcn_ballot_w64(p) != 0;
#else
    return p;
#endif
}

// Bit of rank r counted from the MSB (rs-game-utils/src/bit_flag.rs:104-171):
// equivalently the (popc-1-r)-th set bit counted from the LSB.  Branch-free
// binary search over popcounts (6 steps for 64-bit masks).
DK_HD uint64_t select_msb_rank(uint64_t v, uint32_t r) {
    uint32_t k = (uint32_t)popc64(v) - 1u - r;  // rank from the LSB
    uint32_t pos = 0;
#pragma unroll
    for (int w = 32; w >= 1; w >>= 1) {
        const uint64_t lowmask = (w == 64) ? ~0ULL : ((1ULL << w) - 1ULL);
        const uint32_t c = (uint32_t)popc64((v >> pos) & lowmask);
        const bool go_high = k >= c;
        k = go_high ? k - c : k;
        pos = go_high ? pos + (uint32_t)w : pos;
    }
    return 1ULL << pos;
}

// Per-byte lanes of a u32 (4 players, each <= 255).
DK_HD uint32_t byte_get(uint32_t w, int i) { return (w >> (8 * i)) & 0xFFu; }
DK_HD uint32_t byte_add(uint32_t w, int i, uint32_t v) { return w + (v << (8 * i)); }
DK_HD uint32_t byte_set(uint32_t w, int i, uint32_t v) { return (w & ~(0xFFu << (8 * i))) | ((v & 0xFFu) << (8 * i)); }

// 4-element selects without dynamic register indexing (keeps arrays in VGPRs).
// Written as mask arithmetic: a select chain on the index is recognised by the
// optimiser as h[p] and turned back into a (scratch-memory) array access.
DK_HD uint64_t sel4(const uint64_t h[4], int p) {
    const uint64_t m0 = 0ULL - (uint64_t)(p == 0), m1 = 0ULL - (uint64_t)(p == 1);
    const uint64_t m2 = 0ULL - (uint64_t)(p == 2), m3 = 0ULL - (uint64_t)(p == 3);
    return (h[0] & m0) | (h[1] & m1) | (h[2] & m2) | (h[3] & m3);
}
DK_HD void set4(uint64_t h[4], int p, uint64_t v) {
    h[0] = p == 0 ? v : h[0];
    h[1] = p == 1 ? v : h[1];
    h[2] = p == 2 ? v : h[2];
    h[3] = p == 3 ? v : h[3];
}

}  // namespace dk
