// SmallRng of rand 0.9.0 (= Xoshiro256++) for the GPU, keeping the draw order
// of the reference: seed_from_u64 (SplitMix64), next_u32 = hi32(next_u64),
// u32 random_range = Canon widening multiply (+1 draw in the biased zone),
// shuffle = IncreasingUniform, IteratorRandom::choose = CoinFlipper path.
// (Cargo.lock:1899-1946 pins rand 0.9.0 / rand_core 0.9.3.)
#pragma once
#include "common.h"

namespace dk {

struct Rng {
    uint64_t s0, s1, s2, s3;

    // rotate left by a compile-time amount (Xoshiro256++ uses 23 and 45).  The device form
    // is two funnel shifts (v_alignbit_b32), whose shift operand is taken mod 32: a rotation
    // by a multiple of 32 would come out wrong, so those amounts are rejected at compile time.
    template <int K>
    DK_HD static uint64_t rotl(uint64_t x) {
        static_assert(K > 0 && K < 64 && K % 32 != 0, "rotl: 0 < K < 64, K != 32");
#if defined(__HIP_DEVICE_COMPILE__)
        constexpr int k = K >= 32 ? K - 32 : K;
        uint32_t lo = (uint32_t)x, hi = (uint32_t)(x >> 32);
        if constexpr (K >= 32) { const uint32_t t = lo; lo = hi; hi = t; }
        const uint32_t nh = __builtin_amdgcn_alignbit(hi, lo, 32 - k), nl = __builtin_amdgcn_alignbit(lo, hi, 32 - k);
        return (uint64_t)nh << 32 | nl;
#else
        return (x << K) | (x >> (64 - K));
#endif
    }

    DK_HD static Rng seed_from_u64(uint64_t state) {
        // rand_core 0.9 SeedableRng::seed_from_u64 (SplitMix64); Xoshiro256++ maps an
        // all-zero seed to seed_from_u64(0), whose output is non-zero (no recursion needed)
        Rng r;
        uint64_t out[4];
        for (int pass = 0; pass < 2; ++pass) {
#pragma unroll
            for (int i = 0; i < 4; ++i) {
                state += 0x9e3779b97f4a7c15ULL;
                uint64_t z = state;
                z = (z ^ (z >> 30)) * 0xbf58476d1ce4e5b9ULL;
                z = (z ^ (z >> 27)) * 0x94d049bb133111ebULL;
                out[i] = z ^ (z >> 31);
            }
            if ((out[0] | out[1] | out[2] | out[3]) != 0) break;
            state = 0;
        }
        r.s0 = out[0]; r.s1 = out[1]; r.s2 = out[2]; r.s3 = out[3];
        return r;
    }

    DK_HD uint64_t next_u64() {
        const uint64_t res = rotl<23>(s0 + s3) + s0;
        advance();
        return res;
    }
    DK_HD uint32_t next_u32() { return (uint32_t)(next_u64() >> 32); }
    // a ^ b ^ c (gfx950: one v_bitop3_b32 per half, truth table 0x96; the compiler splits a
    // written three-way XOR into two-input XORs)
    DK_HD static uint64_t xor3(uint64_t a, uint64_t b, uint64_t c) {
#if defined(__HIP_DEVICE_COMPILE__)
        const uint32_t lo = __builtin_amdgcn_bitop3_b32((uint32_t)a, (uint32_t)b, (uint32_t)c, 0x96);
        const uint32_t hi = __builtin_amdgcn_bitop3_b32((uint32_t)(a >> 32), (uint32_t)(b >> 32), (uint32_t)(c >> 32), 0x96);
        return (uint64_t)hi << 32 | lo;
#else
        return a ^ b ^ c;
#endif
    }
    // state transition only (a draw whose value is discarded).  The reference's sequence
    // s2 ^= s0; s3 ^= s1; s1 ^= s2; s0 ^= s3; s2 ^= t; s3 = rotl(s3, 45) written as
    // three-input XORs of the old words
    DK_HD void advance() {
        const uint64_t t = s1 << 17;
        const uint64_t n0 = xor3(s0, s3, s1), n1 = xor3(s1, s2, s0), n2 = xor3(s2, s0, t), n3 = s3 ^ s1;
        s0 = n0; s1 = n1; s2 = n2;
        s3 = rotl<45>(n3);
    }

    // random_range(0..n) on u32 (n >= 1).
    DK_HD uint32_t range_u32(uint32_t n) {
        const uint64_t m = (uint64_t)next_u32() * (uint64_t)n;
        uint32_t result = (uint32_t)(m >> 32);
        const uint32_t lo = (uint32_t)m;
        if (lo > (uint32_t)(0u - n)) {
            const uint32_t hi2 = (uint32_t)(((uint64_t)next_u32() * (uint64_t)n) >> 32);
            result += ((uint32_t)(lo + hi2) < lo) ? 1u : 0u;
        }
        return result;
    }

    // random_bool(p) (Bernoulli, one u64 draw; p < 1).
    DK_HD bool random_bool(double p) {
        const uint64_t p_int = (uint64_t)(p * 18446744073709551616.0);
        return next_u64() < p_int;
    }
};

// uniform pick of one set bit (Bitflag::random_single, bit_flag.rs:86-92)
DK_HD uint64_t random_single(uint64_t mask, Rng& rng) {
    const uint32_t r = rng.range_u32((uint32_t)popc64(mask));
    return select_msb_rank(mask, r);
}

// SliceRandom::shuffle on a 48-entry array via IncreasingUniform.
DK_HD void shuffle48(uint8_t* a, Rng& rng) {
    uint32_t n = 0, chunk = 0;
    uint32_t chunk_remaining = 1;  // IncreasingUniform::new(rng, 0)
    for (int i = 0; i < 48; ++i) {
        const uint32_t next_n = n + 1;
        uint32_t ncr;
        if (chunk_remaining == 0) {
            uint32_t product = next_n, current = next_n + 1;
            while ((uint64_t)product * current <= 0xFFFFFFFFULL) { product *= current; current += 1; }
            chunk = rng.range_u32(product);
            ncr = current - next_n - 1;
        } else {
            ncr = chunk_remaining - 1;
        }
        uint32_t idx;
        if (ncr == 0) idx = chunk;
        else { idx = chunk % next_n; chunk /= next_n; }
        chunk_remaining = ncr;
        n = next_n;
        const uint8_t t = a[i]; a[i] = a[idx]; a[idx] = t;
    }
}

// CoinFlipper of rand 0.9 seq/coin_flipper.rs (IteratorRandom::choose without a
// size hint).  Parity with the reference is unpinned (no fixture exercises it).
struct CoinFlipper {
    uint32_t chunk = 0, remaining = 0;

    // coin_flipper.rs flip_c_heads: the refill (too few bits left and no tail among them) is the
    // only loop; the outcome is then computed by selects, so a wave whose lanes take different
    // outcomes does not run both branches (the CAP sampler calls this once per remaining card)
    DK_HD bool flip_c_heads(uint32_t c, Rng& rng) {
        uint32_t zeros = (uint32_t)clz32(chunk);
        while (zeros >= c && remaining < c) {
            c -= remaining;
            chunk = rng.next_u32();
            remaining = 32;
            zeros = (uint32_t)clz32(chunk);
        }
        const bool tails = zeros < c;
        const uint32_t sh = tails ? zeros + 1 : c;
        chunk = chunk << (sh & 31);
        remaining = tails ? (remaining > sh ? remaining - sh : 0) : remaining - c;
        return !tails;
    }
    DK_HD bool random_ratio(uint64_t n, uint64_t d, Rng& rng) {
        while (n < d) {
            int cc = clz64(n) - (clz64(d) + 1);
            if (cc < 1) cc = 1;
            if (cc > 32) cc = 32;
            const uint32_t c = (uint32_t)cc;
            if (flip_c_heads(c, rng)) {
                n = (c >= 64 || (n >> (64 - c)) != 0) ? ~0ULL : (n << c);
            } else {
                if (c == 1) {
                    const uint64_t next_n = n + n - d;
                    if (next_n == 0 || next_n > n) return false;
                    n = next_n;
                } else {
                    return false;
                }
            }
        }
        return true;
    }
    DK_HD bool random_ratio_one_over(uint64_t d, Rng& rng) {
        uint32_t c = 63u - (uint32_t)clz64(d);
        if (c > 32) c = 32;
        if (flip_c_heads(c, rng)) return random_ratio(1ULL << c, d, rng);
        return false;
    }
};

// Reservoir choice over `count` items in iteration order (CoinFlipper path), item by item: the
// reference's loop (the host check compares choose_unsized with it).
DK_HD int choose_unsized_ref(int count, Rng& rng) {
    CoinFlipper cf;
    int result = -1;
    for (int i = 0; i < count; ++i)
        if (cf.random_ratio_one_over((uint64_t)(i + 1), rng)) result = i;
    return result;
}

// The same choice with runs of "tails" consumed per chunk.  Item i (d = i + 1, c = floor(log2 d))
// is a tail -- not chosen, no draw -- when the chunk's next 1 bit comes after fewer than c zeros;
// it consumes those zeros and the 1.  So from the chunk alone: the item starts are offset 0 and the
// offset after every 1 bit; the first start followed by c zeros (R & S) ends the run of tails, and
// the 1 bits before it are the tails.  Items that are not plain tails inside the chunk (heads, a
// refill) take the item-by-item step above.  Results and generator state equal choose_unsized_ref
// (tests/native/coin_check.cpp).
DK_HD int choose_unsized(int count, Rng& rng) {
    if (count <= 0) return -1;
    CoinFlipper cf;
    int result = 0;   // item 0 (d = 1, c = 0): always chosen, no bits consumed
    int i = 1;
    while (i < count) {
        const uint32_t d = (uint32_t)i + 1u;
        const uint32_t c = 31u - (uint32_t)clz32(d);                 // 1 <= c <= 31 here
        const int end = count < (int)((2u << c) - 1u) ? count : (int)((2u << c) - 1u);   // items sharing c
        const uint32_t x = cf.chunk;
        int take = 0;
        if (x != 0u) {
            uint32_t w = x, span = 1;                                  // OR over windows of c bits
            while (span * 2u <= c) { w |= w << span; span *= 2u; }
            if (span < c) w |= w << (c - span);
            const uint32_t starts = (x >> 1) | 0x80000000u;
            const uint32_t f = ~w & starts;
            const int tails = f ? (clz32(f) == 0 ? 0 : popc32(x >> (32 - clz32(f)))) : popc32(x);
            take = tails < end - i ? tails : end - i;
        }
        if (take > 0) {
            // consume through the take-th 1 bit from the top
            const uint32_t pos = (uint32_t)ctz64(select_msb_rank((uint64_t)x, (uint32_t)(take - 1)));
            const uint32_t sh = 32u - pos;
            cf.chunk = sh >= 32u ? 0u : x << sh;
            cf.remaining -= sh;
            i += take;
        } else {
            if (cf.random_ratio_one_over((uint64_t)d, rng)) result = i;
            ++i;
        }
    }
    return result;
}

}  // namespace dk
