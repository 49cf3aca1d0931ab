// ORACLE — test infrastructure only. Never linked into the product library.
//
// CPU restatement of the parts of `rand 0.9.0` / `rand_core 0.9.3` that the
// reference hot path calls (Cargo.lock:1899-1946 pins these; the crates are not
// vendored under /root/reference, so this restates their published algorithms):
//
//   SmallRng (64-bit)            = Xoshiro256++
//   SeedableRng::seed_from_u64   = SplitMix64 expansion of the u64 seed
//   RngCore::next_u32            = upper 32 bits of next_u64
//   Rng::random_range (u32)      = Canon's widening multiply, one optional extra draw
//   Rng::random_range (usize)    = u32 path when the range fits in u32
//   SliceRandom::shuffle         = IncreasingUniform chunked forward Fisher-Yates
//   Rng::random_bool             = Bernoulli: one next_u64 compared to p * 2^64
//   IteratorRandom::choose       = exact-size path (one range draw) and the
//                                  CoinFlipper path (size_hint (0, None))
//
// Pinned by the golden deal of rs-full-doko/src/hand/hand.rs:558-585 (seed 42).
// `random_bool` and the CoinFlipper path are NOT pinned by any reference fixture.
#pragma once
#include <cstdint>
#include <cstddef>
#include <utility>

namespace oracle {

struct SmallRng {
    uint64_t s[4];

    static inline uint64_t rotl(uint64_t x, int k) { return (x << k) | (x >> (64 - k)); }

    // rand 0.9 Xoshiro256PlusPlus::seed_from_u64 (SplitMix64 with PHI increment).
    static SmallRng seed_from_u64(uint64_t state) {
        SmallRng r;
        const uint64_t PHI = 0x9e3779b97f4a7c15ULL;
        for (int i = 0; i < 4; ++i) {
            state += PHI;
            uint64_t z = state;
            z = (z ^ (z >> 30)) * 0xbf58476d1ce4e5b9ULL;
            z = (z ^ (z >> 27)) * 0x94d049bb133111ebULL;
            z = z ^ (z >> 31);
            r.s[i] = z;
        }
        if ((r.s[0] | r.s[1] | r.s[2] | r.s[3]) == 0) return seed_from_u64(0);
        return r;
    }

    uint64_t next_u64() {
        const uint64_t res = rotl(s[0] + s[3], 23) + s[0];
        const uint64_t t = s[1] << 17;
        s[2] ^= s[0];
        s[3] ^= s[1];
        s[1] ^= s[2];
        s[0] ^= s[3];
        s[2] ^= t;
        s[3] = rotl(s[3], 45);
        return res;
    }

    uint32_t next_u32() { return (uint32_t)(next_u64() >> 32); }

    // UniformInt<u32>::sample_single_inclusive(low, high) — Canon's method
    // without the `unbiased` feature: one widening multiply, and a second
    // draw only when the low word lands in the biased zone.
    uint32_t sample_u32_inclusive(uint32_t low, uint32_t high) {
        const uint32_t range = high - low + 1u;
        if (range == 0) return next_u32();
        const uint64_t m = (uint64_t)next_u32() * (uint64_t)range;
        uint32_t result = (uint32_t)(m >> 32);
        const uint32_t lo_order = (uint32_t)m;
        if (lo_order > (uint32_t)(0u - range)) {
            const uint64_t m2 = (uint64_t)next_u32() * (uint64_t)range;
            const uint32_t new_hi = (uint32_t)(m2 >> 32);
            const bool overflow = (uint32_t)(lo_order + new_hi) < lo_order;
            result += overflow ? 1u : 0u;
        }
        return low + result;
    }

    // random_range(low..high) on u32.
    uint32_t random_range_u32(uint32_t low, uint32_t high) { return sample_u32_inclusive(low, high - 1u); }

    // random_range(low..high) on usize: UniformUsize takes the u32 path when
    // the inclusive high fits in u32 (always true on this hot path).
    size_t random_range_usize(size_t low, size_t high) {
        return (size_t)sample_u32_inclusive((uint32_t)low, (uint32_t)(high - 1));
    }

    // Rng::random_bool(p) -> Bernoulli::new(p).sample(): one u64 draw.
    bool random_bool(double p) {
        const double SCALE = 2.0 * (double)(1ULL << 63);
        if (p >= 1.0) return true;  // ALWAYS_TRUE short-cut
        const uint64_t p_int = (uint64_t)(p * SCALE);
        return next_u64() < p_int;
    }
};

// IncreasingUniform (rand 0.9 seq/increasing_uniform.rs) used by shuffle.
struct IncreasingUniform {
    SmallRng* rng;
    uint32_t n;
    uint32_t chunk;
    uint8_t chunk_remaining;

    IncreasingUniform(SmallRng* r, uint32_t n0) : rng(r), n(n0), chunk(0), chunk_remaining(n0 == 0 ? 1 : 0) {}

    static void calculate_bound_u32(uint32_t m, uint32_t* bound, uint8_t* count) {
        uint32_t product = m;
        uint32_t current = m + 1;
        for (;;) {
            uint64_t p = (uint64_t)product * (uint64_t)current;
            if (p > 0xFFFFFFFFULL) break;
            product = (uint32_t)p;
            current += 1;
        }
        *bound = product;
        *count = (uint8_t)(current - m);
    }

    size_t next_index() {
        const uint32_t next_n = n + 1;
        uint8_t next_chunk_remaining;
        if (chunk_remaining == 0) {
            uint32_t bound; uint8_t remaining;
            calculate_bound_u32(next_n, &bound, &remaining);
            chunk = rng->random_range_u32(0, bound);
            next_chunk_remaining = (uint8_t)(remaining - 1);
        } else {
            next_chunk_remaining = (uint8_t)(chunk_remaining - 1);
        }
        size_t result;
        if (next_chunk_remaining == 0) {
            result = chunk;
        } else {
            result = chunk % next_n;
            chunk /= next_n;
        }
        chunk_remaining = next_chunk_remaining;
        n = next_n;
        return result;
    }
};

// SliceRandom::shuffle -> partial_shuffle(len) with IncreasingUniform.
template <typename T>
void shuffle(T* data, size_t len, SmallRng& rng) {
    if (len <= 1) return;
    IncreasingUniform chooser(&rng, 0);
    for (size_t i = 0; i < len; ++i) {
        size_t index = chooser.next_index();
        std::swap(data[i], data[index]);
    }
}

// CoinFlipper (rand 0.9 seq/coin_flipper.rs), used by IteratorRandom::choose
// for iterators without an exact size hint.  PARITY UNPINNED (no fixture).
struct CoinFlipper {
    SmallRng* rng;
    uint32_t chunk;
    uint32_t chunk_remaining;

    explicit CoinFlipper(SmallRng* r) : rng(r), chunk(0), chunk_remaining(0) {}

    static uint32_t clz32(uint32_t x) { return x == 0 ? 32u : (uint32_t)__builtin_clz(x); }
    static uint32_t clz64(uint64_t x) { return x == 0 ? 64u : (uint32_t)__builtin_clzll(x); }

    bool flip_c_heads(uint32_t c) {
        for (;;) {
            const uint32_t zeros = clz32(chunk);
            if (zeros < c) {
                const uint32_t sh = zeros + 1;
                chunk = chunk << (sh & 31);  // u32::wrapping_shl masks the shift amount
                chunk_remaining = chunk_remaining > sh ? chunk_remaining - sh : 0;  // saturating_sub
                return false;
            } else {
                if (chunk_remaining >= c) {  // checked_sub succeeded
                    chunk_remaining -= c;
                    chunk = chunk << (c & 31);
                    return true;
                }
                c -= chunk_remaining;
                chunk = rng->next_u32();
                chunk_remaining = 32;
            }
        }
    }

    bool random_ratio(uint64_t n, uint64_t d) {
        while (n < d) {
            int64_t cc = (int64_t)clz64(n) - (int64_t)(clz64(d) + 1);
            if (cc < 0) cc = 0;  // saturating_sub
            uint32_t c = (uint32_t)(cc < 1 ? 1 : (cc > 32 ? 32 : cc));
            if (flip_c_heads(c)) {
                const unsigned __int128 prod = (unsigned __int128)n << c;
                n = prod > (unsigned __int128)UINT64_MAX ? UINT64_MAX : (uint64_t)prod;
            } else {
                if (c == 1) {
                    const uint64_t next_n = n + n - d;  // wrapping
                    if (next_n == 0 || next_n > n) return false;
                    n = next_n;
                } else {
                    return false;
                }
            }
        }
        return true;
    }

    bool random_ratio_one_over(uint64_t d) {
        uint32_t c = 64u - 1u - clz64(d);
        if (c > 32) c = 32;
        if (flip_c_heads(c)) {
            const uint64_t numerator = 1ULL << c;
            return random_ratio(numerator, d);
        }
        return false;
    }
};

// IteratorRandom::choose over an iterator with size_hint (0, None):
// reservoir sampling driven by a fresh CoinFlipper. `items` are visited in
// iteration order; returns the chosen index or -1 when empty.
inline int choose_unsized(size_t count, SmallRng& rng) {
    CoinFlipper cf(&rng);
    int result = -1;
    uint64_t consumed = 0;
    for (size_t i = 0; i < count; ++i) {
        consumed += 1;
        if (cf.random_ratio_one_over(consumed)) result = (int)i;
    }
    return result;
}

// IteratorRandom::choose over an ExactSizeIterator (e.g. EnumSet iter):
// 0 -> None, 1 -> first, else nth(random_range(..len)).
inline int choose_sized(size_t count, SmallRng& rng) {
    if (count == 0) return -1;
    if (count == 1) return 0;
    return (int)rng.random_range_usize(0, count);
}

}  // namespace oracle
