// ORACLE / TEST INFRASTRUCTURE — never linked into the product library.
//
// Synthetic "network" for the AlphaZero search parity tests: a pure function of
// the 117 semantic bytes of the packed state (dk_fdo_state), so the oracle, the
// host build of az_core.h and the GPU test (numpy, tests/test_gpu_parity.py)
// all see identical value / logit vectors.  Values are multiples of 1/8 in
// [-1, 0.875], logits multiples of 1/4 in [-4, 3.75].
#pragma once
#include <cstdint>

namespace oracle {
namespace az {

inline uint64_t splitmix64(uint64_t x) {
    uint64_t z = x + 0x9E3779B97F4A7C15ULL;
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ULL;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBULL;
    return z ^ (z >> 31);
}

inline void hash_eval(const uint8_t* packed, float value[4], float logits[39]) {
    uint64_t h = 0xCBF29CE484222325ULL;   // FNV-1a 64
    for (int i = 0; i < 117; ++i) { h ^= packed[i]; h *= 0x100000001B3ULL; }
    for (int k = 0; k < 4; ++k) value[k] = (float)((int)((h >> (8 * k)) & 15u) - 8) * 0.125f;
    for (int a = 0; a < 39; ++a) logits[a] = (float)((int)(splitmix64(h + (uint64_t)a) & 31u) - 16) * 0.25f;
}

}  // namespace az
}  // namespace oracle
