// TEST INFRASTRUCTURE: rng.h's run-length choose_unsized against the item-by-item
// choose_unsized_ref (IteratorRandom::choose's CoinFlipper path): the chosen index and the
// generator state after the call, on random generator states and item counts.
// Usage: coin_check <cases> <seed>
#include <cstdio>
#include <cstdlib>
#include <random>

#include "../../master_doko_reinforcement_learning_amd/csrc/engine/rng.h"

int main(int argc, char** argv) {
    const long cases = argc > 1 ? atol(argv[1]) : 1000000;
    const uint64_t seed = argc > 2 ? strtoull(argv[2], 0, 10) : 1;
    std::mt19937_64 g(seed);
    long n = 0;
    for (long k = 0; k < cases; ++k) {
        const int count = (k % 16 == 0) ? 1 + (int)(g() % 300) : 1 + (int)(g() % 48);
        dk::Rng a = dk::Rng::seed_from_u64(g()), b = a;
        const int ra = dk::choose_unsized_ref(count, a), rb = dk::choose_unsized(count, b);
        if (ra != rb || a.s0 != b.s0 || a.s1 != b.s1 || a.s2 != b.s2 || a.s3 != b.s3) {
            printf("MISMATCH case %ld count %d: ref %d fast %d\n", k, count, ra, rb);
            return 1;
        }
        n += count;
    }
    printf("OK %ld\n", n);
    return 0;
}
